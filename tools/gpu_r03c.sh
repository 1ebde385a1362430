set -o pipefail
bash tools/gpu_check.sh r03c || exit 1
mkdir -p gpurun_out/r03c
timeout -k 10 300 python -u tools/diag_cycles.py gpurun_out/r03c/diag --solves 2 --rounds 3 > gpurun_out/r03c/diag.txt 2>&1 || { echo "diag failed"; tail -20 gpurun_out/r03c/diag.txt; exit 1; }
cat gpurun_out/r03c/diag.txt
for v in nopf hop3; do
  KS_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch_incremental.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03c/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 gpurun_out/r03c/pytest_$v.log; exit 1; }
  tail -1 gpurun_out/r03c/pytest_$v.log
done
bash tools/ab.sh r03c/ab 3 base default nopf hop3
