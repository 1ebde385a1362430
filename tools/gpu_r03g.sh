set -o pipefail
bash tools/gpu_check.sh r03g all || exit 1
timeout -k 10 300 python -u tools/diag_cycles.py gpurun_out/r03g/diag --solves 2 --rounds 3 > gpurun_out/r03g/diag.txt 2>&1 || { echo "diag failed"; tail -20 gpurun_out/r03g/diag.txt; exit 1; }
cat gpurun_out/r03g/diag.txt
bash tools/ab.sh r03g/ab 3 base default
