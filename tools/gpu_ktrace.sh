set -o pipefail
export TMPDIR=/tmp
for v in default prev; do
  if [ $v = prev ]; then export KS_LIB_VARIANT=prev; else unset KS_LIB_VARIANT; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d gpurun_out/kt_$v -o run -- python -u bench.py --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/kt_$v.json 2> gpurun_out/kt_$v.err || exit 1
  echo "== $v"; python tools/kernel_trace.py gpurun_out/kt_$v > gpurun_out/kt_$v.txt
done
