# r04u: derive parent cache A/B
set -e
O=gpurun_out/r04u
mkdir -p $O
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
for v in 0 1 2; do
  SRT_FORM=dv_var=$v timeout -k 10 300 $PYT tests/test_gpu_derive.py -m gpu > $O/tests_$v.log 2>&1
  echo "tests $v ok"
done
for v in 0 1 2; do
  SRT_FORM=dv_var=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5_$v -o run -- python3 bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/c5_$v.log 2>&1
  echo "c5 $v ok"
done
