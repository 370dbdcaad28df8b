# r04n: level kernels with scalar-burst arc offsets; derive chain with 4-target steps
set -e
O=gpurun_out/r04n
mkdir -p $O
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_levels.py tests/test_gpu_derive.py -m gpu > $O/tests.log 2>&1
echo tests-ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_c4.log 2>&1
echo c4-ok
for v in "dv_wg=4" "dv_wg=8"; do
  SRT_FORM=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5_${v//[,=]/_} -o run -- python3 bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/c5_${v//[,=]/_}.log 2>&1
  echo "c5 $v ok"
done
