# r04o: C5 derivation pipelined beside the core chunks (second stream) vs not
set -e
O=gpurun_out/r04o
mkdir -p $O
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_derive.py -m gpu > $O/tests.log 2>&1
echo tests-ok
for v in "dv_pipe=1" "dv_pipe=1,dv_wg=1" "dv_pipe=0"; do
  SRT_FORM=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5_${v//[,=]/_} -o run -- python3 bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/c5_${v//[,=]/_}.log 2>&1
  echo "c5 $v ok"
done
