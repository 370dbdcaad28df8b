set -o pipefail
mkdir -p gpurun_out/r04exp
for v in I J K; do
  env SRT_LIB_PATH=$PWD/tools/exp/lib$v.so timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 1 --no-cpu-baseline > gpurun_out/r04exp/bench_$v.json 2> gpurun_out/r04exp/bench_$v.err || exit $?
  echo "$v done"
done
