#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/r03t_bench_c2.json 2> $O/r03t_bench_c2.err &&
SRT_FW_SQUARE_SPLIT=0 timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/r03t_bench_c2_nosplit.json 2>> $O/r03t_bench_c2.err &&
timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline > $O/r03t_bench_c3.json 2> $O/r03t_bench_c3.err &&
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/r03t_bench_c4.json 2> $O/r03t_bench_c4.err
