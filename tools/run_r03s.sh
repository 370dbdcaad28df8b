#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/r03s_bench_c2.json 2> $O/r03s_bench_c2.err &&
SRT_FW_SQUARE_SPLIT=0 timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/r03s_bench_c2_nosplit.json 2>> $O/r03s_bench_c2.err &&
SRT_FW_SQUARE=0 timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/r03s_bench_c2_rounds.json 2>> $O/r03s_bench_c2.err &&
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/r03s_trace_c2 -o run -- python3 bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline > $O/r03s_trace_c2.log 2>&1
