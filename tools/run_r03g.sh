#!/bin/bash
# round 3: small-matrix min-plus squaring (C2) -- parity, bench, kernel trace
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "c2 or tiers or round_sizes or lookahead or tie or c1 or rgg or barabasi or directed" -x -v --timeout 300 --timeout-method thread > $O/r03g_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/r03g_bench_c2.json 2> $O/r03g_bench_c2.err &&
SRT_FW_SQUARE=0 timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/r03g_bench_c2_rounds.json 2>> $O/r03g_bench_c2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r03g_prof_c2 -o c2 -- python3 -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/r03g_prof_c2.log 2>&1
