#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_msssp.py -v --timeout 120 --timeout-method thread > $O/r03k_msssp.log 2>&1 &&
SRT_MSSSP_PROF=1 timeout -k 10 120 python -u tools/msssp_probe.py c3 > $O/r03k_probe.log 2>&1 &&
timeout -k 10 120 python -u tools/msssp_probe.py c3 >> $O/r03k_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 SRT_MSSSP_DELTA=32 timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 1 >> $O/r03k_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 SRT_MSSSP_DELTA=64 timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 1 >> $O/r03k_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 SRT_MSSSP_DELTA=8 timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 1 >> $O/r03k_probe.log 2>&1  &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "c2 or tiers or round_sizes or c1" -x -v --timeout 300 --timeout-method thread > $O/r03k_parity.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/r03k_bench_c2.json 2> $O/r03k_bench_c2.err &&
SRT_FW_SQUARE_SPLIT=0 timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/r03k_bench_c2_nosplit.json 2>> $O/r03k_bench_c2.err
