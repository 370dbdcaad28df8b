#!/bin/bash
# round 3 state: the full GPU suite, then the bench lines of every config and a kernel trace of C3
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/r03q_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/r03q_bench_c4.json 2> $O/r03q_bench_c4.err &&
timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 > $O/r03q_bench_c2.json 2> $O/r03q_bench_c2.err &&
timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 3 > $O/r03q_bench_c3.json 2> $O/r03q_bench_c3.err &&
timeout -k 10 400 python -u bench.py --workload c5 --steps 3 --warmup 1 > $O/r03q_bench_c5.json 2> $O/r03q_bench_c5.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03q_prof_c3 -o run -- python3 bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/r03q_prof_c3.log 2>&1 &&
timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 3 > $O/r03q_ab.log 2>&1 &&
SRT_LIB_PATH=$PWD/abtest/libprev.so timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 3 >> $O/r03q_ab.log 2>&1 &&
timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 3 >> $O/r03q_ab.log 2>&1
