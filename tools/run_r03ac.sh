#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
SRT_PRED_NT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c4.py -x -q --timeout 300 --timeout-method thread > $O/r03ac_tests.log 2>&1 &&
SRT_PRED_NT=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $O/r03ac_c4_nt1.json 2> $O/r03ac_c4_nt1.err &&
SRT_PRED_NT=0 timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $O/r03ac_c4_nt0.json 2> $O/r03ac_c4_nt0.err &&
SRT_PRED_NT=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $O/r03ac_c4_nt1b.json 2> $O/r03ac_c4_nt1b.err &&
SRT_PRED_NT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03ac_prof_c4 -o run -- python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/r03ac_prof_c4.log 2>&1 &&
SRT_PRED_NT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03ac_prof_c4_nt0 -o run -- python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/r03ac_prof_c4_nt0.log 2>&1
