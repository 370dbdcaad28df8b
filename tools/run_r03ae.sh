#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
SRT_TRANSPOSE_NT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "c2 or complete or dense" --timeout 300 --timeout-method thread > $O/r03ae_tests.log 2>&1 &&
SRT_TRANSPOSE_NT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03ae_prof_nt1 -o run -- python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/r03ae_prof_nt1.log 2>&1 &&
SRT_TRANSPOSE_NT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03ae_prof_nt0 -o run -- python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/r03ae_prof_nt0.log 2>&1
