#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
SRT_ESS_U16=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c4.py tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread > $O/r03af_tests.log 2>&1 &&
SRT_ESS_U16=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $O/r03af_c4.json 2> $O/r03af_c4.err &&
SRT_ESS_U16=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03af_prof_c4 -o run -- python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/r03af_prof_c4.log 2>&1
