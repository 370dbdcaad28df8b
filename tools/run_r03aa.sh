#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread > $O/r03aa_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/r03aa_bench_c2.json 2> $O/r03aa_bench_c2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03aa_prof_c2 -o run -- python3 bench.py --workload c2 --steps 5 --warmup 1 --no-cpu-baseline > $O/r03aa_prof_c2.log 2>&1
