#!/bin/bash
# round 3: state of HEAD after the re-entry -- full GPU suite, C4 and C2 benches
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/r03h_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/r03h_bench_c4.json 2> $O/r03h_bench_c4.err &&
timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/r03h_bench_c2.json 2> $O/r03h_bench_c2.err
