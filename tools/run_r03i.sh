#!/bin/bash
# round 3: multi-source SSSP (msssp.hip) parity first, then the full GPU suite, then benches
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_msssp.py -v --timeout 300 --timeout-method thread > $O/r03i_msssp.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline > $O/r03i_bench_c3.json 2> $O/r03i_bench_c3.err &&
SRT_SPARSE_MS=0 timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline > $O/r03i_bench_c3_wave.json 2>> $O/r03i_bench_c3.err &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/r03i_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/r03i_bench_c4.json 2> $O/r03i_bench_c4.err &&
timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/r03i_bench_c2.json 2> $O/r03i_bench_c2.err
