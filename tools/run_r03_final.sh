#!/bin/bash
# Round-3 state on one MI355X: the whole -m gpu suite, then the four bench lines and the C4 trace.
set -o pipefail
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
for w in c4 c2 c3 c5; do
  timeout -k 10 600 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
done &&
timeout -k 10 300 python -u tools/wide_probe.py 256 > $O/wide_probe.json 2> $O/wide_probe.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_c4.log 2>&1
