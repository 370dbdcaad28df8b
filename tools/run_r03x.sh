#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
for b in 64 128 256 512 1024; do
SRT_SQ_REDUCE_BLOCKS=$b timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03x_prof_$b -o run -- python3 bench.py --workload c2 --steps 5 --warmup 1 --no-cpu-baseline > $O/r03x_prof_$b.log 2>&1 || exit 1
done
