#!/bin/bash
# A/B: arcs in flight per step of the one-key predecessor search (C4, kernel trace per variant)
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
for u in 16 24 32 8; do
SRT_PRED_U=$u timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03ag_prof_u$u -o run -- python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/r03ag_prof_u$u.log 2>&1 || exit 1
done
