#!/bin/bash
# rocprofv3 kernel-trace + PMC passes over one bench step (run on the GPU box from the repo root).
# usage: tools/profile.sh <workload> <tag>
set -e
WL=${1:-c4}
TAG=${2:-r01}
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_${TAG}_${WL}
mkdir -p $OUT
BENCH="python3 $ROOT/bench.py --workload $WL --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BENCH > $OUT/trace.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex fw_update --output-format csv -d $OUT/fetch -o run -- $BENCH > $OUT/fetch.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex fw_update --output-format csv -d $OUT/write -o run -- $BENCH > $OUT/write.log 2>&1
echo profile-done
