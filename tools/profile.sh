#!/bin/bash
# rocprofv3 kernel-trace --stats + separate FETCH_SIZE / WRITE_SIZE passes over one bench step of
# the FW update kernel (run on the GPU box from the repo root), then the summaries for profiles/.
# usage: tools/profile.sh <workload> <tag> [kernel-regex]
set -e
WL=${1:-c4}
TAG=${2:-r01}
KREGEX=${3:-fw16_update}
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_${TAG}_${WL}
mkdir -p $OUT
BENCH="python3 $ROOT/bench.py --workload $WL --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BENCH > $OUT/trace.log 2>&1
echo trace-done
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/fetch -o run -- $BENCH > $OUT/fetch.log 2>&1
echo fetch-done
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/write -o run -- $BENCH > $OUT/write.log 2>&1
echo write-done
python3 $ROOT/tools/pmc_summary.py $OUT "$KREGEX" $OUT/pmc_summary.json --stats-out $OUT/kernel_stats.csv
echo profile-done
