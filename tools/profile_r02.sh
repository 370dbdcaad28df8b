#!/bin/bash
# One-GPU profile of a bench workload: kernel trace + stats, then one rocprofv3 --pmc pass per
# counter group (never combined with tracing): HBM (FETCH_SIZE, WRITE_SIZE), LDS / VALU (SQ), clock
# (GRBM). Summaries land in gpurun_out/prof_<tag>_<wl>/; tools/pmc_summary.py condenses them.
# usage: tools/profile_r02.sh <workload> <tag> <kernel-regex>
set -e
WL=${1:-c4}
TAG=${2:-r02}
KRE=${3:-fwq_update}
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_${TAG}_${WL}
mkdir -p $OUT
BENCH="$ROOT/bench.py --workload $WL --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.log 2>&1
echo trace-done
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/fetch -o run -- python3 $BENCH > $OUT/fetch.log 2>&1
echo fetch-done
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/write -o run -- python3 $BENCH > $OUT/write.log 2>&1
echo write-done
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "$KRE" --output-format csv -d $OUT/sq -o run -- python3 $BENCH > $OUT/sq.log 2>&1
echo sq-done
# with the kernel trace of the same (serialized) launches: the clock is GRBM_GUI_ACTIVE / 8 over
# their own duration
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "$KRE" --output-format csv -d $OUT/grbm -o run -- python3 $BENCH > $OUT/grbm.log 2>&1
echo grbm-done
