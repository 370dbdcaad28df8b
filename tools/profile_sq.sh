#!/bin/bash
# SQ / GRBM counter passes over the FW update kernel (one pass per counter group).
set -e
WL=${1:-c4}
TAG=${2:-sq}
KRE=${3:-fw16_update}
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_${TAG}_${WL}
mkdir -p $OUT
BENCH="python3 $ROOT/bench.py --workload $WL --steps 1 --warmup 0 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex $KRE --output-format csv -d $OUT/sq1 -o run -- $BENCH > $OUT/sq1.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM --kernel-include-regex $KRE --output-format csv -d $OUT/sq2 -o run -- $BENCH > $OUT/sq2.log 2>&1
echo sq-done
