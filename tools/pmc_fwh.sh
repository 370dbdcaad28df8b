#!/bin/bash
# SQ counter passes over the pipelined f16-compare FW update kernel (tools/fw16_ablate, fwh only).
set -e
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_fwh
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
B="$ROOT/tools/fw16_ablate 32768 fwh"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex fwh_update --output-format csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1
echo p1-done
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS --kernel-include-regex fwh_update --output-format csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1
echo p2-done
