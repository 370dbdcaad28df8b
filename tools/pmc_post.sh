#!/bin/bash
# Counter passes over the C4 dense post pass kernels (one build each): kernel trace, where the
# wave cycles go (SQ), L2 hits. Usage: tools/pmc_post.sh [regex]
set -e
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_post
mkdir -p $OUT
K=${1:-"pred_cols2|rel_levels"}
B="$ROOT/bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1
echo trace-done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SMEM --kernel-include-regex "$K" --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1
echo sq-done
timeout -s KILL 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex "$K" --output-format csv -d $OUT/sq2 -o run -- python3 $B > $OUT/sq2.log 2>&1
echo sq2-done
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$K" --output-format csv -d $OUT/tcc -o run -- python3 $B > $OUT/tcc.log 2>&1
echo tcc-done
