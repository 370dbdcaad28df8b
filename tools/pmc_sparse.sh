#!/bin/bash
# Counter passes over the wave-per-source sparse kernel on C3 (one step of bench.py each).
set -e
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
WL=${1:-c3}
OUT=$ROOT/gpurun_out/pmc_sparse_$WL
mkdir -p $OUT
B="python3 $ROOT/bench.py --workload $WL --steps 1 --warmup 0 --no-cpu-baseline"
K=wsssp_kernel
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1
echo trace-done
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $K --output-format csv -d $OUT/fetch -o run -- $B > $OUT/fetch.log 2>&1
echo fetch-done
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $K --output-format csv -d $OUT/write -o run -- $B > $OUT/write.log 2>&1
echo write-done
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex $K --output-format csv -d $OUT/sq -o run -- $B > $OUT/sq.log 2>&1
echo sq-done
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex $K --output-format csv -d $OUT/tcc -o run -- $B > $OUT/tcc.log 2>&1
echo tcc-done
