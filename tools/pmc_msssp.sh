#!/bin/bash
# Counter passes over the multi-source kernel on C3 (one rows(0, n) call each): kernel trace,
# where the wave cycles go (SQ), HBM-side bytes (FETCH_SIZE / WRITE_SIZE, separate passes), L2 hits.
set -e
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_msssp_${1:-c3}
mkdir -p $OUT
B="$ROOT/tools/msssp_probe.py ${1:-c3} --reps 1"
K=msssp_kernel
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1
echo trace-done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --kernel-include-regex $K --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1
echo sq-done
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $K --output-format csv -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.log 2>&1
echo fetch-done
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $K --output-format csv -d $OUT/write -o run -- python3 $B > $OUT/write.log 2>&1
echo write-done
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex $K --output-format csv -d $OUT/tcc -o run -- python3 $B > $OUT/tcc.log 2>&1
echo tcc-done
