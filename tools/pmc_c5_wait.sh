#!/bin/bash
# Two counter passes over the C5 workgroup kernel: L1->L2 read latency (TCP) and where the waves'
# cycles go (SQ). One bench step each; summaries parsed by the caller.
set -e
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_c5_wait
mkdir -p $OUT
B="$ROOT/bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline"
K=wgsssp_kernel
timeout -s KILL 300 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum --kernel-include-regex $K --output-format csv -d $OUT/tcp -o run -- python3 $B > $OUT/tcp.log 2>&1
echo tcp-done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM --kernel-include-regex $K --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1
echo sq-done
