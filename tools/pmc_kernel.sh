#!/bin/bash
# Counter passes over one kernel of a bench workload (run on the GPU box from the repo root):
# where the wave cycles go (SQ), instruction mix, L2 hits, and HBM traffic (FETCH/WRITE_SIZE),
# each pass its own rocprofv3 run.
# usage: tools/pmc_kernel.sh <workload> <kernel-regex> <tag> ["<passes>" (default: sq mix tcc fetch write)]
set -e
WL=${1:-c4}
K=${2:-lvl_pred}
TAG=${3:-pmc}
PASSES=${4:-sq mix tcc fetch write}
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
B="$ROOT/bench.py --workload $WL --steps 1 --warmup 0 --no-cpu-baseline"
run() { # name counters...
    local name=$1
    shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$K" --output-format csv \
        -d $OUT/$name -o run -- python3 $B > $OUT/$name.log 2>&1
    echo "$name-done"
}
for p in $PASSES; do
    case $p in
    sq) run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES ;;
    mix) run mix SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE ;;
    tcc) run tcc TCC_HIT_sum TCC_MISS_sum ;;
    fetch) run fetch FETCH_SIZE ;;
    write) run write WRITE_SIZE ;;
    esac
done
