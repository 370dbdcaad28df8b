#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_msssp.py -v --timeout 120 --timeout-method thread > $O/r03o_msssp.log 2>&1 &&
SRT_MSSSP_PROF=1 timeout -k 10 120 python -u tools/msssp_probe.py c3 > $O/r03o_probe.log 2>&1 &&
timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 3 >> $O/r03o_probe.log 2>&1 &&
SRT_MSSSP_A32=0 timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 3 >> $O/r03o_probe.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --kernel-include-regex msssp_kernel --output-format csv -d $O/r03o_sq -o run -- python3 tools/msssp_probe.py c3 --reps 1 > $O/r03o_sq.log 2>&1
