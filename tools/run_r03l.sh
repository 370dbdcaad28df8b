#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_msssp.py -v --timeout 120 --timeout-method thread > $O/r03l_msssp.log 2>&1 &&
SRT_MSSSP_PROF=1 timeout -k 10 120 python -u tools/msssp_probe.py c3 > $O/r03l_probe.log 2>&1 &&
timeout -k 10 120 python -u tools/msssp_probe.py c3 >> $O/r03l_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 SRT_MSSSP_DELTA=32 timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 1 >> $O/r03l_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 SRT_MSSSP_DELTA=64 timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 1 >> $O/r03l_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 SRT_MSSSP_DELTA=8 timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 1 >> $O/r03l_probe.log 2>&1
