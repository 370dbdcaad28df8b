#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_msssp.py -v --timeout 120 --timeout-method thread > $O/r03m_msssp.log 2>&1 &&
SRT_MSSSP_PROF=1 timeout -k 10 120 python -u tools/msssp_probe.py c3 > $O/r03m_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 SRT_SPARSE_MS=1 timeout -k 10 200 python -u tools/msssp_probe.py c5 --reps 1 >> $O/r03m_probe.log 2>&1 &&
timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 3 >> $O/r03m_probe.log 2>&1 &&
SRT_MSSSP_U16=0 timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 3 >> $O/r03m_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 SRT_MSSSP_DELTA=128 timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 1 >> $O/r03m_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 SRT_MSSSP_DELTA=256 timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 1 >> $O/r03m_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 SRT_MSSSP_DELTA=32 timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 1 >> $O/r03m_probe.log 2>&1 &&
SRT_SPARSE_MS=0 timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 2 >> $O/r03m_probe.log 2>&1
