#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_msssp.py -v --timeout 120 --timeout-method thread > $O/r03n_msssp.log 2>&1 &&
SRT_MSSSP_PROF=1 timeout -k 10 120 python -u tools/msssp_probe.py c3 > $O/r03n_probe.log 2>&1 &&
timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 3 >> $O/r03n_probe.log 2>&1 &&
SRT_MSSSP_U16=0 timeout -k 10 120 python -u tools/msssp_probe.py c3 --reps 3 >> $O/r03n_probe.log 2>&1 &&
bash tools/pmc_msssp.sh c3 >> $O/r03n_probe.log 2>&1
