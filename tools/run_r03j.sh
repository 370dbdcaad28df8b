#!/bin/bash
# round 3: msssp profile on C3
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/msssp_probe.py c3 > $O/r03j_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 timeout -k 10 120 python -u tools/msssp_probe.py c3 >> $O/r03j_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 SRT_MSSSP_DELTA=64 timeout -k 10 120 python -u tools/msssp_probe.py c3 >> $O/r03j_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 SRT_MSSSP_SLOTS=256 timeout -k 10 120 python -u tools/msssp_probe.py c3 >> $O/r03j_probe.log 2>&1 &&
SRT_MSSSP_PROF=1 timeout -k 10 120 python -u tools/msssp_probe.py c3 --nsrc 64 >> $O/r03j_probe.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r03j_prof -o c3 -- python3 -u tools/msssp_probe.py c3 > $O/r03j_prof.log 2>&1
