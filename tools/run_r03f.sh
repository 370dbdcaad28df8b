#!/bin/bash
# round 3: two-deep sharded rounds (cs2) + dense rows for few attached vertices
set -o pipefail
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c4.py -k "virtual or in_process" -x -v --timeout 300 --timeout-method thread > $O/r03f_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py -x -v -s --timeout 300 --timeout-method thread > $O/r03f_dropin.log 2>&1 &&
timeout -k 10 300 python -u tools/solo_rank.py --ranks 8 --which 0,7 --wire-gbps 0,50,64,100,150 > $O/r03f_solo_n8_deep.jsonl 2> $O/r03f_solo_n8.err &&
timeout -k 10 300 python -u tools/solo_rank.py --ranks 4 --which 0 --wire-gbps 0,64 > $O/r03f_solo_n4_deep.jsonl 2> $O/r03f_solo_n4.err &&
SRT_FW_SH_DEEP=0 timeout -k 10 300 python -u tools/solo_rank.py --ranks 4 --which 0 --wire-gbps 0,64 > $O/r03f_solo_n4_shallow.jsonl 2>> $O/r03f_solo_n4.err
