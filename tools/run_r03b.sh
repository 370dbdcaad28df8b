#!/bin/bash
# round 3: C4 bench after the raw-row change, solo-rank wire sweep at N = 8 / 4
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/r03b_bench_c4.json 2> $O/r03b_bench_c4.err &&
timeout -k 10 300 python -u tools/solo_rank.py --ranks 8 --which 0,4,7 --wire-gbps 0,50,64,100,150 > $O/r03b_solo_n8_wire.jsonl 2> $O/r03b_solo_n8.err &&
timeout -k 10 300 python -u tools/solo_rank.py --ranks 4 --which 0,3 --wire-gbps 0,64 > $O/r03b_solo_n4_wire.jsonl 2> $O/r03b_solo_n4.err
