#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03r_prof_c2 -o run -- python3 bench.py --workload c2 --steps 5 --warmup 1 --no-cpu-baseline > $O/r03r_prof_c2.log 2>&1
