#!/bin/bash
set -o pipefail
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 300 --timeout-method thread > $O/r03ab_tests.log 2>&1
