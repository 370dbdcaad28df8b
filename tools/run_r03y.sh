#!/bin/bash
set -o pipefail
bash tools/run_r03w.sh && timeout -k 10 900 bash tools/pmc_post.sh
