#!/bin/bash
# A/B of side-by-side library builds on the GPU box: each variant is a copy of shadow_amd/csrc
# with the change applied (or an older commit's tree, git archive), built with
# make OUT=<repo>/shadow_amd/ab_<v>.so (the product sources carry no variant macros):
# per variant, the level parity tests, then a C4 bench line.
# usage: bash tools/ab_libs.sh <tag> <workload> <variant> [<variant> ...]   (variant "default" or
# the <v> of shadow_amd/ab_<v>.so); AB_TESTS overrides the parity tests run per variant
# (default: tests/test_gpu_levels.py -k match_oracle)
set -o pipefail
TAG=$1; WL=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
for v in "$@"; do
    if [ "$v" = default ]; then LP=""; else LP=$(pwd)/shadow_amd/ab_$v.so; fi
    # variants named x*: timing diagnostics (wrong tables), no parity tests
    [ "${v#x}" = "$v" ] && SRT_LIB_PATH=$LP timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
        ${AB_TESTS:-tests/test_gpu_levels.py -k match_oracle} -m gpu > $O/tests_$v.log 2>&1 || [ "${v#x}" != "$v" ] || { echo "$v tests failed"; exit 1; }
    SRT_LIB_PATH=$LP timeout -k 10 300 python -u bench.py --workload $WL --steps 5 --warmup 1 \
        --no-cpu-baseline > $O/bench_${WL}_$v.json 2> $O/bench_${WL}_$v.err || { echo "$v bench failed"; exit 1; }
    echo "$v $(python3 -c "import json,sys;d=json.loads(open('$O/bench_${WL}_$v.json').read().strip().splitlines()[-1]);r=d['roofline'];ks=r.get('kernels',{});print(d['ms_per_step'], r.get('kernel'), r.get('avg_launch_ms'), {k:v['ms_per_build'] for k,v in ks.items()} if isinstance(ks,dict) else [(k['kernel'],k['avg_launch_ms']) for k in ks])")"
done
