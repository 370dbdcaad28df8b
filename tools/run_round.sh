#!/bin/bash
# One parameterised GPU-box runner (replaces the per-session tools/run_r03*.sh scripts).
#
# usage: bash tools/run_round.sh <tag> <step> [<step> ...]
#   tests[:<pytest -k expr>]       the -m gpu suite (or a -k subset)
#   tfile:<tests/file.py>[:<-k>]   one GPU test file
#   bench:<wl>[:<steps>[:<settings>]]   one bench.py line (c2 c3 c4 c5) -> bench_<wl>*.json
#   prof:<wl>[:<settings>]         rocprofv3 --kernel-trace --stats of a 3-step bench
#   solo:<ranks>:<gbps list>[:<settings>]   tools/solo_rank.py (one rank of N alone)
# <settings>: items joined by '+'; an UPPER-case key is an environment variable
# (SRT_VIRTUAL_RANKS=4), a lower-case one an SRT_FORM key (levels=0+sym=0 -> SRT_FORM=levels=0,sym=0)
#   py:<script>[:<args with , for spaces>]      python tools/<script>
# Every step runs under its own timeout; the steps are chained with && (the first failure ends
# the call). Output lands in gpurun_out/<tag>/.
set -o pipefail
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"

envs() { # "A=1+k=v+j=w" -> env words: A=1 SRT_FORM=k=v,j=w
    [ -z "$1" ] && return 0
    local form="" item
    for item in $(echo "$1" | tr '+' ' '); do
        case $item in
        [A-Z]*) echo -n "$item " ;;
        *) form="${form:+$form,}$item" ;;
        esac
    done
    [ -n "$form" ] && echo -n "SRT_FORM=$form"
    echo
}

run_step() {
    local s=$1
    IFS=':' read -r kind a b c <<< "$s"
    case $kind in
    tests)
        if [ -n "$a" ]; then
            timeout -k 10 900 $PYT tests/ -m gpu -k "$a" > $O/gpu_tests_k.log 2>&1
        else
            timeout -k 10 900 $PYT tests/ -m gpu > $O/gpu_tests.log 2>&1
        fi ;;
    tfile)
        local lg=$O/$(basename $a .py).log
        if [ -n "$b" ]; then
            timeout -k 10 600 $PYT $a -m gpu -k "$b" > $lg 2>&1
        else
            timeout -k 10 600 $PYT $a -m gpu > $lg 2>&1
        fi ;;
    bench)
        local st=${b:-5} sfx=""
        [ -n "$c" ] && sfx="_$(echo $c | tr '+=' '__')"
        env $(envs "$c") timeout -k 10 600 python -u bench.py --workload $a --steps $st \
            --warmup 1 > $O/bench_$a$sfx.json 2> $O/bench_$a$sfx.err ;;
    prof)
        local sfx=""
        [ -n "$b" ] && sfx="_$(echo $b | tr '+=' '__')"
        env $(envs "$b") timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
            -d $O/prof_$a$sfx -o run -- python3 bench.py --workload $a --steps 3 --warmup 1 \
            --no-cpu-baseline > $O/prof_$a$sfx.log 2>&1 ;;
    solo)
        env $(envs "$c") timeout -k 10 600 python -u tools/solo_rank.py --ranks $a --which 0 \
            --wire-gbps $b >> $O/solo_n$a.jsonl 2> $O/solo_n$a.err ;;
    py)
        timeout -k 10 600 python -u tools/$a $(echo "$b" | tr ',' ' ') > $O/${a%.py}.out \
            2> $O/${a%.py}.err ;;
    *)
        echo "unknown step $s"; return 2 ;;
    esac
    local rc=$?
    echo "[run_round] $s -> $rc"
    return $rc
}

for s in "$@"; do
    run_step "$s" || exit $?
done
