set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06zo
mkdir -p $O
bash tools/run_round.sh r06zo tests && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
