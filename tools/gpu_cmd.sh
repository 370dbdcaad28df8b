set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06zs
mkdir -p $O
bash tools/run_round.sh r06zs tests && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err && \
bash tools/run_round.sh r06zs bench:c4:20 prof:c4 && \
timeout -k 10 300 python -u tools/solo_rank.py --ranks 8 --which 0,3,7 --wire-gbps 0,64 > $O/solo_n8.jsonl 2> $O/solo_n8.err && \
timeout -k 10 300 python -u tools/solo_rank.py --ranks 4 --which 0,3 --wire-gbps 0,64 > $O/solo_n4.jsonl 2> $O/solo_n4.err && \
timeout -k 10 300 python -u tools/solo_rank.py --ranks 2 --which 0,1 --wire-gbps 0,64 > $O/solo_n2.jsonl 2> $O/solo_n2.err
