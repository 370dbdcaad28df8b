set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06zh
mkdir -p $O
timeout -k 10 300 python -u tools/solo_rank.py --ranks 8 --which 0,3,7 --wire-gbps 0,64 > $O/solo_n8.jsonl 2> $O/solo_n8.err && \
timeout -k 10 300 python -u tools/solo_rank.py --ranks 4 --which 0,3 --wire-gbps 0,64 > $O/solo_n4.jsonl 2> $O/solo_n4.err && \
timeout -k 10 300 python -u tools/solo_rank.py --ranks 2 --which 0,1 --wire-gbps 0,64 > $O/solo_n2.jsonl 2> $O/solo_n2.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_solo8 -o run -- python3 tools/solo_rank.py --ranks 8 --which 3 --wire-gbps 64 --reps 3 > $O/prof_solo8.log 2>&1 && \
bash tools/run_round.sh r06zh bench:c4:20 bench:c2:20 bench:c3:10 bench:c4metric:3 bench:c5:3 prof:c4
