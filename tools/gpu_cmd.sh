set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06zn
mkdir -p $O
bash tools/run_round.sh r06zn tfile:tests/test_gpu_levels.py tfile:tests/test_gpu_c4.py tfile:tests/test_gpu_protocol.py && \
for i in 1 2; do
for v in prev new; do
LP=""; [ $v = prev ] && LP=$(pwd)/shadow_amd/ab_prev.so
SRT_LIB_PATH=$LP timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 1 --no-cpu-baseline > $O/bench_c4_${v}_$i.json 2> $O/bench_c4_${v}_$i.err || exit 1
SRT_LIB_PATH=$LP timeout -k 10 300 python -u tools/solo_rank.py --ranks 8 --which 0,3,7 --wire-gbps 64 > $O/solo_n8_${v}_$i.jsonl 2> $O/solo_n8_${v}_$i.err || exit 1
done
done && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_solo8 -o run -- python3 tools/solo_rank.py --ranks 8 --which 3 --wire-gbps 64 --reps 3 > $O/prof_solo8.log 2>&1
