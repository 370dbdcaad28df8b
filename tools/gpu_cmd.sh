set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
SRT_LIB_PATH=$(pwd)/shadow_amd/ab_hp.so timeout -k 10 300 python -u tools/solo_rank.py --ranks 8 --which 3 --wire-gbps 64 > $O/solo_hp.jsonl 2> $O/solo_hp.err && \
bash tools/run_round.sh r06q tfile:tests/test_gpu_levels.py && \
for i in 1 2; do
for v in head new; do
LP=""; [ $v = head ] && LP=$(pwd)/shadow_amd/ab_head.so
SRT_LIB_PATH=$LP timeout -k 10 300 python -u tools/solo_rank.py --ranks 8 --which 0,3,7 --wire-gbps 0,64 > $O/solo_n8_${v}_$i.jsonl 2> $O/solo_n8_${v}_$i.err || exit 1
SRT_LIB_PATH=$LP timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 1 --no-cpu-baseline > $O/bench_c4_${v}_$i.json 2> $O/bench_c4_${v}_$i.err || exit 1
done
done
