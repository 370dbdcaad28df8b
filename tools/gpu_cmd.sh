set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06zr
mkdir -p $O
bash tools/run_round.sh r06zr tfile:tests/test_gpu_levels.py tfile:tests/test_gpu_c4.py tfile:tests/test_gpu_protocol.py && \
AB_TESTS="tests/test_gpu_protocol.py tests/test_gpu_levels.py" SRT_LIB_PATH=$(pwd)/shadow_amd/ab_n8.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 tests/test_gpu_protocol.py tests/test_gpu_levels.py -m gpu > $O/tests_n8.log 2>&1 && \
for i in 1 2; do
for v in prev new n8; do
LP=""; [ $v = prev ] && LP=$(pwd)/shadow_amd/ab_prev.so; [ $v = n8 ] && LP=$(pwd)/shadow_amd/ab_n8.so
SRT_LIB_PATH=$LP timeout -k 10 300 python -u bench.py --workload c4 --steps 10 --warmup 1 --no-cpu-baseline > $O/bench_c4_${v}_$i.json 2> $O/bench_c4_${v}_$i.err || exit 1
SRT_LIB_PATH=$LP timeout -k 10 300 python -u tools/solo_rank.py --ranks 8 --which 0,3,7 --wire-gbps 64 > $O/solo_n8_${v}_$i.jsonl 2> $O/solo_n8_${v}_$i.err || exit 1
done
done
