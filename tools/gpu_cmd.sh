set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06zi
mkdir -p $O
SRT_LIB_PATH=$(pwd)/shadow_amd/ab_xp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_xp -o run -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_xp.log 2>&1; \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_def -o run -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_def.log 2>&1
