set -e
for ph in 1 2 3; do
  SRT_FORM=dv_phases=$ph timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04l/p$ph -o run -- python3 bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04l/p$ph.log 2>&1
  echo "phase $ph done"
done
