set -o pipefail
export TMPDIR=/tmp
bash tools/run_round.sh r06w tfile:tests/test_gpu_edge_form.py tfile:tests/test_gpu_dropin.py
