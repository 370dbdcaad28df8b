set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06zj
mkdir -p $O
gcc -O2 -std=gnu11 -Ishadow_amd/csrc -Iinclude tests/gml_parallel_check.c shadow_amd/csrc/gml.c -o /tmp/gmlchk -lpthread -lm && \
python tools/gml_big.py /tmp/big.gml && \
/tmp/gmlchk /tmp/big.gml 16 time > $O/gml_check.txt 2> $O/gml_box16.jsonl && \
/tmp/gmlchk /tmp/big.gml 8 time >> $O/gml_check.txt 2> $O/gml_box8.jsonl && \
bash tools/run_round.sh r06zj tfile:tests/test_gpu_dropin.py tfile:tests/test_gpu_parity.py
