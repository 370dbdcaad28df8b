set -o pipefail
export TMPDIR=/tmp
bash tools/pmc_kernel.sh c4 'lvl_pred|rel_pk|lvl_step|transpose|lvl_arcs' r06zm/pmc_c4 'fetch write tcc'
