set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python tools/diag_hild.py 65536 1010 gpurun_out/diag_hild.json > gpurun_out/diag_hild.log 2>&1
