set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in D0 B1; do
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -f csv -d gpurun_out/pmc_$s -o run -- \
    ./tools/micro/hild_micro --state tools/micro/state$s.bin gpurun_out/q$s.bin > gpurun_out/pmc_$s.log 2>&1 || exit 1
done
