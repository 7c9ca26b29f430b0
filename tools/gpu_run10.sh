set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for s in B1 C D0 D1 D2 D3 D4; do
  timeout -k 10 60 ./tools/micro/hild_micro --state tools/micro/state$s.bin gpurun_out/p$s.bin > gpurun_out/r$s.log 2>&1 || exit 1
done
