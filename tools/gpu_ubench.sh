set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/share > gpurun_out/ubench_share.log 2>&1
