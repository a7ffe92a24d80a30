set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample-mib 0 > gpurun_out/bench3.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample-mib 0 --stream-mib 64 --streams 256 > gpurun_out/bench3_multi.log 2>&1
