# The driver's bench invocation (defaults, incl. the CPU baseline), configs[2], and e2e.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample-mib 0 --stream-mib 64 --streams 256 > gpurun_out/bench_c2.log 2>&1 && \
timeout -k 10 300 python tools/e2e_bench.py > gpurun_out/e2e.log 2>&1
