set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
BSG_LONG_MODE=all timeout -k 5 60 python tools/repro_hang.py > gpurun_out/repro.log 2>&1 && \
BSG_LONG_MODE=off timeout -k 5 60 python tools/repro_hang.py >> gpurun_out/repro.log 2>&1 && \
timeout -k 5 60 python tools/repro_hang.py >> gpurun_out/repro.log 2>&1 && \
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-sample-mib 0 > gpurun_out/bench3.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample-mib 0 --stream-mib 64 --streams 256 > gpurun_out/bench3_multi.log 2>&1
