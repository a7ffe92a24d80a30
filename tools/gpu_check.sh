set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python tools/probe_torch.py > gpurun_out/probe_torch.log 2>&1
echo "probe rc=$?" >> gpurun_out/probe_torch.log
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample-mib 64 --check > gpurun_out/bench1.log 2>&1
