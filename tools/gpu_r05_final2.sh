# Round 5 evidence at the head after BSG_KNOB_POLL: the GPU suite, smoke, the two default bench
# lines (the driver's forms) and the N=2 rehearsal on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05_pytest_gpu_final.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_final.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r05_bench_final.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r05_bench_default_args.log 2>&1 || exit $?
BSG_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 0 > gpurun_out/r05_bench_n2_shared_gpu_rehearsal.log 2>&1
