set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u tools/stress_parity.py 400 400000 > gpurun_out/stress_parity_r02c.log 2>&1 || exit $?
BSG_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_n2_rehearsal.log 2>&1 || exit $?
timeout -k 10 60 python bench.py --gpus 2 > gpurun_out/bench_wrong_gpus.log 2>&1; echo "exit $?" >> gpurun_out/bench_wrong_gpus.log
