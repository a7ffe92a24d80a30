# Round 6, thirteenth GPU call: the bench's N>1 path rehearsed on the one card (two ranks sharing
# it, BSG_BENCH_SHARE_GPU=1: the driver's 8-GPU launch form, torch.distributed.run, barrier and
# max-over-ranks timing, each rank its own configs[1] stream and oracle check).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
BSG_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 0 > gpurun_out/r06_bench_n2_shared_gpu_rehearsal.log 2>&1 || exit $?
