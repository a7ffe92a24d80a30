# Round 4 evidence, part B: rocprofv3 kernel-trace + FETCH_SIZE / WRITE_SIZE passes for configs[1]
# and configs[2], the e2e sweep, per-wave per-lane exit times on configs[2] (BSG_LANE_DIAG build),
# and the N=2 launch rehearsed with both ranks on the one card.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=prof_c1 BENCH_ARGS="--cpu-sample-mib 0 --e2e-mib 0 --configs2-steps 0" bash tools/gpu_trace_args.sh || exit $?
OUT=prof_c2 bash tools/gpu_trace_args.sh || exit $?
timeout -k 10 300 python tools/e2e_bench.py > gpurun_out/r04_e2e.log 2>&1 || exit $?
BSG_LIB_PATH=bs_amd/variants/lib_lanediag.so timeout -k 10 200 python tools/lane_waves.py > gpurun_out/r04_lane_waves.log 2>&1 || exit $?
BSG_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r04_bench_n2_shared_gpu_rehearsal.log 2>&1
