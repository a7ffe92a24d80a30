# Round 5, thirty-third GPU call: where configs[1]'s step time goes after the longest chain
# ends (the step is ~0.13 ms longer than the chain's end): a kernel + memory-copy + HIP API trace
# of bench configs[1] (5 timed steps), for tools/step_gaps.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 5 --warmup 2 --configs2-steps 0 --cpu-sample-mib 0 --e2e-mib 0"
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d gpurun_out/gaps33 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/gaps33.log 2>&1
