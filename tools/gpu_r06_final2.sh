# Round 6 end-of-round evidence at the final head: the GPU suite, smoke, the driver's two bench
# forms, 300 more randomized parity draws (the streaming path changed: first_flush), then the
# kernel traces and counter passes (tools/gpu_r06_final_prof.sh, BSG_BENCH_INIT=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_pytest_gpu_final.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_final.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_bench_final.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r06_bench_default_args.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/stress_parity.py 300 97000 > gpurun_out/r06_stress_parity_final.log 2>&1 || exit $?
bash tools/gpu_r06_final_prof.sh || exit $?
