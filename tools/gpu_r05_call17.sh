# Round 5, seventeenth GPU call: checkpoint of the current head: smoke, the default bench line
# twice (configs[1] + nested configs[2] + e2e + CPU baseline), as the driver runs it.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_ckpt.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r05_bench_ckpt1.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r05_bench_ckpt2.log 2>&1
