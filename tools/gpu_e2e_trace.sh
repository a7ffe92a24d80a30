# Kernel + memory-copy trace of the streaming path (e2e bench, one tile size).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
export E2E_TILES=${E2E_TILES:-64} E2E_MIB=${E2E_MIB:-1024}
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/e2e_trace -o run --output-format csv -- python3 tools/e2e_bench.py > gpurun_out/e2e_trace.log 2>&1
