# Round 6, eighth GPU call: k_scan's fast pass as one aligned asm statement (tools/gen_scan_loop.py).
# The scan parity tests first, then configs[2] and configs[1] against the previous head's library
# (bs_amd/ab/libbsgpu_head.so), three alternations each, then one kernel trace of configs[2] per
# library (k_scan's own time).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan_edges.py tests/test_gpu_parity.py tests/test_gpu_params.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_c8_pytest.log 2>&1 || exit $?
C2="--steps 20 --warmup 5 --streams 256 --stream-mib 64 --e2e-mib 0 --no-writer-e2e --cpu-sample-mib 0"
C1="--steps 20 --warmup 5 --configs2-steps 0 --e2e-mib 0 --no-writer-e2e --cpu-sample-mib 0"
for i in 1 2 3; do
  BSG_LIB_PATH=bs_amd/ab/libbsgpu_head.so timeout -k 10 200 python -u bench.py $C2 > gpurun_out/r06_c8_c2_head_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py $C2 > gpurun_out/r06_c8_c2_asm_$i.log 2>&1 || exit $?
done
for i in 1 2 3; do
  BSG_LIB_PATH=bs_amd/ab/libbsgpu_head.so timeout -k 10 200 python -u bench.py $C1 > gpurun_out/r06_c8_c1_head_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py $C1 > gpurun_out/r06_c8_c1_asm_$i.log 2>&1 || exit $?
done
C2T="--steps 5 --warmup 2 --streams 256 --stream-mib 64 --e2e-mib 0 --no-writer-e2e --cpu-sample-mib 0"
BSG_LIB_PATH=bs_amd/ab/libbsgpu_head.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_c8_trace_head -o run --output-format csv -- python3 bench.py $C2T > gpurun_out/r06_c8_trace_head.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_c8_trace_asm -o run --output-format csv -- python3 bench.py $C2T > gpurun_out/r06_c8_trace_asm.log 2>&1 || exit $?
