# Round 6, sixteenth GPU call: the pre-k_sha ordering kernels with fewer same-address atomics
# (k_lens: one pair per workgroup instead of per wave; k_order's count pass on one workgroup per
# CU, flushed once), against the previous head (bs_amd/ab/libbsgpu_head.so). configs[2] kernel
# traces of both, configs[2] bench lines alternated three times, then the parity, configs,
# blob-hash and early-chain tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
C2T="--steps 5 --warmup 2 --streams 256 --stream-mib 64 --e2e-mib 0 --no-writer-e2e --cpu-sample-mib 0"
BSG_BENCH_INIT=0 BSG_LIB_PATH=bs_amd/ab/libbsgpu_head.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_c16_trace_head -o run --output-format csv -- python3 bench.py $C2T > gpurun_out/r06_c16_trace_head.log 2>&1 || exit $?
BSG_BENCH_INIT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_c16_trace_new -o run --output-format csv -- python3 bench.py $C2T > gpurun_out/r06_c16_trace_new.log 2>&1 || exit $?
C2="--steps 20 --warmup 5 --streams 256 --stream-mib 64 --e2e-mib 0 --no-writer-e2e --cpu-sample-mib 0"
for i in 1 2 3; do
  BSG_LIB_PATH=bs_amd/ab/libbsgpu_head.so timeout -k 10 200 python -u bench.py $C2 > gpurun_out/r06_c16_c2_head_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py $C2 > gpurun_out/r06_c16_c2_new_$i.log 2>&1 || exit $?
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_blob_hash.py tests/test_gpu_params.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_c16_pytest.log 2>&1 || exit $?
