# split::Writer with its records processed on a background thread: the Writer / store / reader /
# concurrency / > 4 GiB tests, the Writer time breakdown against a variant (VARIANT), and the
# host-TSan stress driver in GPU mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=${VARIANT:-bs_amd/variants/lib_pre_data.so}
timeout -k 10 600 python -u -m pytest tests/test_gpu_split_writer.py tests/test_gpu_concurrency.py tests/test_gpu_filestore.py tests/test_gpu_blob_hash.py tests/test_gpu_large_streams.py tests/test_gpu_device_error.py tests/test_gpu_ownership.py tests/test_gpu_abi_errors.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/wbg_pytest.log 2>&1 || exit $?
for r in 1 2; do
  echo "== default" >> gpurun_out/wbg_timing.log
  timeout -k 10 200 python -u tools/writer_timing.py >> gpurun_out/wbg_timing.log 2>&1 || exit $?
  echo "== $V" >> gpurun_out/wbg_timing.log
  BSG_LIB_PATH=$V BSG_LIB_PARTIAL=1 timeout -k 10 200 python -u tools/writer_timing.py >> gpurun_out/wbg_timing.log 2>&1 || exit $?
done
timeout -k 10 600 bash tools/tsan_host.sh gpu > gpurun_out/wbg_tsan_gpu.log 2>&1 || exit $?
