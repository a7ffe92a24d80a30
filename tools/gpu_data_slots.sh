# Data slots decoupled from engines (H2D on a copy stream): streaming parity tests, the e2e
# trace, e2e 1 GiB / 4 GiB A/B against a variant build (VARIANT), Writer/raw A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${VARIANT:-bs_amd/variants/lib_pre_data.so}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split_writer.py tests/test_gpu_concurrency.py tests/test_gpu_device_error.py tests/test_gpu_large_streams.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/ds_pytest.log 2>&1 || exit $?
bash tools/gpu_e2e_trace.sh || exit $?
for r in 1 2; do
  for lib in bs_amd/libbsgpu.so $V; do
    for mib in 1024 4096; do
      echo "== $lib $mib" >> gpurun_out/ds_e2e_ab.log
      BSG_LIB_PATH=$lib BSG_LIB_PARTIAL=1 E2E_MIB=$mib timeout -k 10 120 python -u tools/e2e_trace_run.py >> gpurun_out/ds_e2e_ab.log 2>&1 || exit $?
    done
  done
done
timeout -k 10 400 python -u tools/writer_ab.py bs_amd/libbsgpu.so $V > gpurun_out/ds_writer_ab.log 2>&1 || exit $?
