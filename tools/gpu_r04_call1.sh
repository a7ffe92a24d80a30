mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_large_streams.py tests/test_gpu_blob_hash.py tests/test_gpu_device_error.py -k "past_2_40 or pins_nothing or seek_drops or device_error or reader_verify or forced" > gpurun_out/r04_pytest_new.log 2>&1 && \
timeout -k 10 300 python -u bench.py --check > gpurun_out/r04_bench_base.log 2>&1
