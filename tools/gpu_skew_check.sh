set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench/skew > gpurun_out/skew.log 2>&1 || exit $?
grep -q "asm block loop.*MATCH" gpurun_out/skew.log || exit 3
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split_writer.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_scan.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample-mib 0 --e2e-mib 0 > gpurun_out/bench_c1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample-mib 0 --e2e-mib 0 --stream-mib 64 --streams 256 > gpurun_out/bench_c2.log 2>&1
