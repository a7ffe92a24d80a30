# Round 6: the bench contract test and one bench line in the driver's default form after the
# line gained its host_settings record.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_bench_contract.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r06_c18_pytest.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_c18_bench.log 2>&1 || exit $?
