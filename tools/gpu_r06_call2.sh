# Round 6, second GPU call: the whole GPU suite and smoke after the kernel-file cleanup (the
# rejected variants removed, ISA of the hot loops unchanged), one default bench line with the
# e2e tail breakdown, and one standalone round of the copy-form A/B for the e2e tail comparison.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_c2_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_c2_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_c2_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/host_copy_ab.py 1 > gpurun_out/r06_c2_copy_ab.log 2>&1 || exit $?
