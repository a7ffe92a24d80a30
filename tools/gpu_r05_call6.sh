# Round 5, sixth GPU call: the octet chain loop's K+W load / wait schedules (tools/ubench/oct_var,
# lone wave, state checked), then the whole GPU suite on the new default k_scan (256-thread
# workgroups two per CU, first line with the history block, exact pass fused).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 tools/ubench/oct_var > gpurun_out/r05_oct_var.log 2>&1 || exit $?
python -m bs_amd.build
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_gpu_call6.log 2>&1
