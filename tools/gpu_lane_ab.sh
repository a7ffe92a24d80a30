# GPU tests with the default library, then bench configs[1]/[2] for it and each variant in
# bs_amd/variants/ (A/B on one box), then the lane-diag variant's raw counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -2 gpurun_out/ab/pytest.log
bash tools/gpu_variant_sweep.sh || exit $?
for f in gpurun_out/sweep/*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_ms"], d["sha_path"].get("timeline_us"))')"; done
BSG_DIAG_RAW=1 BSG_LIB_PATH=$PWD/bs_amd/variants/lib_lanediag.so timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 3 --warmup 1 --cpu-sample-mib 0 --e2e-mib 0 > gpurun_out/ab/diag_c2.log 2>&1 || exit $?
echo done
