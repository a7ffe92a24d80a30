# A/B of k_scan builds: parity of every build but the NOLOAD experiment, then configs[2] and
# configs[1] stage times for each build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/scan_ab.log
for lib in bs_amd/libbsgpu.so bs_amd/libbsgpu_v_*.so; do
  case $lib in *noload*) continue;; esac
  BSG_LIB_PATH=$PWD/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_scan.log 2>&1 || exit $?
  echo "$lib parity: $(tail -1 gpurun_out/pytest_scan.log)" >> gpurun_out/scan_ab.log
done
for rep in 1 2; do
for lib in bs_amd/libbsgpu.so bs_amd/libbsgpu_v_*.so; do
  for cfg in "--streams 256 --stream-mib 64" ""; do
    BSG_LIB_PATH=$PWD/$lib timeout -k 10 120 python bench.py $cfg --steps 3 --warmup 1 --cpu-sample-mib 0 --e2e-mib 0 > gpurun_out/sv.json 2>gpurun_out/sv.err || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/sv.json').read()); print('$lib', '$cfg', d['value'], d['stage_ms'])" >> gpurun_out/scan_ab.log
  done
done
done
