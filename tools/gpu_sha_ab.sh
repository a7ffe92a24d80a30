# A/B of k_sha builds: parity of each, then configs[2] / configs[1] lines with the k_sha timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/sha_ab.log
for lib in bs_amd/libbsgpu.so bs_amd/libbsgpu_v_*.so; do
  BSG_LIB_PATH=$PWD/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_sha.log 2>&1 || exit $?
  echo "$lib parity: $(tail -1 gpurun_out/pytest_sha.log)" >> gpurun_out/sha_ab.log
done
for rep in 1 2 3; do
for lib in bs_amd/libbsgpu.so bs_amd/libbsgpu_v_*.so; do
  for cfg in "--streams 256 --stream-mib 64" ""; do
    BSG_LIB_PATH=$PWD/$lib timeout -k 10 120 python bench.py $cfg --steps 3 --warmup 1 --cpu-sample-mib 0 --e2e-mib 0 > gpurun_out/sv.json 2>gpurun_out/sv.err || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/sv.json').read()); p=d['sha_path']; print('$lib', '$cfg', d['value'], d['stage_ms']['k_sha'], p.get('timeline_us'), p['long']['cycles_per_block'])" >> gpurun_out/sha_ab.log
  done
done
done
