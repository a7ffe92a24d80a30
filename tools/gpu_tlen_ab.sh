# A/B of the wave-mode threshold: configs[2] and configs[1] lines with the k_sha timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/tlen_ab.log
for rep in 1 2; do
for lib in bs_amd/libbsgpu.so bs_amd/libbsgpu_v_*.so; do
  for cfg in "--streams 256 --stream-mib 64" ""; do
    BSG_LIB_PATH=$PWD/$lib timeout -k 10 120 python bench.py $cfg --steps 3 --warmup 1 --cpu-sample-mib 0 --e2e-mib 0 > gpurun_out/sv.json 2>gpurun_out/sv.err || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/sv.json').read()); p=d['sha_path']; print('$lib', '$cfg', d['value'], d['stage_ms']['k_sha'], p.get('timeline_us'), p['wave_tickets'], p['nlong'])" >> gpurun_out/tlen_ab.log
  done
done
done
