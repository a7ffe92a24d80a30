# k_scan stage time for experiment builds (results meaningless except the default build):
# loads from HBM and/or LDS table lookups replaced by register arithmetic.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/scan_variants.log
for v in libbsgpu.so libbsgpu_nolds.so libbsgpu_noload.so libbsgpu_nolds_noload.so; do
  BSG_LIB_PATH=$PWD/bs_amd/$v timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 2 --warmup 1 --cpu-sample-mib 0 --e2e-mib 0 > gpurun_out/sv.json 2>/dev/null || true
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sv.json').read()); print('$v', d['stage_ms'])" >> gpurun_out/scan_variants.log 2>&1 || echo "$v failed" >> gpurun_out/scan_variants.log
done
