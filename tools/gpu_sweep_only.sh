# bench configs[1]/[2] for the default library and each variant in bs_amd/variants/, one line each.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_variant_sweep.sh || exit $?
for f in gpurun_out/sweep/*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_ms"], d["sha_path"].get("timeline_us"), d["sha_path"].get("wave_tickets"))')"; done
