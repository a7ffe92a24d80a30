# Round 5, tenth GPU call: the e2e streaming path (1 GiB through bsg_write) by tile size and
# engine slots (tools/e2e_trace_run.py, 5 reps each, no profiler).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "256 3" "128 3" "64 3" "128 4" "64 4" "64 6"; do
  set -- $cfg
  echo "== tile $1 MiB, slots $2" >> gpurun_out/r05_e2e_tiles.log
  E2E_TILE_MIB=$1 BSG_STREAM_SLOTS=$2 timeout -k 10 120 python3 tools/e2e_trace_run.py 2>&1 | python3 -c "
import sys, json
for l in sys.stdin:
    try: d = json.loads(l)
    except Exception: print(l.rstrip()); continue
    print(d['rep'], d['seconds'], d['write_phase_s'], d['chunks'], d['gib_per_s'])" >> gpurun_out/r05_e2e_tiles.log || exit $?
done
