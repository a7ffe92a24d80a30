# Streaming (PCIe-inclusive) rate: slots x tile sweep on a 4 GiB stream, then the 1 GiB default.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/e2e_sweep.log
for k in 3 4; do
  echo "slots=$k" >> gpurun_out/e2e_sweep.log
  BSG_STREAM_SLOTS=$k E2E_MIB=4096 E2E_TILES=64,128,256,512 timeout -k 10 300 python tools/e2e_bench.py >> gpurun_out/e2e_sweep.log 2>&1 || exit $?
done
