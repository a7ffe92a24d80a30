set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/e2e_threads.log
for t in 4 8 12 16; do
  echo "copy_threads=$t" >> gpurun_out/e2e_threads.log
  BSG_COPY_THREADS=$t E2E_MIB=4096 E2E_TILES=256,512 timeout -k 10 300 python tools/e2e_bench.py 2>&1 | grep "C ABI" >> gpurun_out/e2e_threads.log || exit $?
done
