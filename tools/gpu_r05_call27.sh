# Round 5, twenty-seventh GPU call: per-lane blocks per iteration 3 and job-switch lead 3 on the
# leaner per-lane loop (ballot-guarded branches, shared load base), against the default (2, 4):
# configs[2], three interleaved rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in new bpi3 lead3; do
    if [ $v = new ]; then lib=bs_amd/libbsgpu.so; else lib=bs_amd/variants/lib_$v.so; fi
    echo "== $v round $r" >> gpurun_out/r05_ab27_c2.log
    BSG_LIB_PATH=$lib timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 10 --warmup 3 --cpu-sample-mib 0 --e2e-mib 0 >> gpurun_out/r05_ab27_c2.log 2>&1 || exit $?
  done
done
