# Runs bench.py configs[1] and configs[2] against each library variant in bs_amd/variants/
# (plus the default build) and prints value + k_sha timeline per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
for lib in bs_amd/libbsgpu.so bs_amd/variants/lib_*.so; do
  n=$(basename $lib .so)
  BSG_LIB_PATH=$PWD/$lib timeout -k 10 120 python bench.py --steps 5 --warmup 2 --cpu-sample-mib 0 --e2e-mib 0 > gpurun_out/sweep/${n}_c1.log 2>&1 || exit $?
  BSG_LIB_PATH=$PWD/$lib timeout -k 10 120 python bench.py --streams 256 --stream-mib 64 --steps 3 --warmup 1 --cpu-sample-mib 0 --e2e-mib 0 > gpurun_out/sweep/${n}_c2.log 2>&1 || exit $?
  echo "$n done"
done
