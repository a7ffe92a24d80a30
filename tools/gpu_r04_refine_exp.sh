# Where k_refine's time goes (experiment builds, timing only): the default, one that returns
# after its table load and strip-start cache (rexp1), one without the table load (rexp2).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rexp
export TMPDIR=/tmp
for v in base rexp1 rexp2; do
  BSG_LIB_PATH=bs_amd/variants/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rexp/$v -o run --output-format csv -- python3 bench.py --cpu-sample-mib 0 --e2e-mib 0 --steps 5 --warmup 2 > gpurun_out/rexp/$v.log 2>&1 || exit $?
done
