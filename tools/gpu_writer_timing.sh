# split::Writer time breakdown (tools/writer_timing.py): the default build and a variant
# (VARIANT), twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=${VARIANT:-bs_amd/variants/lib_pre_data.so}
for r in 1 2; do
  echo "== default" >> gpurun_out/writer_timing.log
  timeout -k 10 200 python -u tools/writer_timing.py >> gpurun_out/writer_timing.log 2>&1 || exit $?
  echo "== $V" >> gpurun_out/writer_timing.log
  BSG_LIB_PATH=$V BSG_LIB_PARTIAL=1 timeout -k 10 200 python -u tools/writer_timing.py >> gpurun_out/writer_timing.log 2>&1 || exit $?
done
