# A/B of the host-memory paths between the current library and a variant (tools/writer_ab.py),
# then the first-use costs with the current library.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python tools/writer_ab.py bs_amd/libbsgpu.so ${AB_VARIANTS:-bs_amd/variants/libbsgpu_pre_ring.so} > gpurun_out/writer_ab.log 2>&1 || exit $?
timeout -k 10 600 python tools/first_writer.py cold1m cold1m cold1m first4g first4g > gpurun_out/first_writer.log 2>&1 || exit $?
