# Builds libbsgpu variants with different k_sha tier thresholds / waves per workgroup into
# bs_amd/variants/ (experiments; the default build is bs_amd/libbsgpu.so).
set -e
cd "$(dirname "$0")/.."
mkdir -p bs_amd/variants
SRC="bs_amd/csrc/bsgpu_kernels.hip bs_amd/csrc/bsgpu_host.cpp bs_amd/csrc/bs_split.cpp bs_amd/csrc/bs_filestore.cpp"
build() {  # name, extra flags
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-value -Wno-unused-result $2 -o bs_amd/variants/lib_$1.so $SRC &
}
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  build "$name" "$flags"
done
wait
ls -la bs_amd/variants
