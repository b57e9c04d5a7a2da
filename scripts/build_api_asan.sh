# Host-sanitizer build of the C-ABI driver (tests/sanitize/api_driver.cpp): host code of
# wf_api.cpp and the .hip files under ASan + UBSan, device code as in the product build.
# Cross-compiles here (no GPU needed); scripts/gpu_r2.sh runs the binary on the GPU box.
set -eu
cd "$(dirname "$0")/.."
OUT=tests/sanitize/api_driver_asan
H="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer -Xarch_host -fno-sanitize-recover=all"
F="--offload-arch=gfx950 -O1 -g -ffp-contract=off -std=c++17 -Iinclude -Iwaafle_amd/csrc"
objs=""
for s in waafle_amd/csrc/wf_staged.hip waafle_amd/csrc/wf_fast.hip waafle_amd/csrc/wf_genecall.hip waafle_amd/csrc/wf_junctions.hip waafle_amd/csrc/wf_api.cpp tests/sanitize/api_driver.cpp; do
  o=/tmp/asan_$(basename $s).o
  /opt/rocm/bin/hipcc $F $H -c $s -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fsanitize=address,undefined $objs -o $OUT
echo built $OUT
