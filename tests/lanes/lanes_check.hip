// Checks the cross-lane primitives of wf_lanes.h against __shfl_xor / a serial scan on the
// GPU: prints one line per primitive and exits non-zero on a mismatch.
// Built by waafle_amd/build.py (tests/lanes/lanes_check), run by tests/test_gpu_lanes.py.
#include <hip/hip_runtime.h>
#include <cstdio>

#include "wf_lanes.h"

using namespace wf;

__global__ void k_check(unsigned* out) {
  const int lane = threadIdx.x;
  const unsigned x = 0x9E3779B9u * (unsigned)(lane + 1) ^ 0x5bd1e995u;
  out[0 * 64 + lane] = xor_lanes<1>(x) == __shfl_xor(x, 1, 64);
  out[1 * 64 + lane] = xor_lanes<2>(x) == __shfl_xor(x, 2, 64);
  out[2 * 64 + lane] = xor_lanes<4>(x) == __shfl_xor(x, 4, 64);
  out[3 * 64 + lane] = xor_lanes<8>(x) == __shfl_xor(x, 8, 64);
  out[4 * 64 + lane] = xor_lanes<16>(x) == __shfl_xor(x, 16, 64);
  out[5 * 64 + lane] = xor_lanes<32>(x) == __shfl_xor(x, 32, 64);
  const double d = (double)x * 1.25;
  out[6 * 64 + lane] = xor_lanes<32>(d) == __shfl_xor(d, 32, 64) && xor_lanes<4>(d) == __shfl_xor(d, 4, 64);
  const int v = (int)(x % 7u);
  int tot = 0;
  const int ex = wave_excl_scan_dpp(v, &tot);
  int ref = 0, rtot = 0;
  for (int i = 0; i < 64; ++i) {
    const int vi = __shfl(v, i, 64);
    if (i < lane) ref += vi;
    rtot += vi;
  }
  out[7 * 64 + lane] = ex == ref && tot == rtot;
  out[8 * 64 + lane] = wave_sum_dpp(v) == rtot;
  uint64_t m = 1ull << (lane % 37);
  uint64_t ro = 0;
  for (int i = 0; i < 64; ++i) ro |= __shfl(m, i, 64);
  out[9 * 64 + lane] = wave_or_dpp(m) == ro;
}

int main() {
  unsigned* d = nullptr;
  const int n = 10;
  if (hipMalloc(&d, n * 64 * sizeof(unsigned)) != hipSuccess) return 2;
  hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, d);
  unsigned h[n * 64];
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  const char* names[n] = {"xor1", "xor2", "xor4", "xor8", "xor16", "xor32", "xor_f64", "excl_scan",
                          "sum", "or64"};
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    int ok = 1;
    for (int l = 0; l < 64; ++l) ok &= h[i * 64 + l] == 1u;
    printf("%-12s %s\n", names[i], ok ? "ok" : "MISMATCH");
    bad += !ok;
  }
  (void)hipFree(d);
  return bad ? 1 : 0;
}
