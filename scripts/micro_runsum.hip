// Micro-benchmark of the one-run closed forms (pw_run_sum, pw_const_sum, one_run_mean) on
// the device: shader clocks per call, one wave per SIMD and four, with lanes drawn like the
// synthetic decoy runs (locus 250-1500 sites, runs covering 80-100% at a random offset).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I include -I waafle_amd/csrc \
//         scripts/micro_runsum.hip -o scripts/micro_runsum && scripts/micro_runsum
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
#include <algorithm>
#include "wf_device.h"

using namespace wf;

// The previous pw_run_sum (three divergent leaf evaluations), kept here as the A/B and
// bit-exactness reference of the current one.
__device__ __forceinline__ double pw_run_sum_v1(int n, int lo, int hi, double v) {
  lo = max(lo, 0);
  hi = min(hi, n);
  if (hi <= lo) return 0.0;
  const int a0 = n >> 4;
  int K = 0, m = n;
  unsigned sel = 0;
  while (m > 128) {
    const int a = m >> 4;
    sel |= (a != (a0 >> K) ? 1u : 0u) << K;
    m -= 8 * a;
    ++K;
  }
  int Db = 0, Dmax = -1, xB = 0, xC = 0;
  bool need16 = false;
  if (K > 0) {
    Db = max(0, 28 - __clz(a0));
    Dmax = max(K - 1, Db);
    xB = a0 >> Db;
    xC = Dmax == Db + 1 ? a0 >> (Db + 1) : 0;
    need16 = Db >= 1 && (a0 >> (Db - 1)) == 16;
  }
  // a node: start s, size z, spine (kind 0) or pair node of size 8 * (B_{t-1} + cls), depth t
  struct Nd { int s, z, kind, cls, t; };
  auto child = [&](const Nd& x, bool right) -> Nd {
    if (x.kind == 0) {
      const int nl = 8 * (x.z >> 4);
      return right ? Nd{x.s + nl, x.z - nl, 0, 0, x.t + 1} : Nd{x.s, nl, 1, (int)((sel >> x.t) & 1u), x.t + 1};
    }
    const int xx = x.z >> 3, xl = xx >> 1, Bt = a0 >> x.t;
    return right ? Nd{x.s + 8 * xl, 8 * (xx - xl), 1, (xx - xl) - Bt, x.t + 1} : Nd{x.s, 8 * xl, 1, xl - Bt, x.t + 1};
  };
  Nd nd{0, n, 0, 0, 0};
  bool whole = false;
  for (;;) {                                         // down to the split node
    if (lo <= nd.s && hi >= nd.s + nd.z) { whole = true; break; }
    if (nd.z <= 128) return run_leaf(lo, hi, v, nd.s, nd.z);
    const int nl = nd.kind == 0 ? 8 * (nd.z >> 4) : 8 * ((nd.z >> 3) >> 1);
    if (hi <= nd.s + nl) nd = child(nd, false);
    else if (lo >= nd.s + nl) nd = child(nd, true);
    else break;
  }
  // the two paths: terminal depth / type (0 whole spine, 1 whole pair, 2 leaf) / class /
  // leaf sum, and per depth: a whole sibling to add, is it the spine, its class
  struct Path { int tu, ty, tc; unsigned ev, evk, evc; double lv; };
  auto walk = [&](bool suffix) -> Path {
    Path q{0, 0, 0, 0u, 0u, 0u, 0.0};
    Nd x = child(nd, !suffix);
    for (;;) {
      if (suffix ? lo <= x.s : hi >= x.s + x.z) { q.tu = x.t; q.ty = x.kind; q.tc = x.cls; return q; }
      if (x.z <= 128) {
        q.tu = x.t; q.ty = 2;
        q.lv = suffix ? run_leaf(lo, x.s + x.z, v, x.s, x.z) : run_leaf(x.s, hi, v, x.s, x.z);
        return q;
      }
      const Nd L = child(x, false), R = child(x, true);
      if (suffix ? lo < R.s : hi > R.s) {
        const Nd& w = suffix ? R : L;                // the whole sibling
        q.ev |= 1u << w.t;
        q.evk |= (w.kind == 0 ? 1u : 0u) << w.t;
        q.evc |= (unsigned)w.cls << w.t;
        x = suffix ? L : R;
      } else {
        x = suffix ? R : L;
      }
    }
  };
  Path p0{0, 0, 0, 0u, 0u, 0u, 0.0}, p1{0, 0, 0, 0u, 0u, 0u, 0.0};
  if (!whole) {
    p0 = walk(true);
    p1 = walk(false);
  }
  const int mL = m < 8 ? m : m >> 3;
  const int imax = max(max(xB, mL), need16 ? 16 : 0);
  double t = 0.0, sB = 0.0, sC = 0.0, sL = 0.0;
  for (int i = 1; i <= imax; ++i) {
    t += v;
    sB = i == xB ? t : sB;
    sC = i == xC ? t : sC;
    sL = i == mL ? t : sL;
  }
  double R;                                          // the spine below the current depth
  if (m < 8) {
    R = sL;
  } else {
    R = 8.0 * sL;
    for (int x = 0; x < (m & 7); ++x) R += v;
  }
  double q0 = 0.0, q1 = 0.0, acc0 = 0.0, acc1 = 0.0;
  for (int d = Dmax; d >= -1; --d) {                 // tree depth u = d + 1, bottom up
    const int u = d + 1;
    if (d >= 0) {
      const int B = a0 >> d;
      if (d >= Db) {
        const double sd = d == Db ? sB : sC;
        q0 = 8.0 * sd;
        q1 = 8.0 * (sd + v);
      } else {
        const double c0 = q0, c1 = q1;
        q0 = (B & 1) ? c0 + c1 : c0 + c0;
        q1 = (B & 1) ? c1 + c1 : c0 + c1;
        if (B == 16) q0 = 8.0 * t;
      }
    }
    if (whole) {
      if (u == nd.t) return nd.kind == 0 ? R : (nd.cls ? q1 : q0);
    } else {
      if (u == p0.tu) acc0 = p0.ty == 2 ? p0.lv : (p0.ty == 0 ? R : (p0.tc ? q1 : q0));
      if (u <= p0.tu && ((p0.ev >> u) & 1u))
        acc0 = acc0 + (((p0.evk >> u) & 1u) ? R : (((p0.evc >> u) & 1u) ? q1 : q0));
      if (u == p1.tu) acc1 = p1.ty == 2 ? p1.lv : (p1.ty == 0 ? R : (p1.tc ? q1 : q0));
      if (u <= p1.tu && ((p1.ev >> u) & 1u))
        acc1 = (((p1.evc >> u) & 1u) ? q1 : q0) + acc1;
      if (u == nd.t + 1) return acc0 + acc1;
    }
    if (d >= 0 && d < K) R = (((sel >> d) & 1u) ? q1 : q0) + R;
  }
  return 0.0;                                        // (not reached)
}


__global__ void k_exact(const int* len, const int* lo, const int* hi, const double* v, int n, unsigned long long* bad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double a = pw_run_sum(len[i], lo[i], hi[i], v[i]), b = pw_run_sum_v1(len[i], lo[i], hi[i], v[i]);
  if (__double_as_longlong(a) != __double_as_longlong(b)) atomicAdd(bad, 1ull);
}

template <int MODE>
__global__ __launch_bounds__(64) void k_micro(const int* len, const int* lo, const int* hi, const double* v, int reps,
                                              double* out, unsigned long long* cyc) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  int n = len[i], a = lo[i], b = hi[i];
  double x = v[i], acc = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    double y;
    if (MODE == 0) y = pw_run_sum(n, a, b, x);
    else if (MODE == 1) y = pw_const_sum(n, x);
    else if (MODE == 2) y = run_leaf(a & 127, (b & 127) + 1, x, 0, 128);
    else y = pw_run_sum_v1(n, a, b, x);
    acc += y;
    x = x + (y > 1e300 ? 1.0 : 0.0);                 // (a dependence: no hoisting)
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[i] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int waves_max = 256 * 4 * 4, n = waves_max * 64, reps = 64;
  std::mt19937 rng(7);
  std::vector<int> len(n), lo(n), hi(n);
  std::vector<double> v(n);
  for (int i = 0; i < n; ++i) {
    len[i] = 250 + rng() % 1250;
    const int a = (int)(len[i] * (0.8 + 0.2 * (rng() % 1000) / 1000.0));
    lo[i] = rng() % (len[i] - a + 1);
    hi[i] = lo[i] + a;
    v[i] = 0.7 + 0.2 * (rng() % 1000) / 1000.0;
  }
  int *dl, *dlo, *dhi;
  double *dv, *dout;
  unsigned long long* dc;
  hipMalloc(&dl, n * 4); hipMalloc(&dlo, n * 4); hipMalloc(&dhi, n * 4);
  hipMalloc(&dv, n * 8); hipMalloc(&dout, n * 8); hipMalloc(&dc, waves_max * 8);
  hipMemcpy(dl, len.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dlo, lo.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dhi, hi.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dv, v.data(), n * 8, hipMemcpyHostToDevice);
  {
    // bit-exactness of pw_run_sum against the previous form: every length below 8192 with
    // random runs (whole, prefix, suffix, short, any) and the decoy-like lanes above
    std::vector<int> L2, A2, B2;
    std::vector<double> V2;
    for (int len_ = 1; len_ < 8192; ++len_)
      for (int k = 0; k < 24; ++k) {
        int a = 0, b = len_;
        const int kind = k % 5;
        if (kind == 1) a = rng() % len_;
        else if (kind == 2) b = 1 + rng() % len_;
        else if (kind == 3) { a = rng() % len_; b = std::min(len_, a + 1 + (int)(rng() % 9)); }
        else if (kind == 4) { a = rng() % len_; b = a + 1 + rng() % (len_ - a); }
        L2.push_back(len_); A2.push_back(a); B2.push_back(b);
        V2.push_back(0.05 + 0.95 * (rng() % 100000) / 100000.0);
      }
    const int m = (int)L2.size();
    int *el, *ea, *eb; double* ev; unsigned long long* ebad;
    (void)hipMalloc(&el, m * 4); (void)hipMalloc(&ea, m * 4); (void)hipMalloc(&eb, m * 4);
    (void)hipMalloc(&ev, m * 8); (void)hipMalloc(&ebad, 8);
    (void)hipMemcpy(el, L2.data(), m * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(ea, A2.data(), m * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(eb, B2.data(), m * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(ev, V2.data(), m * 8, hipMemcpyHostToDevice);
    (void)hipMemset(ebad, 0, 8);
    hipLaunchKernelGGL(k_exact, dim3((m + 255) / 256), dim3(256), 0, 0, el, ea, eb, ev, m, ebad);
    unsigned long long bad = 0;
    (void)hipMemcpy(&bad, ebad, 8, hipMemcpyDeviceToHost);
    printf("pw_run_sum vs previous form: %d cases, %llu differ\n", m, bad);
  }
  const char* names[4] = {"pw_run_sum", "pw_const_sum", "run_leaf(128)", "pw_run_sum (previous)"};
  for (int mode = 0; mode < 4; ++mode) {
    for (int per_simd : {1, 4}) {
      const int waves = 256 * 4 * per_simd;
      for (int warm = 0; warm < 2; ++warm) {
        if (mode == 0) hipLaunchKernelGGL(k_micro<0>, dim3(waves), dim3(64), 0, 0, dl, dlo, dhi, dv, reps, dout, dc);
        if (mode == 1) hipLaunchKernelGGL(k_micro<1>, dim3(waves), dim3(64), 0, 0, dl, dlo, dhi, dv, reps, dout, dc);
        if (mode == 2) hipLaunchKernelGGL(k_micro<2>, dim3(waves), dim3(64), 0, 0, dl, dlo, dhi, dv, reps, dout, dc);
        if (mode == 3) hipLaunchKernelGGL(k_micro<3>, dim3(waves), dim3(64), 0, 0, dl, dlo, dhi, dv, reps, dout, dc);
      }
      hipDeviceSynchronize();
      std::vector<unsigned long long> c(waves);
      hipMemcpy(c.data(), dc, waves * 8, hipMemcpyDeviceToHost);
      double s = 0;
      for (auto x : c) s += (double)x;
      // s_memtime counts at the constant 100 MHz reference clock on gfx9? report raw ticks too
      printf("%-16s %d wave/SIMD: %.1f ticks per call per wave\n", names[mode], per_simd, s / waves / reps);
    }
  }
  return 0;
}
