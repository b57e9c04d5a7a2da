// Cross-lane primitives of one wave64 on gfx950 without the LDS crossbar.
//
// __shfl_xor / __shfl_up compile to ds_bpermute_b32: an LDS round trip per exchange, and a
// wave-wide scan or butterfly is six of them back to back.  Here every exchange is a VALU
// op: DPP row permutations for strides 1, 2, 4, 8 (quad_perm, row_half_mirror, row_mirror;
// strides 4 and 8 as two of them), and the CDNA4 permlane swaps for 16 and 32.
//
// Preconditions: every lane of the wave is active (the permutations read the source lane's
// register whatever its exec bit), and J is a power of two below 64.  tests/lanes/
// lanes_check.hip compares each primitive with __shfl_xor / a serial scan on the GPU.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

namespace wf {

constexpr int kDppQuadSwap1 = 0xB1;      // quad_perm [1,0,3,2]
constexpr int kDppQuadSwap2 = 0x4E;      // quad_perm [2,3,0,1]
constexpr int kDppQuadRev = 0x1B;        // quad_perm [3,2,1,0]
constexpr int kDppRowShr1 = 0x111;       // row_shr:n = 0x110 + n
constexpr int kDppRowMirror = 0x140;
constexpr int kDppRowHalfMirror = 0x141;
constexpr int kDppRowBcast15 = 0x142;
constexpr int kDppRowBcast31 = 0x143;

template <int Ctrl, int RowMask = 0xF, int BankMask = 0xF, bool BoundZero = false>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t old, uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, Ctrl, RowMask, BankMask, BoundZero);
}

// x of lane (lane ^ J)
template <int J>
__device__ __forceinline__ uint32_t xor_lanes(uint32_t x) {
  static_assert(J == 1 || J == 2 || J == 4 || J == 8 || J == 16 || J == 32, "stride");
  if constexpr (J == 1) {
    return dpp_u32<kDppQuadSwap1>(0u, x);
  } else if constexpr (J == 2) {
    return dpp_u32<kDppQuadSwap2>(0u, x);
  } else if constexpr (J == 4) {            // (i ^ 3) mirrored in its half row = i ^ 4
    return dpp_u32<kDppRowHalfMirror>(0u, dpp_u32<kDppQuadRev>(0u, x));
  } else if constexpr (J == 8) {            // half-row mirror, then row mirror = i ^ 8
    return dpp_u32<kDppRowMirror>(0u, dpp_u32<kDppRowHalfMirror>(0u, x));
  } else if constexpr (J == 16) {
    // odd rows of the first operand swap with even rows of the second: with both x, the
    // first comes back as rows (0,0,2,2) and the second as (1,1,3,3)
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (__lane_id() & 16) ? r[0] : r[1];
  } else {
    // the upper half of the first operand swaps with the lower half of the second
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return (__lane_id() & 32) ? r[0] : r[1];
  }
}
template <int J>
__device__ __forceinline__ int xor_lanes(int x) { return (int)xor_lanes<J>((uint32_t)x); }
template <int J>
__device__ __forceinline__ uint64_t xor_lanes(uint64_t x) {
  return (uint64_t)xor_lanes<J>((uint32_t)x) | ((uint64_t)xor_lanes<J>((uint32_t)(x >> 32)) << 32);
}
template <int J>
__device__ __forceinline__ long long xor_lanes(long long x) { return (long long)xor_lanes<J>((uint64_t)x); }
template <int J>
__device__ __forceinline__ double xor_lanes(double x) {
  return __longlong_as_double((long long)xor_lanes<J>((uint64_t)__double_as_longlong(x)));
}

// xor_lanes with a stride known after unrolling (a constant j folds the switch)
template <class T>
__device__ __forceinline__ T xor_lanes_rt(T x, int j) {
  switch (j) {
    case 1: return xor_lanes<1>(x);
    case 2: return xor_lanes<2>(x);
    case 4: return xor_lanes<4>(x);
    case 8: return xor_lanes<8>(x);
    case 16: return xor_lanes<16>(x);
    default: return xor_lanes<32>(x);
  }
}

// f(std::integral_constant<int, J>) for J = 32, 16, ..., 1 (the butterfly's strides)
template <class F>
__device__ __forceinline__ void each_stride(F f) {
  f(std::integral_constant<int, 32>{});
  f(std::integral_constant<int, 16>{});
  f(std::integral_constant<int, 8>{});
  f(std::integral_constant<int, 4>{});
  f(std::integral_constant<int, 2>{});
  f(std::integral_constant<int, 1>{});
}

// x of lane src (src wave-uniform): v_readlane, no LDS
__device__ __forceinline__ int lane_bcast(int x, int src) { return __builtin_amdgcn_readlane(x, src); }
__device__ __forceinline__ uint64_t lane_bcast(uint64_t x, int src) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, src) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), src) << 32);
}
__device__ __forceinline__ double lane_bcast(double x, int src) {
  return __longlong_as_double((long long)lane_bcast((uint64_t)__double_as_longlong(x), src));
}

// Butterfly over the whole wave: op(x, partner) at strides 32, 16, ..., 1; every lane ends
// with the same value when op is commutative and associative (sum, or, min, max).
template <class T, class Op>
__device__ __forceinline__ T wave_butterfly(T x, Op op) {
  x = op(x, xor_lanes<32>(x));
  x = op(x, xor_lanes<16>(x));
  x = op(x, xor_lanes<8>(x));
  x = op(x, xor_lanes<4>(x));
  x = op(x, xor_lanes<2>(x));
  x = op(x, xor_lanes<1>(x));
  return x;
}
__device__ __forceinline__ int wave_sum_dpp(int x) {
  return wave_butterfly(x, [](int a, int b) { return a + b; });
}
__device__ __forceinline__ long long wave_sum_dpp(long long x) {
  return wave_butterfly(x, [](long long a, long long b) { return a + b; });
}
__device__ __forceinline__ uint64_t wave_or_dpp(uint64_t x) {
  return wave_butterfly(x, [](uint64_t a, uint64_t b) { return a | b; });
}

// Exclusive prefix sum over the wave's lanes (lane order) and the total: an inclusive scan
// within each 16-lane row by row_shr 1, 2, 4, 8 (lanes shifted in from outside the row read
// 0), then row 15's sum broadcast into rows 1 and 3 and row 31's into rows 2 and 3.
__device__ __forceinline__ int wave_excl_scan_dpp(int v, int* total) {
  uint32_t x = (uint32_t)v;
  x += dpp_u32<kDppRowShr1 + 0, 0xF, 0xF, true>(0u, x);
  x += dpp_u32<kDppRowShr1 + 1, 0xF, 0xF, true>(0u, x);
  x += dpp_u32<kDppRowShr1 + 3, 0xF, 0xF, true>(0u, x);
  x += dpp_u32<kDppRowShr1 + 7, 0xF, 0xF, true>(0u, x);
  x += dpp_u32<kDppRowBcast15, 0xA, 0xF, false>(0u, x);
  x += dpp_u32<kDppRowBcast31, 0xC, 0xF, false>(0u, x);
  *total = __builtin_amdgcn_readlane((int)x, 63);
  return (int)x - v;
}

}  // namespace wf
