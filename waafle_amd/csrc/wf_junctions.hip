// waafle_junctions on MI355X (gfx950): per-site read-pair coverage and gene-gene junction
// support for a batch of contigs, replacing the per-pair loop of
// waafle_junctions.py:428-451 and evaluate_contig :292-316.
//
//   k_jn_cover   thread per concordant read pair: coverage[L:R+1] += 1 as two difference
//                marks (integer atomics, so the result is order independent), and the pair's
//                hit loci (find_hit_loci :277-286): a junction between start-sorted loci j
//                and j+1 gains one pair when the pair hits both
//   device scans difference marks -> coverage, coverage -> prefix sums (int64); each
//                contig owns len + 1 slots (the last one is a sentinel that takes the -1 of
//                reads running past the contig end), so one global scan serves every contig
//   k_jn_eval    thread per junction: gene and junction coverage means from the prefix sums
//                (integer sums are exact, so np.mean's pairwise order does not matter), the
//                ratio in the reference's float order
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <string>

#include "wf_internal.h"

namespace wf {
namespace {

// Python slice [a:b] on a sequence of length n -> [lo, hi) with lo <= hi
__device__ __forceinline__ void py_slice(int64_t a, int64_t b, int64_t n, int64_t& lo, int64_t& hi) {
  if (a < 0) { a += n; if (a < 0) a = 0; } else if (a > n) a = n;
  if (b < 0) { b += n; if (b < 0) b = 0; } else if (b > n) b = n;
  lo = a;
  hi = b > a ? b : a;
}

// utils.calc_overlap(a1, a2, b1, b2, normalize=False) (utils.py:487-500)
__device__ __forceinline__ int64_t overlap_sites(int64_t a1, int64_t a2, int64_t b1, int64_t b2) {
  if (a1 > a2) { const int64_t t = a1; a1 = a2; a2 = t; }
  if (b1 > b2) { const int64_t t = b1; b1 = b2; b2 = t; }
  if (b1 > a2 || a1 > b2) return 0;
  return min(a2, b2) - max(a1, b1) + 1;
}

__global__ void k_jn_cover(const JnArgs A) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= A.n_pairs) return;
  const int c = A.pair_contig[p];
  const int64_t s1 = A.m1_start[p], e1 = A.m1_end[p], s2 = A.m2_start[p], e2 = A.m2_end[p];
  // coverage (waafle_junctions.py:432-436): L = min(coords) - 1, R = max(coords) - 1
  const int64_t L = min(min(s1, e1), min(s2, e2)) - 1, R = max(max(s1, e1), max(s2, e2)) - 1;
  const int64_t n = A.site_off[c + 1] - A.site_off[c] - 1;       // contig length
  int64_t lo, hi;
  py_slice(L, R + 1, n, lo, hi);
  if (hi > lo) {
    atomicAdd(&A.diff[A.site_off[c] + lo], 1);
    atomicAdd(&A.diff[A.site_off[c] + hi], -1);                    // hi <= n: sentinel slot
  }
  // hit loci (find_hit_loci, :277-286) in start order; a junction (j, j+1) is supported when
  // both flanking loci are hit (identical codes have identical coordinates, so the code set
  // of the reference and the per-locus flags agree)
  const int64_t l0 = A.loc_off[c], l1 = A.loc_off[c + 1];
  const int64_t rmax = max(max(s1, e1), max(s2, e2));
  bool prev = false;
  int64_t first = -1;
  uint64_t mask = 0;
  for (int64_t k = l0; k < l1; ++k) {
    const int64_t a1 = A.loc_start[k], a2 = A.loc_end[k];
    if (A.loc_forward && a1 > rmax) break;       // sorted by start, start <= end: no
                                                 // later locus reaches the pair
    const bool hit = overlap_sites(a1, a2, s1, e1) >= A.min_sites ||
                     overlap_sites(a1, a2, s2, e2) >= A.min_sites;
    if (hit && prev) atomicAdd(&A.junction_hits[k - 1], 1);
    if (hit && A.locus_hits) atomicAdd(&A.locus_hits[k], 1);
    if (hit) {                                   // the pair's hit set (gene-pair hits)
      if (first < 0) first = k;
      if (k - first < 64) mask |= 1ull << (k - first);
      else if (A.pair_first) atomicAdd(A.overflow, 1u);
    }
    prev = hit;
  }
  if (A.pair_first) {
    A.pair_first[p] = first;
    A.pair_mask[p] = mask;
  }
}

__device__ __forceinline__ double range_mean(const JnArgs& A, int c, int64_t a, int64_t b) {
  // np.mean(coverage[a:b]) on the contig's array; nan for an empty slice
  const int64_t base = A.site_off[c], n = A.site_off[c + 1] - base - 1;
  int64_t lo, hi;
  py_slice(a, b, n, lo, hi);
  if (hi <= lo) return __builtin_nan("");
  const int64_t s = A.prefix[base + hi - 1] - (base + lo > 0 ? A.prefix[base + lo - 1] : 0);
  return (double)s / (double)(hi - lo);
}

__global__ void k_jn_eval(const JnArgs A) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= A.n_loci) return;
  const int c = A.loc_contig[j];
  if (j + 1 >= A.loc_off[c + 1]) return;                          // last locus of its contig
  const int64_t s1 = A.loc_start[j], e1 = A.loc_end[j], s2 = A.loc_start[j + 1], e2 = A.loc_end[j + 1];
  const int64_t gap = s2 - e1 - 1;
  const double cov1 = range_mean(A, c, s1 - 1, e1);
  const double cov2 = range_mean(A, c, s2 - 1, e2);
  const double covj = gap <= 0 ? 0.0 : range_mean(A, c, e1 - 1, s2);
  const double mean = (cov1 + cov2) / 2.0;                        // np.mean of the two
  A.cov1[j] = cov1;
  A.cov2[j] = cov2;
  A.covj[j] = covj;
  A.ratio[j] = covj / (mean + 1e-6);
}

}  // namespace

#define JN_TRY(x)                                                                       \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) { *err = std::string(#x) + ": " + hipGetErrorString(e_); return -2; } \
  } while (0)

int junctions_run(const JnArgs& a, void* tmp, size_t tmp_bytes, hipStream_t s, std::string* err) {
  const int64_t S = a.n_sites;
  if (S <= 0) return 0;
  JN_TRY(hipMemsetAsync(a.diff, 0, (size_t)S * sizeof(int32_t), s));
  JN_TRY(hipMemsetAsync(a.junction_hits, 0, (size_t)std::max<int64_t>(a.n_loci, 1) * sizeof(int32_t), s));
  if (a.locus_hits)
    JN_TRY(hipMemsetAsync(a.locus_hits, 0, (size_t)std::max<int64_t>(a.n_loci, 1) * sizeof(int32_t), s));
  if (a.pair_first) JN_TRY(hipMemsetAsync(a.overflow, 0, sizeof(unsigned), s));
  if (a.n_pairs > 0)
    hipLaunchKernelGGL(k_jn_cover, dim3((unsigned)((a.n_pairs + 255) / 256)), dim3(256), 0, s, a);
  JN_TRY(hipGetLastError());
  size_t need = tmp_bytes;
  // marks -> coverage: the running sum returns to 0 at every contig's sentinel slot, so int32
  // accumulation is exact; coverage -> prefix sums in int64
  JN_TRY(hipcub::DeviceScan::InclusiveSum(tmp, need, a.diff, a.coverage, (int)S, s));
  need = tmp_bytes;
  JN_TRY(hipcub::DeviceScan::InclusiveSum(tmp, need, a.coverage, a.prefix, (int)S, s));
  if (a.n_loci > 0)
    hipLaunchKernelGGL(k_jn_eval, dim3((unsigned)((a.n_loci + 255) / 256)), dim3(256), 0, s, a);
  JN_TRY(hipGetLastError());
  return 0;
}

size_t junctions_tmp_bytes(int64_t n_sites) {
  size_t t1 = 0, t2 = 0;
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, t1, (const int32_t*)nullptr, (int64_t*)nullptr,
                                         (int)std::max<int64_t>(n_sites, 1), (hipStream_t)0);
  (void)hipcub::DeviceScan::InclusiveSum(nullptr, t2, (const int64_t*)nullptr, (int64_t*)nullptr,
                                         (int)std::max<int64_t>(n_sites, 1), (hipStream_t)0);
  return std::max(t1, t2);
}

}  // namespace wf
