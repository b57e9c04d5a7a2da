// waafle_genecaller's gene calls on the GPU (gfx950 / MI355X): hits of one contig group ->
// connected components of overlapping intervals -> merged genes (waafle_genecaller.py:107-170,
// main loop :199-233).  One wave per contig group (grid-stride), its intervals in LDS:
//
//   1. hits with scov_modified >= --min-scov become intervals [min(q), max(q)] with the hit's
//      strand (hits2ints :107-113, INode :455-466 of utils.py), compacted in file order;
//   2. a bitonic sort by (start, file position) -- Python's stable sort by start (:141);
//   3. edges i < j with calc_overlap >= --min-overlap (utils.py:487-500); the reference's
//      `break` on a disjoint j (:150-152) only skips pairs that cannot overlap, because j's
//      start is past i's stop, so the edge set is every overlapping pair;
//   4. components by hooking: each edge points the larger root at the smaller one
//      (atomicMin), pointer jumping, repeated until no edge joins two roots.  The final root
//      is the component's smallest sorted position -- the reference's "first unvisited"
//      inode (:155-158), which fixes the output order;
//   5. merge (merge_inodes :125-136): start of the root (the smallest start), max stop, and
//      the strand of the longest member, ties to "-" (sorted([len, strand])[-1]);
//   6. genes with stop - start + 1 >= --min-gene-length, in component order.
//
// --stranded is accepted and ignored, as upstream: `args.stranded == "on"` compares a bool
// with a string (waafle_genecaller.py:212-215), so strand never splits a group there.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "wf_internal.h"

namespace wf {

namespace {

constexpr int kGcNT = 64;

__global__ __launch_bounds__(kGcNT) void k_genecall(GcArgs A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int cap = A.cap;
  uint64_t* s_key = reinterpret_cast<uint64_t*>(smem);          // (start << 32 | position)
  int* s_lo = reinterpret_cast<int*>(s_key + cap);              // by file position
  int* s_hi = s_lo + cap;
  int* s_par = s_hi + cap;                                      // by sorted position
  int* s_stop = s_par + cap;
  int* s_best = s_stop + cap;                                   // len << 1 | minus
  int8_t* s_st = reinterpret_cast<int8_t*>(s_best + cap);
  __shared__ int s_flag;
  const int lane = threadIdx.x;
  for (int g = blockIdx.x; g < A.n_groups; g += gridDim.x) {
    const int64_t h0 = A.hit_off[g], h1 = A.hit_off[g + 1];
    // 1. filtered intervals, file order
    int m = 0;
    for (int64_t hb = h0; hb < h1; hb += kGcNT) {
      const int64_t h = hb + lane;
      const bool keep = h < h1 && A.scov[h] >= A.min_scov;
      const uint64_t bm = __ballot(keep);
      if (keep) {
        const int p = m + __popcll(bm & ((1ull << lane) - 1ull));
        if (p < cap) {
          const int a = A.qlo[h], b = A.qhi[h];
          s_lo[p] = min(a, b);
          s_hi[p] = max(a, b);
          s_st[p] = A.strand[h];
        }
      }
      m += __popcll(bm);
    }
    if (m > cap) {                                  // more intervals than the LDS holds
      if (lane == 0) { A.n_genes[g] = 0; A.status[g] = -4; }
      continue;
    }
    int n2 = 2;
    while (n2 < m) n2 <<= 1;
    __syncthreads();
    for (int t = lane; t < n2; t += kGcNT)
      s_key[t] = t < m ? ((uint64_t)(uint32_t)s_lo[t] << 32) | (uint32_t)t : ~0ull;
    __syncthreads();
    // 2. stable sort by start
    for (int k = 2; k <= n2; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = lane; i < (n2 >> 1); i += kGcNT) {
          const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1));
          const int hi = lo | j;
          const bool up = (lo & k) == 0;
          const uint64_t a = s_key[lo], b = s_key[hi];
          if ((a > b) == up) { s_key[lo] = b; s_key[hi] = a; }
        }
        __syncthreads();
      }
    }
    for (int t = lane; t < m; t += kGcNT) {
      const int p = (int)(uint32_t)s_key[t];
      const int len = s_hi[p] - s_lo[p] + 1;
      s_par[t] = t;
      s_stop[t] = s_hi[p];
      s_best[t] = (len << 1) | (s_st[p] == 1 ? 1 : 0);
    }
    __syncthreads();
    // 3-4. components over the overlap edges
    auto start_of = [&](int t) { return (int)(s_key[t] >> 32); };
    auto find = [&](int t) {
      while (s_par[t] != t) t = s_par[t];
      return t;
    };
    // --min-overlap <= 0: a disjoint pair scores int 0 >= threshold upstream, so every pair
    // is an edge (and the reference never breaks): one component
    if (!(A.min_overlap > 0.0)) {
      for (int t = lane; t < m; t += kGcNT) s_par[t] = 0;
      __syncthreads();
    }
    for (; A.min_overlap > 0.0;) {
      if (lane == 0) s_flag = 0;
      __syncthreads();
      for (int t = lane; t < m; t += kGcNT) {
        const int a1 = start_of(t), b1 = s_stop[t];
        for (int u = t + 1; u < m; ++u) {
          const int a2 = start_of(u);
          if (a2 > b1) break;                       // calc_overlap == 0 from here on
          const int b2 = s_stop[u];
          const int ov = min(b1, b2) - a2 + 1;
          const int den = min(b1 - a1 + 1, b2 - a2 + 1);
          if (!((double)ov / (double)den >= A.min_overlap)) continue;
          const int ra = find(t), rb = find(u);
          if (ra != rb) {
            atomicMin(&s_par[max(ra, rb)], min(ra, rb));
            s_flag = 1;
          }
        }
      }
      __syncthreads();
      for (int t = lane; t < m; t += kGcNT) s_par[t] = find(t);   // pointer jumping
      __syncthreads();
      if (!s_flag) break;
    }
    // 5. merge into the root
    for (int t = lane; t < m; t += kGcNT) {
      const int r = s_par[t];
      if (r != t) {
        atomicMax(&s_stop[r], s_stop[t]);
        atomicMax(&s_best[r], s_best[t]);
      }
    }
    __syncthreads();
    // 6. genes in root order
    int n_out = 0;
    for (int tb = 0; tb < m; tb += kGcNT) {
      const int t = tb + lane;
      bool emit = false;
      int a = 0, b = 0;
      if (t < m && s_par[t] == t) {
        a = start_of(t);
        b = s_stop[t];
        emit = (double)(b - a + 1) >= A.min_gene_length;
      }
      const uint64_t bm = __ballot(emit);
      if (emit) {
        const int64_t o = h0 + n_out + __popcll(bm & ((1ull << lane) - 1ull));
        A.gene_start[o] = a;
        A.gene_stop[o] = b;
        A.gene_strand[o] = (int8_t)(s_best[t] & 1);
      }
      n_out += __popcll(bm);
    }
    if (lane == 0) { A.n_genes[g] = n_out; A.status[g] = 0; }
    __syncthreads();
  }
}

}  // namespace

hipError_t launch_genecall(const GcArgs& a, int cus, hipStream_t s) {
  const size_t lds = (size_t)a.cap * (8 + 4 * 5 + 1);
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_genecall),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(16, (160 * 1024) / lds));
  const int grid = (int)std::min<int64_t>(a.n_groups, (int64_t)cus * per_cu);
  if (grid > 0) hipLaunchKernelGGL(k_genecall, dim3(grid), dim3(kGcNT), lds, s, a);
  return hipGetLastError();
}

}  // namespace wf
