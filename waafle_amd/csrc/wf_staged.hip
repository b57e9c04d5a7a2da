// Staged form of the contig-scoring path (gfx950 / MI355X).  Instead of one workgroup
// carrying a contig through every phase (wf_kernels.hip), each phase is a flat kernel over
// all contigs' items, so every phase fills the chip at its own natural granularity:
//
//   contigs     k_att_contig<0>                workgroup per contig, thread per hit: attached
//                                              loci counted (orgscorer.py:359-369)
//               device exclusive scan          -> attachment offsets per contig
//               k_att_contig<1>                site ranges (:371-382), annotation winners
//                                              in LDS (:383-392)
//   per level   k_sort_contig                  per-contig LDS sort of (contig rank, clade,
//                                              locus) keys (device radix sort for huge
//                                              contigs) -> segments = equal keys (:394-406)
//               k_seg_flags + scan + k_segs    segment boundaries
//               k_seg_rec                      thread per one-run segment: exact mean
//               k_leaf + k_seg_combine         lane per numpy leaf, thread per segment: exact
//                                              mean of the other segments
//               k_one                          wave per contig: explain_one (+ meld_one)
//               k_decide / k_decide_big        workgroup per contig: maxes, weak loci,
//                                              explain_one/two, melds, LGT filters
//                                              (decide_level, shared with the fused form);
//                                              raised contigs re-keyed to parents (:431-445)
//
// The numpy pairwise-sum leaf tables depend only on the length of a buffer (<= 8192), so
// they are generated once per context into a device table (k_lut_*), with the same
// generator the fused kernels use.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <string>
#include <vector>

#include "wf_device.h"

namespace wf {

namespace {

__device__ __forceinline__ int upper_index(const int64_t* off, int n, int64_t x) {
  // largest c in [0, n) with off[c] <= x  (off is non-decreasing, off[0] = 0)
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= x) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ int lower_bound_i32(const int32_t* a, int n, int x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Counts of the current level: from the host (kernel arguments) when it knows them, else
// from the previous level's device counter word (rank slots << 40 | attachments) -- the
// pipelined levels (staged_score) enqueue a level before the host has read that word.
__device__ __forceinline__ void lvl_counts(const SArgs& S, int& n_act, int64_t& n_keys) {
  if (S.in_counts) {
    const unsigned long long v = *S.in_counts;
    n_act = (int)(v >> 40);
    n_keys = (int64_t)(v & ((1ull << 40) - 1));
  }
}

__device__ __forceinline__ int seg_count(const SArgs& S, int64_t n_keys) {
  return n_keys > 0 ? S.seg_id[n_keys - 1] : 0;
}


// ---- numpy leaf tables by buffer length ------------------------------------------------
__global__ void k_lut_count(int32_t* cnt) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n > kNpyBuf) return;
  cnt[n] = n == 0 ? 0 : gen_leaves(0, n, nullptr);
}
__global__ void k_lut_fill(const int32_t* off, int4* lut) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n < 1 || n > kNpyBuf) return;
  gen_leaves(0, n, lut + off[n]);
}

// ---- contigs, hits, attachments ----------------------------------------------------------
__global__ void k_init(const KArgs K) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= K.n_contigs) return;
  K.call[c] = WF_CALL_UNCLASSIFIED;
  K.crit[c] = 0.0; K.rank[c] = 0.0; K.c1[c] = -1; K.c2[c] = -1; K.dir[c] = 0;
  K.iters[c] = 0; K.nm1[c] = 0; K.nm2[c] = 0; K.pair_evals[c] = 0; K.status[c] = 0;
  K.need[c] = 0;
  if (K.ppot) K.ppot[c] = 0;
}

// Hits -> attachments, one workgroup per contig (grid-stride).  The contig's loci are
// staged in LDS; hits are taken in chunks of kAttNT (one thread each, the contig's loci in
// GFF order), so attachments come out in (hit, locus) order -- the order the reference
// paints sites in (orgscorer.py:359-382).  Pass 0 only counts (attachments, a leaf bound
// and the largest contig); pass 1 writes them at the contig's offset and does the
// annotation transfer (orgscorer.py:383-392) for the contig's loci in LDS.
constexpr int kAttNT = 64;       // one wave per contig: many contigs in flight ...
constexpr int kAttNTBig = 512;   // ... or 8 when the batch's contigs have thousands of hits (the
constexpr int kAttBigHits = 2048;   // cfg5 stress shape: one wave stepped ~80 dependent chunks)
constexpr int kAttLoc = 128;      // loci staged in LDS (more: read from HBM)

struct LocView {
  int lo, len, st;
};

template <int PASS, int NT>
// (S_arg first: the per-contig loop re-reads the argument block through kernarg_fresh)
__global__ __launch_bounds__(NT) void k_att_contig(const SArgs S_arg, int64_t* ccnt,
                                                       int64_t* cleaves, unsigned long long* cmax,
                                                       const int32_t* list, int n_list) {
  __shared__ int s_lo[kAttLoc], s_len[kAttLoc], s_nl[kAttLoc];
  __shared__ int8_t s_st[kAttLoc];
  __shared__ unsigned long long s_best[kAnnSlots];
  __shared__ int s_hit[kAnnSlots];
  __shared__ int s_scan[NT / 64];
  __shared__ long long s_red[2][NT / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = blockIdx.x; i < n_list; i += gridDim.x) {
    const SArgs& S = kernarg_fresh<SArgs>(S_arg);
    const KArgs& K = S.k;
    const DevParams& P = K.p;
    const int c = list ? list[i] : i;               // list: the contigs k_fast handed over
    const int64_t h0 = K.hit_off[c], h1 = K.hit_off[c + 1];
    const int64_t l0 = K.loc_off[c];
    const int G = (int)(K.loc_off[c + 1] - l0);
    const bool lds_loc = G <= kAttLoc;
    if (lds_loc)
      for (int g = tid; g < G; g += NT) {
        const int a = K.lstart[l0 + g], b = K.lend[l0 + g];
        s_lo[g] = min(a, b);
        const int len = max(a, b) - min(a, b) + 1;
        s_len[g] = len;
        s_st[g] = K.lstrand[l0 + g];
        if (PASS == 0)
          s_nl[g] = (len / kNpyBuf) * (S.lut_off[kNpyBuf + 1] - S.lut_off[kNpyBuf]) +
                    (S.lut_off[len % kNpyBuf + 1] - S.lut_off[len % kNpyBuf]);
      }
    const int ns = K.n_sys;
    const bool hkey = K.hkey != nullptr && ns <= 6;  // (the key holds systems 0-5)
    const bool lds_ann = PASS == 1 && (int64_t)G * ns <= kAnnSlots;
    if (lds_ann)
      for (int i = tid; i < G * ns; i += NT) { s_best[i] = 0ull; s_hit[i] = -1; }
    __syncthreads();
    auto locus = [&](int g) -> LocView {
      if (lds_loc) return LocView{s_lo[g], s_len[g], s_st[g]};
      const int a = K.lstart[l0 + g], b = K.lend[l0 + g];
      return LocView{min(a, b), max(a, b) - min(a, b) + 1, K.lstrand[l0 + g]};
    };
    // loci ascending and disjoint (the usual GFF) with min_overlap > 0: a hit attaches only to
    // loci it overlaps, a run found by binary search (the wave kernels' rule) instead of a
    // test against every locus -- O(H log G) rather than O(H G) for the cfg5 stress contigs
    bool ordered = lds_loc && P.min_overlap > 0.0;
    if (ordered) {
      bool bad = false;
      for (int g = 1 + tid; g < G; g += NT) bad = bad || s_lo[g] <= s_lo[g - 1] + s_len[g - 1] - 1;
      ordered = !__syncthreads_or(bad);
    }
    // the loci hit h attaches to, in GFF order: f(g, L) for each
    auto each_locus = [&](int qlo, int qhi, int hs, auto f) {
      if (ordered) {
        int g = 0;                                   // first locus ending at or after qlo
        for (int k = 64; k > 0; k >>= 1)
          if (g + k <= G && s_lo[g + k - 1] + s_len[g + k - 1] - 1 < qlo) g += k;
        for (; g < G; ++g) {
          const LocView L{s_lo[g], s_len[g], s_st[g]};
          if (L.lo > qhi) break;
          if (attaches(P, qlo, qhi, hs, L.lo, L.len, L.st)) f(g, L);
        }
        return;
      }
      for (int g = 0; g < G; ++g) {
        const LocView L = locus(g);
        if (attaches(P, qlo, qhi, hs, L.lo, L.len, L.st)) f(g, L);
      }
    };
    long long n_tot = 0, nl_tot = 0;
    int64_t base = PASS == 1 ? S.catt_off[c] : 0;
    for (int64_t hb = h0; hb < h1; hb += NT) {
      const int64_t h = hb + tid;
      int n = 0;
      long long nl = 0;
      int qlo = 0, qhi = 0, hs = 0, clade = 0;
      double sc = 0.0;
      uint32_t m = 0u;
      bool scov_ok = false;
      if (h < h1) {                                 // every field of the hit in one round of loads
        qlo = K.qlo[h]; qhi = K.qhi[h];
        if (PASS == 1) sc = K.score[h];
        if (hkey) {                                 // the packed word: 20 B a hit instead of 33
          const uint32_t k = K.hkey[h];
          scov_ok = (k & kKeyScov) != 0u;
          hs = P.stranded && (k & kKeyMinus) ? 1 : 0;
          clade = (int)(k & kKeyTaxon);
          m = k >> kKeySys;
        } else {
          scov_ok = K.scov[h] >= P.min_scov;
          hs = P.stranded ? K.hstrand[h] : 0;
          if (PASS == 1) {
            clade = K.taxon[h];
            m = ns > 0 ? K.sysmask[h] : 0u;
          }
        }
      }
      const bool live = h < h1 && scov_ok;
      if (live) {
        each_locus(qlo, qhi, hs, [&](int g, const LocView& L) {
          ++n;
          if (PASS == 0)
            nl += lds_loc ? s_nl[g]
                          : (L.len / kNpyBuf) * (S.lut_off[kNpyBuf + 1] - S.lut_off[kNpyBuf]) +
                                (S.lut_off[L.len % kNpyBuf + 1] - S.lut_off[L.len % kNpyBuf]);
        });
      }
      if (PASS == 0) {
        n_tot += n;
        nl_tot += nl;
        continue;
      }
      // exclusive scan of n over the chunk (hit order)
      int x = n;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      if (lane == 63) s_scan[w] = x;
      __syncthreads();
      int wbase = 0, total = 0;
#pragma unroll
      for (int i = 0; i < NT / 64; ++i) {
        wbase += i < w ? s_scan[i] : 0;
        total += s_scan[i];
      }
      __syncthreads();
      int64_t o = base + wbase + x - n;
      base += total;
      if (n == 0) continue;
      for (int j = 0; j < P.jump; ++j) clade = K.parent[clade];   // orgscorer.py:955-957
      const bool ann = m != 0 && sc >= P.annot_ref;
      each_locus(qlo, qhi, hs, [&](int g, const LocView& L) {
        const int h1s = max(0, qlo - L.lo);
        const int h2s = min(L.len - 1, qhi - L.lo);
        const int start = min(h1s, L.len);
        int stop = h2s + 1;                        // site[h1:h2+1], python slice rules
        if (stop < 0) { stop += L.len; if (stop < 0) stop = 0; }
        S.att_lo[o] = start;
        S.att_hi[o] = stop;                        // empty when stop <= start
        S.att_loc[o] = g;
        S.att_clade[o] = clade;
        S.att_hit[o] = (int)h;
        S.att_sc[o] = sc;
        ++o;
        if (ann) {                                  // annotation pass 1: best score bits
          for (int b = 0; b < ns; ++b) {
            if (!((m >> b) & 1u)) continue;
            if (lds_ann) atomicMax(&s_best[g * ns + b], dbits(sc));
            else atomicMax(reinterpret_cast<unsigned long long*>(&S.annot_best[(l0 + g) * ns + b]), dbits(sc));
          }
        }
      });
    }
    if (PASS == 0) {
      long long a = n_tot, b = nl_tot;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off, 64);
        b += __shfl_xor(b, off, 64);
      }
      if (lane == 0) { s_red[0][w] = a; s_red[1][w] = b; }
      __syncthreads();
      if (tid == 0) {
        long long ta = 0, tb = 0;
        for (int i = 0; i < NT / 64; ++i) { ta += s_red[0][i]; tb += s_red[1][i]; }
        ccnt[c] = ta;
        cleaves[c] = tb;
      }
      __syncthreads();
      continue;
    }
    if (ns > 0) {
      // annotation pass 2: the last hit (largest index) at the best score, per (locus,
      // system); every attachment of this contig is in [catt_off[c], base)
      __syncthreads();
      const int64_t a0 = S.catt_off[c];
      for (int64_t a = a0 + tid; a < base; a += NT) {
        const int h = S.att_hit[a];
        const uint32_t m = hkey ? K.hkey[h] >> kKeySys : K.sysmask[h];
        const double sc = S.att_sc[a];
        if (m == 0 || !(sc >= P.annot_ref)) continue;
        const int g = S.att_loc[a];
        for (int b = 0; b < ns; ++b) {
          if (!((m >> b) & 1u)) continue;
          if (lds_ann) {
            if (s_best[g * ns + b] == dbits(sc)) atomicMax(&s_hit[g * ns + b], h);
          } else if (S.annot_best[(l0 + g) * ns + b] == dbits(sc)) {
            atomicMax(&K.annot[(l0 + g) * ns + b], h);
          }
        }
      }
      __syncthreads();
      if (lds_ann)
        for (int i = tid; i < G * ns; i += NT) K.annot[l0 * ns + i] = s_hit[i];
    }
    __syncthreads();
  }
}

// ---- one roll-up level -------------------------------------------------------------------
__device__ __forceinline__ uint64_t make_key(const SArgs& S, int crank, int a) {
  return ((uint64_t)crank << (S.key_tb + S.key_lb)) | ((uint64_t)(uint32_t)S.att_clade[a] << S.key_lb) |
         (uint64_t)S.att_loc[a];
}

// Keys of every active contig's attachments at act_base[rank] (level 0: all contigs, at
// their own attachment offsets).  Used with the device radix sort.
__global__ void k_keys_active(const SArgs S, int n_act, uint64_t* keys, int32_t* vals) {
  for (int cr = blockIdx.x; cr < n_act; cr += gridDim.x) {
    const int c = S.act ? S.act[cr] : cr;
    const int64_t a0 = S.catt_off[c], a1 = S.catt_off[c + 1];
    const int64_t base = S.act_base ? S.act_base[cr] : a0;   // level 0: own offsets
    for (int64_t i = threadIdx.x; i < a1 - a0; i += blockDim.x) {
      keys[base + i] = make_key(S, cr, (int)(a0 + i));
      vals[base + i] = (int)(a0 + i);
    }
  }
}

// Segments only ever group attachments of one contig, and the contigs' key blocks already
// sit in rank order (level 0: attachment order; later levels: act_base is handed out in
// rank order), so sorting each contig's (key, attachment) pairs on its own -- in LDS, one
// workgroup per contig -- gives the same sequence as one global radix sort of the level.
// Ties keep attachment order.  Keys are built here (no separate key kernel).  In LDS one
// 64-bit word per attachment: its key without the contig-rank bits (constant within the
// contig) over its 13-bit index in the contig, so the word order is the (key, attachment)
// order and the full key is rebuilt on the way out.  Dynamic LDS: sort_cap x 8 bytes.
// 32 KiB of LDS.  8,192 (the cfg5 stress contigs, ~5,000 attachments) measured slower than
// the device radix sort at cfg5 (r4k: 14.1 against 12.0 ms per 6,250-contig pass: 2 workgroups
// per CU, 91 barrier-separated LDS stages, then k_seg_build's wave walking 5,000 keys)
constexpr int kSortMax = 4096;
constexpr int kSortIdxBits = 13;
static_assert(kSortMax <= (1 << kSortIdxBits), "contig-local index field");

template <int NT>
__global__ __launch_bounds__(NT) void k_sort_contig(const SArgs S, int n_act,
                                                          int level, uint64_t* keys, int32_t* vals) {
  int64_t n_keys_ = 0;
  lvl_counts(S, n_act, n_keys_);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint64_t* sk = reinterpret_cast<uint64_t*>(smem);
  __shared__ int s_red[NT / 64];
  const uint64_t rank_shift = (uint64_t)(S.key_tb + S.key_lb);
  const int tid = threadIdx.x;
  for (int cr = blockIdx.x; cr < n_act; cr += gridDim.x) {
    const int c = S.act ? S.act[cr] : cr;
    const int64_t a0 = S.catt_off[c], a1 = S.catt_off[c + 1];
    const int n = (int)(a1 - a0);
    if (n == 0) {
      if (tid == 0) S.seg_cnt[cr] = 0;
      continue;
    }
    const int64_t base = S.act_base ? S.act_base[cr] : a0;   // level 0: own offsets
    int n2 = 2;
    while (n2 < n) n2 <<= 1;
    for (int t = tid; t < n2; t += NT)
      sk[t] = t < n ? (make_key(S, 0, (int)(a0 + t)) << kSortIdxBits) | (uint64_t)t : ~0ull;
    __syncthreads();
    for (int k = 2; k <= n2; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < (n2 >> 1); i += NT) {
          const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1));   // i with a 0 inserted at bit j
          const int hi = lo | j;
          const bool up = (lo & k) == 0;
          const uint64_t ka = sk[lo], kb = sk[hi];
          if ((ka > kb) == up) { sk[lo] = kb; sk[hi] = ka; }
        }
        __syncthreads();
      }
    }
    int ns = 0;                                      // distinct keys = segments
    const uint64_t crank_bits = (uint64_t)cr << rank_shift;
    for (int t = tid; t < n; t += NT) {
      const uint64_t w = sk[t];
      keys[base + t] = crank_bits | (w >> kSortIdxBits);
      vals[base + t] = (int)(a0 + (int64_t)(w & ((1u << kSortIdxBits) - 1)));
      ns += (t == 0 || (w >> kSortIdxBits) != (sk[t - 1] >> kSortIdxBits)) ? 1 : 0;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ns += __shfl_xor(ns, off, 64);
    if (NT > 64) {
      if ((tid & 63) == 0) s_red[tid >> 6] = ns;
      __syncthreads();
      if (tid == 0)
        for (int w = 1; w < NT / 64; ++w) ns += s_red[w];
    }
    if (tid == 0) S.seg_cnt[cr] = ns;
    __syncthreads();
  }
  if (blockIdx.x == 0 && tid == 0) S.seg_cnt[n_act] = 0;   // exclusive scan -> crank_first
}

// Contigs of more than kSortMax attachments (up to kRadixMax: the cfg5 stress contigs, ~5,000
// each), one 512-thread workgroup per contig, LDS radix sort: the contig's 32-bit keys (clade
// << lb | locus; rank bits added on the way out) and 16-bit attachment indices, ping-pong in
// LDS, sorted by stable counting passes of 8 bits (3 for the usual 20-bit key).  Per pass
// each wave owns a contiguous slice of the elements: per-wave digit counts (the lanes of a
// 64-element chunk that share a digit found by 8 ballots, one LDS add per digit group), a
// digit-major / wave-minor prefix, then each wave scatters its chunks in order (rank =
// lanes below with the same digit).  Same order as the bitonic sort of the (key, index)
// words, so k_seg_build follows unchanged.  (The round-4 bitonic 8,192 sort took 91
// barrier-separated stages per contig and measured slower than the device radix sort.)
constexpr int kRadixMax = 8192;
constexpr int kRadixNT = 512;
constexpr int kRadixBits = 8;
constexpr int kRadixBins = 1 << kRadixBits;
// dynamic LDS for a capacity of `cap` attachments (a multiple of 512): two key and two index
// buffers, the per-wave digit counts -- 80 KB at cap 6,144 (two workgroups per CU), 104 KB at 8,192
inline size_t radix_lds(int cap, bool packed = false) {
  return (size_t)cap * 2 * (packed ? 4 : 4 + 2) + (size_t)(kRadixNT / 64) * kRadixBins * 4 + 64;
}

// The sort's LDS (dynamic, radix_lds(cap, packed) bytes): the ping-pong key and index buffers
// (packed: 32-bit words only) and the per-wave digit counts
struct RadixLds {
  uint32_t* kb0;
  uint16_t* ib0;
  int* cnt;                                            // [wave][bin]
  int cap;
  __device__ RadixLds(char* smem, int cap_, bool packed = false)
      : kb0(reinterpret_cast<uint32_t*>(smem)), ib0(reinterpret_cast<uint16_t*>(smem + 8 * (size_t)cap_)),
        cnt(reinterpret_cast<int*>(smem + (packed ? 8 : 12) * (size_t)cap_)), cap(cap_) {}
  __device__ uint32_t* kb(int x) const { return kb0 + x * cap; }   // buffer x of the pair
  __device__ uint16_t* ib(int x) const { return ib0 + x * cap; }
};

// The stable LSD passes over n loaded elements (buffer 0; BITS-bit digits of the low kbits
// bits above `skip`): each wave owns a contiguous slice; per-wave digit counts (type CT) from
// BITS ballots, a digit-major / wave-minor prefix, then each wave scatters its chunks in order.
// PACKED: the key and its index share one 32-bit word (no index buffers).  Returns the
// buffer holding the sorted sequence.
template <bool PACKED, int BITS = kRadixBits, class CT = int>
__device__ __forceinline__ int radix_passes(const RadixLds& R, int n, int kbits, int skip, int* s_red) {
  constexpr int kW = kRadixNT / 64, kBins = 1 << BITS;
  static_assert(kBins <= kRadixNT && kW * kBins * sizeof(CT) <= kW * kRadixBins * sizeof(int), "count area");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  CT* const cnt = reinterpret_cast<CT*>(R.cnt);
  // wave w's slice [lo, hi) of the elements
  const int per = (n + kW - 1) / kW;
  const int lo = min(n, w * per), hi = min(n, lo + per);
  int cur = 0;
  for (int shift = 0; shift < kbits; shift += BITS) {
    for (int i = tid; i < kW * kBins; i += kRadixNT) cnt[i] = 0;
    __syncthreads();
    // the lanes of this chunk with the same digit (d), from BITS ballots
    auto group = [&](int i, int& d) -> uint64_t {
      const bool live = i < hi;
      d = live ? (int)((R.kb(cur)[i] >> (skip + shift)) & (kBins - 1)) : 0;
      uint64_t m = __ballot(live);
#pragma unroll
      for (int b = 0; b < BITS; ++b) {
        const uint64_t bal = __ballot((d >> b) & 1);
        m &= ((d >> b) & 1) ? bal : ~bal;
      }
      return live ? m : 0ull;
    };
    for (int i0 = lo; i0 < hi; i0 += 64) {           // per-wave digit counts
      int d;
      const uint64_t m = group(i0 + lane, d);
      if (m && (m & below) == 0ull) cnt[w * kBins + d] += (CT)__popcll(m);   // (the group's first lane)
    }
    __syncthreads();
    // offsets: digit-major, wave-minor (thread d walks the waves of digit d, then a scan of
    // the digit totals across the block)
    int tot = 0;
    if (tid < kBins)
      for (int x = 0; x < kW; ++x) {
        const int v = cnt[x * kBins + tid];
        cnt[x * kBins + tid] = (CT)tot;
        tot += v;
      }
    // exclusive scan of the digit totals (thread d: digit d)
    int incl = tot;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    if (lane == 63) s_red[w] = incl;
    __syncthreads();
    if (tid < kBins) {
      int pre = incl - tot;
      for (int x = 0; x < w; ++x) pre += s_red[x];
      for (int x = 0; x < kW; ++x) cnt[x * kBins + tid] += (CT)pre;
    }
    __syncthreads();
    // scatter, each wave its chunks in order (stable)
    for (int i0 = lo; i0 < hi; i0 += 64) {
      int d;
      const uint64_t m = group(i0 + lane, d);
      if (m) {
        const int pos = cnt[w * kBins + d] + __popcll(m & below);
        R.kb(cur ^ 1)[pos] = R.kb(cur)[i0 + lane];
        if (!PACKED) R.ib(cur ^ 1)[pos] = R.ib(cur)[i0 + lane];
      }
      wave_sync();                                   // (reads of the counts before the update)
      if (m && (m >> lane) == 1ull) cnt[w * kBins + d] += (CT)__popcll(m);   // (the group's last lane)
      wave_sync();
    }
    __syncthreads();
    cur ^= 1;
  }
  return cur;
}

// One contig's n > 0 attachments [a0, a0 + n) sorted by key (clade << lb | locus) in LDS (the
// whole workgroup); returns the buffer holding the sorted keys and their contig-local indices.
__device__ __forceinline__ int radix_sort_contig(const SArgs& S, int64_t a0, int n, const RadixLds& R, int* s_red) {
  const int tid = threadIdx.x;
  // (the attachments' clade and locus loads of four strides issued together)
  for (int i0 = 0; i0 < n; i0 += 4 * kRadixNT) {
    uint32_t kk[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + r * kRadixNT + tid;
      kk[r] = i < n ? (uint32_t)make_key(S, 0, (int)(a0 + i)) : 0u;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + r * kRadixNT + tid;
      if (i < n) {
        R.kb(0)[i] = kk[r];
        R.ib(0)[i] = (uint16_t)i;
      }
    }
  }
  return radix_passes<false>(R, n, S.key_tb + S.key_lb, 0, s_red);   // (<= 32 bits: checked on the host)
}

// The same order from one 32-bit word per attachment: the contig's clades present (a bitmap
// over the taxonomy's ids, aliasing the digit counts until the passes) ranked in id order, so
// (rank << lb | locus) << kSortIdxBits | index fits 32 bits and sorts exactly as (clade,
// locus, index).  8 instead of 12 bytes of LDS per attachment, and only as many passes as the
// contig's ranks need.  Requires lb <= 6 and a bitmap + word prefix of at most the count
// area (n_tax <= kPackTaxMax); returns the buffer of sorted words.
constexpr int kPackTaxMax = (kRadixNT / 64) * kRadixBins * 4 / 6 * 32;   // (6 B a bitmap word <= the counts)
__device__ __forceinline__ int radix_sort_packed(const SArgs& S, int64_t a0, int n, int n_tax, const RadixLds& R,
                                                 int* s_red) {
  constexpr int kW = kRadixNT / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nw = (n_tax + 31) >> 5;
  uint32_t* const bm = reinterpret_cast<uint32_t*>(R.cnt);
  uint16_t* const bpre = reinterpret_cast<uint16_t*>(bm + nw);
  for (int i = tid; i < nw; i += kRadixNT) bm[i] = 0u;
  __syncthreads();
  for (int i = tid; i < n; i += kRadixNT) {
    const uint32_t cl = (uint32_t)S.att_clade[a0 + i], g = (uint32_t)S.att_loc[a0 + i];
    atomicOr(&bm[cl >> 5], 1u << (cl & 31u));
    R.kb(0)[i] = cl << 8 | g;                        // (clade, locus) until the ranks are known
  }
  __syncthreads();
  // the ranks' word prefix: thread t sums words [t k, t k + k), a block scan of the sums
  const int k = (nw + kRadixNT - 1) / kRadixNT;
  int own = 0;
  for (int x = tid * k; x < min(nw, tid * k + k); ++x) own += __popc(bm[x]);
  int incl = own;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) s_red[w] = incl;
  __syncthreads();
  int pre = incl - own, present = 0;
#pragma unroll
  for (int x = 0; x < kW; ++x) {
    pre += x < w ? s_red[x] : 0;
    present += s_red[x];
  }
  for (int x = tid * k; x < min(nw, tid * k + k); ++x) {
    bpre[x] = (uint16_t)pre;
    pre += __popc(bm[x]);
  }
  __syncthreads();
  const int lb = S.key_lb;
  for (int i = tid; i < n; i += kRadixNT) {
    const uint32_t x = R.kb(0)[i], cl = x >> 8;
    const uint32_t rank = bpre[cl >> 5] + __popc(bm[cl >> 5] & ((1u << (cl & 31u)) - 1u));
    R.kb(0)[i] = ((rank << lb) | (x & 255u)) << kSortIdxBits | (uint32_t)i;
  }
  __syncthreads();
  const int rbits = 32 - __clz(max(present - 1, 1));
  // up to 16 key bits: 8-bit digits; 17-18 (level 0 at cfg5): two passes of 9-bit digits with
  // 16-bit counts in the same count area instead of three of 8 (level 0 1.10 -> 0.98 ms; the
  // ninth ballot made the 16-bit levels slower)
  return rbits + lb <= 2 * kRadixBits || rbits + lb > 18
             ? radix_passes<true>(R, n, rbits + lb, kSortIdxBits, s_red)
             : radix_passes<true, 9, uint16_t>(R, n, rbits + lb, kSortIdxBits, s_red);
}

__global__ __launch_bounds__(kRadixNT) void k_sort_radix(const SArgs S, int n_act, int level, uint64_t* keys,
                                                       int32_t* vals) {
  int64_t n_keys_ = 0;
  lvl_counts(S, n_act, n_keys_);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const RadixLds R(smem, S.sort_cap);                  // (the level's largest contig, rounded up)
  __shared__ int s_red[kRadixNT / 64];
  constexpr int kW = kRadixNT / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t rank_shift = (uint64_t)(S.key_tb + S.key_lb);
  for (int cr = blockIdx.x; cr < n_act; cr += gridDim.x) {
    const int c = S.act ? S.act[cr] : cr;
    const int64_t a0 = S.catt_off[c], a1 = S.catt_off[c + 1];
    const int n = (int)(a1 - a0);
    const int64_t base = S.act_base ? S.act_base[cr] : a0;   // level 0: own offsets
    if (n == 0) {
      if (tid == 0) S.seg_cnt[cr] = 0;
      continue;
    }
    const int cur = radix_sort_contig(S, a0, n, R, s_red);
    int ns = 0;                                      // distinct keys = segments
    const uint64_t crank_bits = (uint64_t)cr << rank_shift;
    for (int t = tid; t < n; t += kRadixNT) {
      const uint32_t k = R.kb(cur)[t];
      keys[base + t] = crank_bits | (uint64_t)k;
      vals[base + t] = (int)(a0 + (int64_t)R.ib(cur)[t]);
      ns += (t == 0 || k != R.kb(cur)[t - 1]) ? 1 : 0;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ns += __shfl_xor(ns, off, 64);
    if (lane == 0) s_red[w] = ns;
    __syncthreads();
    if (tid == 0) {
      for (int x = 1; x < kW; ++x) ns += s_red[x];
      S.seg_cnt[cr] = ns;
    }
    __syncthreads();
  }
  if (blockIdx.x == 0 && tid == 0) S.seg_cnt[n_act] = 0;   // exclusive scan -> crank_first
}

// Segments of each contig from its sorted keys (one wave per contig), at the contig's
// offset from the scan of per-contig segment counts: segment starts and ranks, the
// attachments gathered into sorted order, the rank -> first segment map and the segment
// total.  Replaces the flag / scan / segment / gather / rank-map kernels of the radix path.
__global__ __launch_bounds__(64) void k_seg_build(const SArgs S, int n_act, int level, int64_t n_keys) {
  lvl_counts(S, n_act, n_keys);
  const int lane = threadIdx.x;
  if (blockIdx.x == 0 && lane == 0 && n_keys > 0) {
    const int total = S.crank_first[n_act];
    S.seg_start[total] = (int)n_keys;
    S.seg_id[n_keys - 1] = total;                    // seg_count()
  }
  const KArgs& K = S.k;
  const uint64_t lmask = (1ull << S.key_lb) - 1, tmask = (1ull << S.key_tb) - 1;
  for (int cr = blockIdx.x; cr < n_act; cr += gridDim.x) {
    const int c = S.act ? S.act[cr] : cr;
    const int n = (int)(S.catt_off[c + 1] - S.catt_off[c]);
    const int64_t base = S.act_base ? S.act_base[cr] : S.catt_off[c];
    int sbase = S.crank_first[cr];
    const int64_t l0 = K.loc_off[c];
    const int G = (int)(K.loc_off[c + 1] - l0);
    int glen = 0;                                    // lane g: length of locus g (G <= 64)
    if (lane < G) {
      const int a = K.lstart[l0 + lane], b = K.lend[l0 + lane];
      glen = max(a, b) - min(a, b) + 1;
    }
    for (int t0 = 0; t0 < n; t0 += 64) {
      const int t = t0 + lane;
      const bool live = t < n;
      uint64_t key = 0, prev = 0;
      int a = 0;
      if (live) {
        key = S.keys[base + t];
        prev = t > 0 ? S.keys[base + t - 1] : ~key;
        a = S.vals[base + t];
        S.satt_lohi[base + t] = make_int2(S.att_lo[a], S.att_hi[a]);
        S.satt_sc[base + t] = S.att_sc[a];
      }
      const bool head = live && key != prev;
      const uint64_t hm = __ballot(head);
      const int g = (int)(key & lmask);
      int len = __shfl(glen, g & 63, 64);
      if (head) {
        if (G > 64) {
          const int a = K.lstart[l0 + g], b = K.lend[l0 + g];
          len = max(a, b) - min(a, b) + 1;
        }
        const int seg = sbase + __popcll(hm & ((1ull << lane) - 1ull));
        S.seg_start[seg] = (int)(base + t);
        S.seg_crank[seg] = cr;
        S.seg_cg[seg] = make_int2((int)((key >> S.key_lb) & tmask), g);
        S.seg_len[seg] = len;
      }
      sbase += __popcll(hm);
    }
  }
}

// k_seg_build for the contigs of the LDS radix sort (4,097..8,192 attachments: the cfg5 stress
// contigs), one 512-thread workgroup per contig: the same outputs, a chunk of 512 sorted keys
// per step (segment heads counted per wave by ballot, then across the waves through LDS)
// instead of one wave stepping 64 keys at a time through ~5,000.
__global__ __launch_bounds__(kRadixNT) void k_seg_build_wide(const SArgs S, int n_act, int level, int64_t n_keys) {
  lvl_counts(S, n_act, n_keys);
  constexpr int kW = kRadixNT / 64;
  __shared__ int s_glen[64];
  __shared__ int s_cnt[kW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (blockIdx.x == 0 && tid == 0 && n_keys > 0) {
    const int total = S.crank_first[n_act];
    S.seg_start[total] = (int)n_keys;
    S.seg_id[n_keys - 1] = total;                    // seg_count()
  }
  const KArgs& K = S.k;
  const uint64_t lmask = (1ull << S.key_lb) - 1, tmask = (1ull << S.key_tb) - 1;
  for (int cr = blockIdx.x; cr < n_act; cr += gridDim.x) {
    const int c = S.act ? S.act[cr] : cr;
    const int n = (int)(S.catt_off[c + 1] - S.catt_off[c]);
    const int64_t base = S.act_base ? S.act_base[cr] : S.catt_off[c];
    int sbase = S.crank_first[cr];
    const int64_t l0 = K.loc_off[c];
    const int G = (int)(K.loc_off[c + 1] - l0);
    if (tid < 64 && tid < G) {                       // locus lengths (G <= 64)
      const int a = K.lstart[l0 + tid], b = K.lend[l0 + tid];
      s_glen[tid] = max(a, b) - min(a, b) + 1;
    }
    __syncthreads();
    // kSbR chunks of kRadixNT keys per step: their key, index and attachment loads issued
    // together (one dependent gather round per step, not per chunk)
    constexpr int kSbR = 4;
    for (int t00 = 0; t00 < n; t00 += kSbR * kRadixNT) {
      uint64_t key[kSbR], prev[kSbR];
      int av[kSbR];
#pragma unroll
      for (int r = 0; r < kSbR; ++r) {
        const int t = t00 + r * kRadixNT + tid;
        key[r] = 0; prev[r] = 0; av[r] = 0;
        if (t < n) {
          key[r] = S.keys[base + t];
          prev[r] = t > 0 ? S.keys[base + t - 1] : ~key[r];
          av[r] = S.vals[base + t];
        }
      }
#pragma unroll
      for (int r = 0; r < kSbR; ++r) {
        const int t = t00 + r * kRadixNT + tid;
        if (t < n) {
          const int a = av[r];
          S.satt_lohi[base + t] = make_int2(S.att_lo[a], S.att_hi[a]);
          S.satt_sc[base + t] = S.att_sc[a];
        }
      }
#pragma unroll
      for (int r = 0; r < kSbR; ++r) {
        const int t0 = t00 + r * kRadixNT;
        if (t0 >= n) break;                            // (uniform)
        const int t = t0 + tid;
        const bool head = t < n && key[r] != prev[r];
        const uint64_t hm = __ballot(head);
        if (lane == 0) s_cnt[w] = __popcll(hm);
        __syncthreads();
        int before = 0, total = 0;
#pragma unroll
        for (int x = 0; x < kW; ++x) {
          before += x < w ? s_cnt[x] : 0;
          total += s_cnt[x];
        }
        if (head) {
          const int g = (int)(key[r] & lmask);
          int len;
          if (G <= 64) {
            len = s_glen[g];
          } else {
            const int a = K.lstart[l0 + g], b = K.lend[l0 + g];
            len = max(a, b) - min(a, b) + 1;
          }
          const int seg = sbase + before + __popcll(hm & ((1ull << lane) - 1ull));
          S.seg_start[seg] = (int)(base + t);
          S.seg_crank[seg] = cr;
          S.seg_cg[seg] = make_int2((int)((key[r] >> S.key_lb) & tmask), g);
          S.seg_len[seg] = len;
        }
        sbase += total;
        __syncthreads();                             // (s_cnt reused by the next chunk)
      }
    }
  }
}

__global__ void k_seg_flags(const SArgs S, int64_t n) {
  int n_act_ = 0;
  lvl_counts(S, n_act_, n);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) S.flags[i] = (i == 0 || S.keys[i] != S.keys[i - 1]) ? 1 : 0;
}

__global__ void k_segs(const SArgs S, int64_t n) {
  int n_act_ = 0;
  lvl_counts(S, n_act_, n);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (S.flags[i]) {
    const int s = S.seg_id[i] - 1;
    S.seg_start[s] = (int)i;
    S.seg_crank[s] = (int)(S.keys[i] >> (S.key_tb + S.key_lb));
  }
  if (i == n - 1) S.seg_start[S.seg_id[i]] = (int)n;
}

// crank_first[cr] = first segment of active contig cr (segments are sorted by rank; ranks
// without segments get the next rank's start), crank_first[n_act] = segment count.
__global__ void k_crank_first(const SArgs S, int64_t n_keys, int n_act) {
  lvl_counts(S, n_act, n_keys);
  const int ns = seg_count(S, n_keys);
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s > ns) return;
  const int c0 = s == 0 ? -1 : S.seg_crank[s - 1];
  const int c1 = s == ns ? n_act : S.seg_crank[s];
  for (int cr = c0 + 1; cr <= c1; ++cr) S.crank_first[cr] = s;
}

// Attachments copied into sorted order, so each segment's are contiguous.
__global__ void k_gather(const SArgs S, int64_t n) {
  int n_act_ = 0;
  lvl_counts(S, n_act_, n);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int a = S.vals[i];
  S.satt_lohi[i] = make_int2(S.att_lo[a], S.att_hi[a]);
  S.satt_sc[i] = S.att_sc[a];
}

// ---- exact segment means, leaf-parallel ------------------------------------------------
// A segment's site array (length n) is summed by numpy as 8192-element buffers added in
// order from 0.0, each buffer by the pairwise tree whose leaves the LUT lists.  Leaves are
// evaluated independently (one thread each, closed forms; the rare multi-run leaf by eight
// cooperating lanes), then one thread per segment combines its leaf values in tree order.
struct SegInfo {
  int kb, ke, c, g, len;
};

__device__ __forceinline__ SegInfo seg_info(const SArgs& S, int s) {
  const KArgs& K = S.k;
  SegInfo i;
  i.kb = S.seg_start[s];
  i.ke = S.seg_start[s + 1];
  const uint64_t key = S.keys[i.kb];
  const int crank = (int)(key >> (S.key_tb + S.key_lb));
  i.g = (int)(key & ((1ull << S.key_lb) - 1));
  i.c = S.act ? S.act[crank] : crank;
  const int64_t l = K.loc_off[i.c] + i.g;
  const int ls = K.lstart[l], le = K.lend[l];
  i.len = max(ls, le) - min(ls, le) + 1;
  return i;
}

__device__ __forceinline__ int lut_count(const SArgs& S, int m) { return S.lut_off[m + 1] - S.lut_off[m]; }

// Per segment: its leaf count (for the leaf offsets scan) and a self-contained record, so
// the leaf kernels resolve a segment with one load.
//
// Segments whose site array is ONE run of value v over a zero background -- a single
// attachment (lo, hi, v), or any number of them all dominated by the highest one that covers
// the whole locus (lo = 0, hi = len, v = that score) -- are finished right here by their own
// thread (one buffer, <= kThreadLeaves leaves: every species-level segment of a <= 2.9 kb
// locus).  Every leaf then has the same closed form (run_leaf), so the lanes of a wave run
// one code path; the leaves go in tree order onto a register stack, exactly as k_leaf +
// k_seg_combine do, without the leaf list, the leaf values or the leaf -> segment map ever
// touching HBM.  Their leaf count is reported as 0, so the leaf kernels skip them.



// --write-details gene spans (make_gene_spans_field, orgscorer.py:770-789), thread per
// segment, before k_seg_rec compacts the attachment ranges.  The clade's site array at the
// locus is nonzero exactly on the union of its attachments' [lo, hi) ranges with score > 0;
// the reference lists the first and last site (1-based) of every maximal nonzero run
// longer than one site.  Runs come out in site order by repeated selection (a segment has
// few attachments; this is a diagnostic output).  span_cnt = -1: no nonzero site (upstream
// raises IndexError).  Runs go to spans[2 * seg_start[s] ...] (at most one per attachment).
__global__ void k_seg_spans(const SArgs S, int64_t n_keys, int32_t* span_cnt, int32_t* spans) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= seg_count(S, n_keys)) return;
  const int t0 = S.seg_start[s], t1 = S.seg_start[s + 1];
  int pos = 0, cnt = 0;
  bool any = false;
  for (;;) {
    int lo = INT_MAX;                                // next run: smallest live start >= pos
    for (int t = t0; t < t1; ++t) {
      const int2 x = S.satt_lohi[t];
      if (S.satt_sc[t] > 0.0 && x.y > x.x && x.x >= pos && x.x < lo) lo = x.x;
    }
    if (lo == INT_MAX) break;
    any = true;
    int hi = lo;
    for (bool grew = true; grew;) {                  // absorb every range reaching the run
      grew = false;
      for (int t = t0; t < t1; ++t) {
        const int2 x = S.satt_lohi[t];
        if (S.satt_sc[t] > 0.0 && x.y > x.x && x.x <= hi && x.y > hi) { hi = x.y; grew = true; }
      }
    }
    if (hi - lo >= 2) {
      spans[2 * ((int64_t)t0 + cnt)] = lo + 1;
      spans[2 * ((int64_t)t0 + cnt) + 1] = hi;
      ++cnt;
    }
    pos = hi;
  }
  span_cnt[s] = any ? cnt : -1;
}

struct RecAtt {
  int2 x;                                            // site range [lo, hi)
  double sc;
};

// One segment's mean or record (k_seg_rec's per-segment body): its na attachments are get(t),
// t < na, in sorted order; a record's attachments are written through put(k, att) (the list
// the wave / leaf kernels read at sorted positions kb...; in_place: get(t) already reads
// position kb + t, so only moved entries are written).  One run: the exact mean into
// seg_mean[s]; else seg_rec[s] and, for 5..64 attachments of a short locus, to_wave
// (k_seg_wave).  Returns the segment's leaves for the leaf kernels (0: finished here or by
// k_seg_wave).
template <class Get, class Put>
__device__ __forceinline__ int seg_record(const SArgs& S, int64_t s, int kb, int na, int len, Get get, Put put,
                                          bool in_place, bool& to_wave) {
  int nl = (len / kNpyBuf) * lut_count(S, kNpyBuf) + lut_count(S, len % kNpyBuf);
  int lo = 0, hi = 0;
  double v = 0.0;
  bool one_run = false, listed = in_place;           // listed: the record's list is in place
  const bool thread_ok = len < kNpyBuf && nl <= kThreadLeaves;
  to_wave = false;
  if (na == 1) {
    if (thread_ok) {
      const RecAtt t = get(0);
      lo = t.x.x; hi = t.x.y; v = t.sc;
      one_run = true;
    }
  } else if (na <= kPruneMax) {
    double F = 0.0;                                  // best whole-locus attachment
#pragma unroll 4
    for (int t = 0; t < na; ++t) {
      const RecAtt e = get(t);
      if (e.x.x <= 0 && e.x.y >= len && e.sc > F) F = e.sc;
    }
    // attachments at or below F (or empty) change no site: the envelope is
    // max(F, the others).  None left: one run of F.  Otherwise the survivors are
    // compacted, with F as one whole-locus attachment after them, so the leaf
    // kernel sees few attachments (usually <= kRegAtt: register path).
    int kept = 0;
#pragma unroll 4
    for (int t = 0; t < na; ++t) {
      const RecAtt e = get(t);
      if (e.x.x < e.x.y && e.sc > F) {
        if (!in_place || kept != t) put(kept, e);
        ++kept;
      }
    }
    if (kept == 0 && thread_ok) {
      lo = 0; hi = len; v = F; one_run = true;
    } else {
      // F > 0 came from an attachment that was not kept (its score is F), so the list
      // never grows; it may have shifted, so F is always re-appended
      if (F > 0.0) {
        put(kept, RecAtt{make_int2(0, len), F});
        ++kept;
      }
      na = kept;
      listed = true;
    }
  }
  if (one_run) {
    S.seg_mean[s] = one_run_mean(PtrLut{S.lut + S.lut_off[len]}, nl, len, lo, hi, v);
    return 0;
  }
  if (!listed)
    for (int t = 0; t < na; ++t) put(t, get(t));
  S.seg_rec[s] = make_int4(kb, na, len, nl);
  // many attachments (higher roll-up levels): one wave per segment (k_seg_wave)
  to_wave = na > kRegAtt && na <= 64 && nl <= 64 && len < kNpyBuf;
  return to_wave ? 0 : nl;
}

// the segments k_seg_rec / k_front_radix hand to k_seg_wave: one list append per wave
__device__ __forceinline__ void wave_list_add(const SArgs& S, int64_t s, bool to_wave) {
  const uint64_t bm = __ballot(to_wave);
  if (bm) {
    const int lane = threadIdx.x & 63, leader = __builtin_ctzll(bm);
    int base = 0;
    if (lane == leader) base = (int)atomicAdd(&S.counters[7], (unsigned long long)__popcll(bm));
    base = __shfl(base, leader, 64);
    if (to_wave) S.wave_list[base + __popcll(bm & ((1ull << lane) - 1ull))] = (int)s;
  }
}

__global__ void k_seg_rec(const SArgs S, int64_t n_keys) {
  int n_act_ = 0;
  lvl_counts(S, n_act_, n_keys);
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s > n_keys) return;
  int nl = 0;
  bool to_wave = false;
  if (s < seg_count(S, n_keys)) {
    SegInfo si;
    if (S.seg_len) {                                 // k_seg_build wrote length and (clade, locus)
      si.kb = S.seg_start[s];
      si.ke = S.seg_start[s + 1];
      si.len = S.seg_len[s];
    } else {
      si = seg_info(S, (int)s);
      S.seg_cg[s] = make_int2((int)((S.keys[si.kb] >> S.key_lb) & ((1ull << S.key_tb) - 1)), si.g);
    }
    const int kb = si.kb;
    nl = seg_record(
        S, s, kb, si.ke - kb, si.len, [&](int t) { return RecAtt{S.satt_lohi[kb + t], S.satt_sc[kb + t]}; },
        [&](int k, const RecAtt& e) { S.satt_lohi[kb + k] = e.x; S.satt_sc[kb + k] = e.sc; }, true, to_wave);
  }
  S.seg_nleaf[s] = nl;
  wave_list_add(S, s, to_wave);
}

// The stress contigs' segment front end in one launch (round 6; for the contigs of the LDS
// radix sort, 4,097..8,192 attachments: k_sort_radix + k_seg_build_wide + k_seg_rec + the
// leaf-count scan + k_leaf_expand otherwise).  One 512-thread workgroup per contig, the
// contigs claimed in rank order from a counter (fr[0]):
//   * the LDS radix sort of the contig's keys (radix_sort_contig);
//   * segment heads from the sorted keys in LDS (ballots per 64 keys, a scan of the chunk
//     counts), segment starts into the spare key buffer;
//   * the contig's first segment from a decoupled look-back over the ranks before it: each
//     rank publishes its segment count as soon as it has it (status A), then its inclusive
//     prefix (P); wave 0 reads 64 ranks per step and stops at the nearest P.  A rank waits
//     only on smaller ranks, claimed earlier by resident workgroups that publish A without
//     waiting on anything, so the wait ends (bounded anyway: counters[4] records a timeout
//     and the host fails the call);
//   * one thread per segment: seg_record over the attachments read through the sorted local
//     indices (range and score loaded here, once), the leaf-path segments' leaves allocated
//     from fr[1] with leaf_seg written here.
// Only the segment table the decisions read (crank_first, seg_cg, seg_mean) and the records
// of the rare wave / leaf segments reach HBM: no keys, sorted attachment copies, segment
// starts or per-segment leaf counts.  fr: [0] ticket, [1] leaves, [4 + cr] rank cr's status
// (zeroed per level).
// PACKED (the usual shape: lb <= 6, n_tax <= kPackTaxMax): radix_sort_packed, 8 bytes of LDS
// per attachment, three workgroups per CU at the cfg5 size (80 VGPRs); else radix_sort_contig.
constexpr unsigned long long kLbA = 1ull << 62, kLbP = 2ull << 62, kLbVal = (1ull << 62) - 1ull;

// (S_arg first: the per-contig loop re-reads the argument block through kernarg_fresh, as
// k_big_sparse -- held across the loop its fields spill SGPRs into VGPR lanes)
template <bool PACKED>
__global__ __launch_bounds__(kRadixNT, PACKED ? 6 : 1) void k_front_radix(const SArgs S_arg, int n_act, int64_t n_keys,
                                                                         int n_tax, unsigned long long* fr) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int kW = kRadixNT / 64;
  __shared__ int s_red[kW];
  __shared__ int s_glen[64];
  __shared__ int s_chunk[kRadixMax / 64];
  __shared__ int s_cr, s_ns, s_sbase;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
  unsigned long long* const lb = fr + 4;
  for (;;) {
    if (tid == 0) s_cr = (int)atomicAdd(&fr[0], 1ull);
    __syncthreads();
    const int cr = s_cr;
    if (cr >= n_act) break;                          // (uniform)
    const SArgs& S = kernarg_fresh<SArgs>(S_arg);
    const KArgs& K = S.k;
    const RadixLds R(smem, S.sort_cap, PACKED);
    const uint32_t lmask = (1u << S.key_lb) - 1u, tmask = (uint32_t)((1ull << S.key_tb) - 1ull);
    const int c = S.act ? S.act[cr] : cr;
    const int64_t a0 = S.catt_off[c];
    const int n = (int)(S.catt_off[c + 1] - a0);
    const int64_t base = S.act_base ? S.act_base[cr] : a0;   // level 0: own offsets
    const int64_t l0 = K.loc_off[c];
    const int G = (int)(K.loc_off[c + 1] - l0);
    if (tid < 64 && tid < G) {                       // locus lengths (G <= 64)
      const int x = K.lstart[l0 + tid], y = K.lend[l0 + tid];
      s_glen[tid] = max(x, y) - min(x, y) + 1;
    }
    const int cur = n == 0 ? 0 : PACKED ? radix_sort_packed(S, a0, n, n_tax, R, s_red) : radix_sort_contig(S, a0, n, R, s_red);
    const uint32_t* const kk = R.kb(cur);            // sorted keys (PACKED: words)
    const uint16_t* const ii = R.ib(cur);            // (!PACKED) their indices
    uint32_t* const sst = R.kb(cur ^ 1);             // segment starts (the spare key buffer)
    auto key_at = [&](int t) -> uint32_t { return PACKED ? kk[t] >> kSortIdxBits : kk[t]; };
    auto idx_at = [&](int t) -> int { return PACKED ? (int)(kk[t] & ((1u << kSortIdxBits) - 1u)) : (int)ii[t]; };
    // segment heads: per-chunk counts, their exclusive scan (wave 0, two chunks a lane)
    const int nch = (n + 63) >> 6;
    for (int ch = w; ch < nch; ch += kW) {
      const int t = ch * 64 + lane;
      const uint64_t m = __ballot(t < n && (t == 0 || key_at(t) != key_at(t - 1)));
      if (lane == 0) s_chunk[ch] = __popcll(m);
    }
    __syncthreads();
    if (w == 0) {
      const int x0 = 2 * lane < nch ? s_chunk[2 * lane] : 0, x1 = 2 * lane + 1 < nch ? s_chunk[2 * lane + 1] : 0;
      int incl = x0 + x1;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
      }
      if (2 * lane < nch) s_chunk[2 * lane] = incl - x0 - x1;
      if (2 * lane + 1 < nch) s_chunk[2 * lane + 1] = incl - x1;
      if (lane == 63) s_ns = incl;
    }
    __syncthreads();
    const int ns = s_ns;
    for (int ch = w; ch < nch; ch += kW) {
      const int t = ch * 64 + lane;
      const bool head = t < n && (t == 0 || key_at(t) != key_at(t - 1));
      const uint64_t m = __ballot(head);
      if (head) sst[s_chunk[ch] + __popcll(m & below)] = (uint32_t)t;
    }
    // look-back: this rank's first segment
    if (w == 0) {
      if (lane == 0)
        __hip_atomic_store(&lb[cr], (cr == 0 ? kLbP : kLbA) | (unsigned long long)ns, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      long long excl = 0;
      for (int top = cr - 1; top >= 0;) {
        const int r = top - lane;
        unsigned long long v = r >= 0 ? 0ull : kLbP;   // (before rank 0: a zero prefix)
        for (int spin = 0;; ++spin) {
          if (r >= 0 && (v >> 62) == 0ull)
            v = __hip_atomic_load(&lb[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (__ballot((v >> 62) == 0ull) == 0ull) break;
          if (spin >= (1 << 22)) {                   // (never expected: fail the call, not the GPU)
            if (lane == 0) atomicExch(&S.counters[4], 1ull);
            if ((v >> 62) == 0ull) v = kLbA;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        const uint64_t pm = __ballot((v >> 62) == 2ull);
        const int first_p = pm ? __builtin_ctzll(pm) : 64;
        long long add = lane <= first_p ? (long long)(v & kLbVal) : 0;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) add += __shfl_xor(add, off, 64);
        excl += add;
        if (pm) break;
        top -= 64;
      }
      if (lane == 0) {
        if (cr > 0)
          __hip_atomic_store(&lb[cr], kLbP | (unsigned long long)(excl + ns), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        s_sbase = (int)excl;
        S.crank_first[cr] = (int)excl;
        if (cr == n_act - 1) {
          S.crank_first[n_act] = (int)excl + ns;
          if (n_keys > 0) S.seg_id[n_keys - 1] = (int)excl + ns;   // seg_count()
        }
      }
    }
    __syncthreads();
    const int sbase = s_sbase;
    for (int s0 = w * 64; s0 < ns; s0 += kRadixNT) {  // (wave-uniform trips: wave_list_add ballots)
      const int sl = s0 + lane;
      bool to_wave = false;
      const int64_t s = (int64_t)sbase + sl;
      if (sl < ns) {
        const int t0 = (int)sst[sl], t1 = sl + 1 < ns ? (int)sst[sl + 1] : n;
        const uint32_t key = key_at(t0);
        const int g = (int)(key & lmask);
        int len;
        if (G <= 64) {
          len = s_glen[g];
        } else {
          const int x = K.lstart[l0 + g], y = K.lend[l0 + g];
          len = max(x, y) - min(x, y) + 1;
        }
        S.seg_cg[s] = make_int2(PACKED ? S.att_clade[a0 + idx_at(t0)] : (int)((key >> S.key_lb) & tmask), g);
        const int kb = (int)(base + t0);
        const int nl = seg_record(
            S, s, kb, t1 - t0, len,
            [&](int t) {
              const int64_t a = a0 + idx_at(t0 + t);
              return RecAtt{make_int2(S.att_lo[a], S.att_hi[a]), S.att_sc[a]};
            },
            [&](int k, const RecAtt& e) { S.satt_lohi[kb + k] = e.x; S.satt_sc[kb + k] = e.sc; }, false, to_wave);
        if (nl > 0) {                                // the leaf kernels' share (rare)
          const int o = (int)atomicAdd(&fr[1], (unsigned long long)nl);
          S.leaf_off[s] = o;
          for (int j = 0; j < nl; ++j) S.leaf_seg[o + j] = (int)s;
        }
      }
      wave_list_add(S, s, to_wave);
    }
    __syncthreads();                                 // (LDS and s_cr reused by the next contig)
  }
}

// After k_front_radix: the leaf total where the leaf kernels read it (leaf_off[segments]).
__global__ void k_front_fin(const SArgs S, int n_act, const unsigned long long* fr) {
  if (threadIdx.x == 0 && blockIdx.x == 0) S.leaf_off[S.crank_first[n_act]] = (int)fr[1];
}

// Segments with 5..64 attachments, one wave each: the max-envelope is swept once into runs
// (lane i holds attachment i; run value = wave max over the covering ones, run end = wave
// min over the next boundaries), then lane q evaluates leaf q from the runs -- each of the
// eight stride accumulators adds its sites in site order, a run of value v contributing v
// k_c times (zero runs add nothing: x + 0.0 = x for x >= 0) -- and lane 0 folds the leaves
// in tree order.  Same sums as k_leaf's per-leaf stride walks, without rescanning the
// attachments for every run of every leaf.
__global__ __launch_bounds__(64) void k_seg_wave(const SArgs S) {
  __shared__ WaveRuns W;
  const int lane = threadIdx.x;
  const int count = (int)S.counters[7];
  for (int i = blockIdx.x; i < count; i += gridDim.x) {
    const int s = S.wave_list[i];
    const int4 rec = S.seg_rec[s];                  // (kb, attachments, length, leaves)
    int lo = 0, hi = 0;
    double sc = 0.0;
    if (lane < rec.y) {
      const int2 x = S.satt_lohi[rec.x + lane];
      if (x.x < x.y) { lo = x.x; hi = x.y; sc = S.satt_sc[rec.x + lane]; }
    }
    const double m = wave_seg_mean(PtrLut{S.lut + S.lut_off[rec.z]}, rec.w, rec.z, lo, hi, sc, W);
    if (lane == 0) S.seg_mean[s] = m;
  }
}

// leaf j of a segment: (start within the locus, length)
__device__ __forceinline__ int2 leaf_span(const SArgs& S, int len, int j) {
  const int full = len / kNpyBuf, per = lut_count(S, kNpyBuf);
  int chunk, m, jj;
  if (j < full * per) { chunk = j / per; jj = j - chunk * per; m = kNpyBuf; }
  else { chunk = full; jj = j - full * per; m = len - full * kNpyBuf; }
  const int4 e = S.lut[S.lut_off[m] + jj];
  return make_int2(chunk * kNpyBuf + e.x, e.y);
}

__global__ void k_leaf_expand(const SArgs S, int64_t n_keys) {
  int n_act_ = 0;
  lvl_counts(S, n_act_, n_keys);
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= seg_count(S, n_keys)) return;
  const int o = S.leaf_off[s], n = S.seg_nleaf[s];
  for (int j = 0; j < n; ++j) S.leaf_seg[o + j] = (int)s;
}

// One lane per leaf.  Leaves without a closed form (multi-run envelopes, ~3% of the
// partial leaves) are finished cooperatively by the wave right away: lane octet j takes
// the j-th of them, lane c of the octet its stride accumulator c, and the eight sums are
// combined as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) with xor shuffles (float addition is
// commutative, so the result is exact).  Wave-uniform loop: every lane runs the same trips.
__global__ void k_leaf(const SArgs S, int64_t n_keys) {
  int n_act_ = 0;
  lvl_counts(S, n_act_, n_keys);
  const int ns = seg_count(S, n_keys);
  const int TL = S.leaf_off[ns];
  const SortedSrc src{S.satt_lohi, S.satt_sc};
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  for (int base = wave * 64; base < TL; base += nwaves * 64) {
    const int i = base + lane;
    const bool has = i < TL;
    int4 r = make_int4(0, 0, 0, 0);
    int st = 0, ln = 0;
    double v = 0.0;
    bool runs = false;
    SegAttT<SortedSrc> at;
    if (has) {
      const int s = S.leaf_seg[i];
      r = S.seg_rec[s];
      const int2 span = leaf_span(S, r.z, i - S.leaf_off[s]);
      st = span.x; ln = span.y;
      at.load(src, r.x, r.x + r.y);
      runs = !at.leaf_fast(src, st, ln, v);
    }
    uint64_t pend = __ballot(runs);
    while (pend) {
      const int oct = lane >> 3, c = lane & 7;
      uint64_t m = pend;
      for (int k = 0; k < oct && m; ++k) m &= m - 1;
      const int src_lane = m ? __builtin_ctzll(m) : lane;
      const int okb = __shfl(r.x, src_lane, 64), ona = __shfl(r.y, src_lane, 64);
      const int ost = __shfl(st, src_lane, 64), oln = __shfl(ln, src_lane, 64);
      double acc = 0.0;
      if (m) {
        SegAttT<SortedSrc> a2;
        a2.load(src, okb, okb + ona);
        acc = a2.stride_sum(src, ost, oln >> 3, c);
      }
      acc = acc + __shfl_xor(acc, 1, 64);
      acc = acc + __shfl_xor(acc, 2, 64);
      acc = acc + __shfl_xor(acc, 4, 64);
      const int j = __popcll(pend & ((1ull << lane) - 1ull));
      const double body = __shfl(acc, (j & 7) * 8, 64);
      if (runs && j < 8) { v = at.add_tail(src, st, ln, body); runs = false; }
      for (int k = 0; k < 8 && pend; ++k) pend &= pend - 1;
    }
    if (has) S.leaf_val[i] = v;
  }
}

__device__ __forceinline__ void seg_combine_one(const SArgs& S, int s) {
  const int len = S.seg_rec[s].z;
  const double* lv = S.leaf_val + S.leaf_off[s];
  double total = 0.0;
  int j = 0;
  for (int o = 0; o < len; o += kNpyBuf) {
    const int m = min(kNpyBuf, len - o);
    const int4* lt = S.lut + S.lut_off[m];
    const int nl = lut_count(S, m);
    SumStack stk;
    for (int q = 0; q < nl; ++q, ++j) {
      stk.push(lv[j]);
      for (int a = 0; a < lt[q].z; ++a) stk.add_top();
    }
    total += stk.s0;
  }
  S.seg_mean[s] = total / (double)len;
}

// One thread per leaf-path segment, found from the leaf side (the thread of a segment's
// first leaf): a grid-stride loop over the level's leaves instead of a thread for every
// segment of the level (most of which k_seg_rec already finished).
__global__ void k_seg_combine(const SArgs S, int64_t n_keys) {
  int n_act_ = 0;
  lvl_counts(S, n_act_, n_keys);
  const int TL = S.leaf_off[seg_count(S, n_keys)];
  for (int jl = blockIdx.x * blockDim.x + threadIdx.x; jl < TL; jl += gridDim.x * blockDim.x) {
    const int s = S.leaf_seg[jl];
    if (jl != S.leaf_off[s]) continue;
    seg_combine_one(S, s);
  }
}


// ---- explain_one, one wave per contig (orgscorer.py:407-429, 585-597, 621-631) ---------
// The common case needs no gene-score matrix: the contig's segments (sorted by clade, then
// locus) are staged in LDS, per-locus maxes are LDS atomics, and each clade run scores
// itself (crit = min, rank = numpy-order mean over the unmasked loci, zeros where the clade
// has no segment).  The best option is a wave argmax by (rank, larger clade id) -- the
// sorted-order tie policy of decide_one -- and the winner's synteny is 'A' on every unmasked
// locus ('~' elsewhere), since its crit >= k1.  Contigs with more segments than the stage
// holds, more than 64 loci or --weak-loci assign-unknown (virtual "Unknown" row) go to the
// dense workgroup (k_decide<1>); contigs without a one-clade option go to explain_two.
// Upper bound of decide_contig's arena for P clade rows (segments + 1) and G loci: every
// take() of decide_contig with its 16-byte alignment, plus the mask-class workspace.
__host__ __device__ int64_t arena_bound(int64_t P, int64_t G) {
  int64_t cls = 0;
  if (P >= kClsMin) {
    int64_t n2 = 1;
    while (n2 < P) n2 <<= 1;
    cls = n2 * 8 + (P + 1) * 4 + (int64_t)kClsMaxPairs * 8 + ((int64_t)kClsMaxPairs + 1) * 8 + 64;
  }
  return 20 * 16 + P * (4 + 4 + 8 + 4 + 4 + 4 + 8 + 4) + 8 * P * G + G * (8 + 4 + 4 + 1 + 4) +
         8 * (P / 32 + 2) + cls;
}

constexpr int kOneCap = 384;

// (S_arg first: the per-contig loop re-reads the argument block through kernarg_fresh --
// held across the loop it spilled 64 SGPRs)
__global__ __launch_bounds__(64) void k_one(const SArgs S_arg, int n_act, int level,
                                            int64_t n_keys) {
  lvl_counts(S_arg, n_act, n_keys);
  __shared__ int2 s_cg[kOneCap];
  __shared__ double s_v[kOneCap];
  __shared__ double s_rank[kOneCap];     // rank of the option whose clade run starts here, or -1
  __shared__ int s_mem[kOneCap];
  __shared__ unsigned long long s_max[64];
  __shared__ unsigned long long s_head[kOneCap / 64];   // clade-run heads, one ballot per 64
  __shared__ int s_cnt;
  const int lane = threadIdx.x;
  // straight to the segment-table decision (k_big_sparse): the dense matrix cannot fit the
  // arena (or every decision is routed there; routed ones with few segments take explain_one
  // here first)
  auto straight_big = [](const SArgs& S, int G, int ns) {
    return S.sparse_on && G <= 63 &&
           (S.route_sparse || (ns > kOneCap && arena_bound(ns + 1, G) + 4096 > S.dec_lds_bytes)) &&
           !(S.route_sparse && !S.force_big && ns <= kOneCap && S.k.p.weak != 2);
  };
  // those first, a contig per lane: one list append (and one need_bytes max) per wave instead
  // of one contended atomic per contig (the cfg5 stress levels: every contig goes there)
  for (int base = blockIdx.x * 64; base < n_act; base += gridDim.x * 64) {
    const SArgs& S = kernarg_fresh<SArgs>(S_arg);
    const KArgs& K = S.k;
    const int cr = base + lane;
    bool big = false;
    int c = 0;
    int64_t need = 0;
    if (cr < n_act) {
      c = S.act ? S.act[cr] : cr;
      const int64_t l0 = K.loc_off[c];
      const int G = (int)(K.loc_off[c + 1] - l0);
      const int so = n_keys > 0 ? S.crank_first[cr] : 0;
      const int ns = (n_keys > 0 ? S.crank_first[cr + 1] : 0) - so;
      big = K.hit_off[c + 1] != K.hit_off[c] && G != 0 && straight_big(S, G, ns);
      if (big) need = arena_bound(ns + 1, G) + 4096;    // (the HBM-slot decision, should it decline)
    }
    const uint64_t bm = __ballot(big);
    if (bm) {
      const int leader = __builtin_ctzll(bm);
      unsigned long long first = 0;
      if (lane == leader) first = atomicAdd(&S.counters[2], (unsigned long long)__popcll(bm));
      const int slot = (int)__shfl((long long)first, leader, 64) + __popcll(bm & ((1ull << lane) - 1ull));
      if (big) {
        K.need[c] = need;
        S.big_list[2 * slot] = cr;
        S.big_list[2 * slot + 1] = c;
      }
      long long mx = need;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) mx = max(mx, (long long)__shfl_xor(mx, off, 64));
      if (lane == leader) atomicMax(&S.counters[3], (unsigned long long)mx);
    }
  }
  for (int cr = blockIdx.x; cr < n_act; cr += gridDim.x) {
    const SArgs& S = kernarg_fresh<SArgs>(S_arg);
    const KArgs& K = S.k;
    const DevParams& P = K.p;
    const int c = S.act ? S.act[cr] : cr;
    const int64_t l0 = K.loc_off[c];
    const int G = (int)(K.loc_off[c + 1] - l0);
    const int64_t h0 = K.hit_off[c];
    if (K.hit_off[c + 1] == h0 || G == 0) continue;       // never evaluated (orgscorer.py:959)
    const int so = n_keys > 0 ? S.crank_first[cr] : 0;
    const int ns = (n_keys > 0 ? S.crank_first[cr + 1] : 0) - so;
    if (straight_big(S, G, ns)) continue;               // (listed above)
    const bool to_sparse = S.sparse_on && G <= 63;
    // routed decisions without an explain_one option go to k_big_sparse for explain_two
    auto push_big = [&]() {
      if (lane == 0) {
        const int64_t need = arena_bound(ns + 1, G) + 4096;
        K.need[c] = need;
        const int slot = (int)atomicAdd(&S.counters[2], 1ull);
        S.big_list[2 * slot] = cr;
        S.big_list[2 * slot + 1] = c;
        atomicMax(&S.counters[3], (unsigned long long)need);
      }
    };
    if (ns > kOneCap || G > 64 || P.weak == 2 || S.force_big) {
      if (lane == 0) {
        const int slot = (int)atomicAdd(&S.counters[6], 1ull);
        S.one_list[2 * slot] = cr;
        S.one_list[2 * slot + 1] = c;
      }
      continue;
    }
    for (int t = lane; t < ns; t += 64) {
      s_cg[t] = S.seg_cg[so + t];
      s_v[t] = S.seg_mean[so + t];
    }
    s_max[lane] = 0;
    __syncthreads();
    // per-locus max over known clades (:407-411); clade-run heads
    const int nch = (ns + 63) / 64;
    for (int i = 0; i < nch; ++i) {
      const int t = 64 * i + lane;
      bool hd = false;
      if (t < ns) {
        const int2 cg = s_cg[t];
        const double v = s_v[t];
        if (cg.x != K.unknown && v > 0.0) atomicMax(&s_max[cg.y], dbits(v));
        hd = t == 0 || s_cg[t - 1].x != cg.x;
      }
      const unsigned long long hm = __ballot(hd);
      if (lane == 0) s_head[i] = hm;
    }
    __syncthreads();
    // weak loci: ignore -> mask (:420-427), penalize -> none (:413-414)
    const double mx = __longlong_as_double((long long)s_max[lane]);
    const uint64_t um = __ballot(lane < G && (P.weak != 0 || mx >= P.kmin));
    const int Gu = __popcll(um);
    if (Gu == 0) {
      if (level > 0 && lane == 0) {                       // np.min of an empty array upstream
        K.iters[c] = (int16_t)min(level + 1, 32767);
        K.status[c] = WF_E_EMPTYMASK;
      }                                                   // level 0: skipped contig (:959)
      continue;
    }
    // Contig.score of every clade run (:447-461); options have crit >= k1 (:585-597)
    double br = -__builtin_inf(), bcrit = 0.0;
    long long bk = -1;
    for (int t = lane; t < ns; t += 64) {
      double rk = -1.0;
      const int clade = s_cg[t].x;
      // a run of fewer than Gu segments misses an unmasked locus: crit 0.0 < k1 (k1 > 0),
      // no option, and its rank is never read
      bool can = t == 0 || s_cg[t - 1].x != clade;
      if (can && P.k1 > 0.0) {
        int i = t >> 6;
        unsigned long long m = s_head[i] & ((t & 63) == 63 ? 0ull : ~((2ull << (t & 63)) - 1ull));
        while (m == 0ull && ++i < nch) m = s_head[i];
        const int re = m ? 64 * i + __builtin_ctzll(m) : ns;
        can = re - t >= Gu;
      }
      if (can) {
        uint64_t m = um;
        int q = t;
        double crit = 0.0;
        bool firstv = true;
        auto next = [&]() -> double {
          const int g = __builtin_ctzll(m);
          m &= m - 1;
          while (q < ns && s_cg[q].x == clade && s_cg[q].y < g) ++q;
          const double v = (q < ns && s_cg[q].x == clade && s_cg[q].y == g) ? s_v[q] : 0.0;
          crit = (firstv || v < crit) ? v : crit;
          firstv = false;
          return v;
        };
        const double rank = (0.0 + np_sum_seq(Gu, next)) / (double)Gu;
        if (crit >= P.k1) {
          rk = rank;
          if (better(rank, clade, br, bk)) { br = rank; bk = clade; bcrit = crit; }
        }
      }
      s_rank[t] = rk;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double r2 = __shfl_xor(br, off, 64), c2 = __shfl_xor(bcrit, off, 64);
      const long long k2 = __shfl_xor(bk, off, 64);
      if (better(r2, k2, br, bk)) { br = r2; bk = k2; bcrit = c2; }
    }
    if (bk < 0) {                                          // explain_two (:570)
      if (to_sparse && S.route_sparse) {
        push_big();
        continue;
      }
      if (lane == 0) {
        const int slot = (int)atomicAdd(&S.counters[5], 1ull);
        S.two_list[2 * slot] = cr;
        S.two_list[2 * slot + 1] = c;
      }
      continue;
    }
    // meld_one (:621-631): options within --range of the best
    if (lane == 0) s_cnt = 0;
    __syncthreads();
    if (P.dis1 == 1)
      for (int t = lane; t < ns; t += 64) {
        const double rk = s_rank[t];
        if (rk >= 0.0 && (br - rk) <= P.range) s_mem[atomicAdd(&s_cnt, 1)] = s_cg[t].x;
      }
    __syncthreads();
    const int nm = s_cnt;
    if (P.dis1 == 1 && nm == 0) {                          // negative --range upstream crash
      if (lane == 0) K.status[c] = WF_E_BADINPUT;
      continue;
    }
    int lca = (int)bk;
    if (P.dis1 == 1) {
      int acc = -1;
      for (int i = lane; i < nm; i += 64) acc = lca2(K, acc, s_mem[i]);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) acc = lca2(K, acc, __shfl_xor(acc, off, 64));
      lca = acc;
    }
    const int64_t mbase = 2 * h0 + 2 * (int64_t)c;
    for (int i = lane; i < nm; i += 64) K.meld[mbase + i] = s_mem[i];
    if (lane < G) K.syn[l0 + lane] = ((um >> lane) & 1ull) ? 'A' : '~';   // set_synteny_one
    if (lane == 0) {
      K.call[c] = WF_CALL_NO_LGT;
      K.crit[c] = bcrit;
      K.rank[c] = br;
      K.c1[c] = lca;
      K.c2[c] = -1;
      K.nm1[c] = nm;
      K.iters[c] = (int16_t)(level + 1);
      if (level == 0) K.pair_evals[c] = 0;
    }
    __syncthreads();                                       // LDS reuse by the next contig
  }
}

// Decision workgroup for one contig at one level.  Builds the gene-score matrix of the
// level (rows = clades in id order, the virtual "Unknown" row of --weak-loci
// assign-unknown included) from the contig's segments, then runs decide_level.
// Returns false when the arena is too small (caller hands the contig to the HBM tier).
// PHASE 0: the whole level (HBM-slot tier); 1: prologue + explain_one, contigs without a
// one-clade explanation are queued for phase 2; 2: prologue + explain_two + roll-up.
template <int NT, int PHASE>
__device__ __forceinline__ bool decide_contig(const SArgs& S, int c, int cr, int level, char* abase, int64_t acap,
                              Ctl& ctl, int64_t n_keys, bool in_lds = true) {
  const KArgs& K = S.k;
  const DevParams& P = K.p;
  const int tid = threadIdx.x;
  const int64_t h0 = K.hit_off[c];
  const int H = (int)(K.hit_off[c + 1] - h0);
  Contig C;
  C.l0 = K.loc_off[c];
  C.G = (int)(K.loc_off[c + 1] - C.l0);
  C.h0 = h0;
  C.H = H;
  C.mbase = 2 * h0 + 2 * (int64_t)c;
  const int G = C.G;
  if (H == 0 || G == 0) return true;            // never evaluated (orgscorer.py:959)
  STAMP_INIT();
  if (tid == 0) {
    ctl.status = 0;
    ctl.p_unk = -1;
  }
  const int so = n_keys > 0 ? S.crank_first[cr] : 0;
  const int se = n_keys > 0 ? S.crank_first[cr + 1] : 0;
  const int ns = se - so;
  __syncthreads();
  const int Pmax = ns + 1;
  Arena ar{abase, acap, 0};
  C.cl_id = ar.take<int>(Pmax);
  C.S = ar.take<double>((int64_t)Pmax * G);
  C.maxes = ar.take<uint64_t>(G);
  C.ign = ar.take<int>(G);
  C.um = ar.take<int>(G);
  C.pot = ar.take<int>(Pmax);
  C.mask = ar.take<uint64_t>(Pmax);
  C.mem1 = ar.take<int>(Pmax);
  C.mem2 = ar.take<int>(Pmax);
  C.bm1 = ar.take<unsigned>((Pmax + 31) / 32);
  C.bm2 = ar.take<unsigned>((Pmax + 31) / 32);
  C.best_syn = ar.take<uint8_t>(G);
  C.loc_len = ar.take<int>(G);                  // ambiguous fraction weights (orgscorer.py:693-702)
  C.sib_of = ar.take<int>(Pmax);
  if (P.sister_on && G <= 64) C.hm = ar.take<uint64_t>(Pmax);
  int* seg_ci = ar.take<int>(ns + 1);
  if (Pmax >= kClsMin) {                         // mask classes for a large explain_two
    C.xcap = cls_bytes(Pmax);
    C.xws = ar.take<char>(C.xcap);
  }
  // routed decisions go to k_big_sparse -- unless it would decline them (> 63 loci: the
  // segment-table form's locus masks), then the arena decides here
  if (!ar.fits() || (in_lds && S.route_sparse && G <= 63)) {
    if (tid == 0) K.need[c] = ar.used + 4096;
    __syncthreads();
    return false;
  }
  for (int g = tid; g < G; g += NT) {
    const int ls = K.lstart[C.l0 + g], le = K.lend[C.l0 + g];
    C.loc_len[g] = max(ls, le) - min(ls, le) + 1;
  }
  const uint64_t cmask = (1ull << S.key_tb) - 1;
  (void)cmask;
  auto clade_of = [&](int s) { return S.seg_cg[s].x; };
  // clade list = distinct clades of the segments (sorted by id = name order)
  const int per = (ns + NT - 1) / NT;
  const int b = min(ns, tid * per), e = min(ns, b + per);
  int nc = 0;
  for (int t = b; t < e; ++t)
    if (t == 0 || clade_of(so + t) != clade_of(so + t - 1)) ++nc;
  int Pn;
  int ci = block_scan<NT>(nc, &Pn, ctl) - 1;
  for (int t = b; t < e; ++t) {
    const int cl = clade_of(so + t);
    if (t == 0 || cl != clade_of(so + t - 1)) {
      ++ci;
      C.cl_id[ci] = cl;
      if (cl == K.unknown) ctl.p_unk = ci;
    }
    seg_ci[t] = ci;
  }
  __syncthreads();
  if (P.weak == 2 && ctl.p_unk < 0) {            // virtual "Unknown" row (orgscorer.py:416-418)
    if (tid == 0) {
      int pos = 0;
      while (pos < Pn && C.cl_id[pos] < K.unknown) ++pos;
      for (int q = Pn; q > pos; --q) C.cl_id[q] = C.cl_id[q - 1];
      C.cl_id[pos] = K.unknown;
      ctl.p_unk = pos;
    }
    __syncthreads();
    const int pos = ctl.p_unk;
    for (int t = tid; t < ns; t += NT)
      if (seg_ci[t] >= pos) seg_ci[t] += 1;
    ++Pn;
  }
  for (int i = tid; i < Pn * G; i += NT) C.S[i] = 0.0;
  __syncthreads();
  for (int t = tid; t < ns; t += NT) {
    C.S[(int64_t)seg_ci[t] * G + S.seg_cg[so + t].y] = S.seg_mean[so + t];
  }
  __syncthreads();
  STAMP(7);
  const int iteration = level + 1;
  bool first = level == 0;
  int64_t pair_evals = level == 0 ? 0 : K.pair_evals[c];
  int dec;
  if (PHASE == 0) {
    dec = decide_level<NT>(K, C, ctl, c, Pn, iteration, first, pair_evals);
  } else {
    dec = decide_prologue<NT>(K, C, ctl, Pn, first);
    if (PHASE == 1 && dec == kDecNext) {
      dec = decide_one<NT>(K, C, ctl, c, Pn, iteration, pair_evals);
      if (dec == kDecNext) {
        if (tid == 0) {
          const int slot = (int)atomicAdd(&S.counters[5], 1ull);
          S.two_list[2 * slot] = cr;
          S.two_list[2 * slot + 1] = c;
        }
        return true;
      }
    } else if (PHASE == 2 && dec == kDecNext) {
      dec = decide_two<NT>(K, C, ctl, c, Pn, iteration, pair_evals);
    }
  }
  if (dec == kDecDone) return true;
  if (dec == kDecRaise && iteration + 1 <= kMaxIter) {
    // roll up (orgscorer.py:431-445): this contig's attachments move to the parent clade
    const int64_t a0 = S.catt_off[c], a1 = S.catt_off[c + 1];
    if (tid == 0) {
      // slot (high 24 bits) and attachment base (low 40) from ONE atomic, so the bases of
      // the next level ascend with the rank (the per-contig sort relies on it)
      const unsigned long long old =
          atomicAdd(&S.counters[0], (1ull << 40) | (unsigned long long)(a1 - a0));
      const int slot = (int)(old >> 40);
      S.act_next[slot] = c;
      S.act_base_next[slot] = (int64_t)(old & ((1ull << 40) - 1));
      K.pair_evals[c] = pair_evals;
    }
    // re-key to the parent clade, 4 attachments per lane in flight (two dependent loads each)
    for (int64_t ab = a0; ab < a1; ab += 4 * NT) {
      int cl[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t a = ab + r * NT + tid;
        cl[r] = a < a1 ? S.att_clade[a] : 0;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) cl[r] = K.parent[cl[r]];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t a = ab + r * NT + tid;
        if (a < a1) S.att_clade[a] = cl[r];
      }
    }
    STAMP_SYNC();
    STAMP(19);
    return true;
  }
  if (tid == 0) {                                // unclassified after evaluation
    const int it = dec == kDecRaise ? iteration + 1 : iteration;
    K.iters[c] = (int16_t)min(it, 32767);
    K.pair_evals[c] = pair_evals;
    K.status[c] = dec == kDecRaise ? WF_E_RUNAWAY : ctl.status;
  }
  return true;
}

constexpr int kDecNT = 64;   // one wave per contig decision: no cross-wave barriers

template <int PHASE, int NT = kDecNT>
__global__ __launch_bounds__(NT, 2) void k_decide(const SArgs S, int n_act,
                                                   int level, int64_t n_keys) {
  lvl_counts(S, n_act, n_keys);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ Ctl ctl;
  if constexpr (PHASE == 3) {
    // one launch for both lists: the contigs k_one handed over get the whole level
    // (PHASE 0 logic), the contigs it left open get explain_two (PHASE 2)
    const int c1 = (int)S.counters[6], c2 = (int)S.counters[5];
    for (int i = blockIdx.x; i < c1 + c2; i += gridDim.x) {
      const bool whole = i < c1;
      const int32_t* L = whole ? S.one_list : S.two_list;
      const int j = whole ? i : i - c1;
      const int cr = L[2 * j], c = L[2 * j + 1];
      const bool ok = whole ? decide_contig<NT, 0>(S, c, cr, level, smem, S.dec_lds_bytes, ctl, n_keys)
                            : decide_contig<NT, 2>(S, c, cr, level, smem, S.dec_lds_bytes, ctl, n_keys);
      if (!ok && threadIdx.x == 0) {
        const int slot = (int)atomicAdd(&S.counters[2], 1ull);
        S.big_list[2 * slot] = cr;
        S.big_list[2 * slot + 1] = c;
        atomicMax(&S.counters[3], (unsigned long long)S.k.need[c]);
      }
      __syncthreads();
    }
  } else {
  const int32_t* list = PHASE == 1 ? S.one_list : S.two_list;
  const int count = PHASE == 1 ? (list ? (int)S.counters[6] : n_act) : (int)S.counters[5];
  for (int i = blockIdx.x; i < count; i += gridDim.x) {
    const int cr = list ? list[2 * i] : i;
    const int c = list ? list[2 * i + 1] : (S.act ? S.act[cr] : cr);
    const bool ok = decide_contig<NT, PHASE>(S, c, cr, level, smem, S.dec_lds_bytes, ctl, n_keys);
    if (!ok && threadIdx.x == 0) {
      const int slot = (int)atomicAdd(&S.counters[2], 1ull);
      S.big_list[2 * slot] = cr;
      S.big_list[2 * slot + 1] = c;
      atomicMax(&S.counters[3], (unsigned long long)S.k.need[c]);
    }
    __syncthreads();
  }
  }
}

// The dense decision in an HBM slot: the contigs k_big_sparse declined (big2_list,
// counters[1]), or every contig of big_list (counters[2]) when the sparse form is off.
__global__ __launch_bounds__(kBlock, 2) void k_decide_big(const SArgs S, int level,
                                                          int64_t n_keys, int use2) {
  int n_act_ = 0;
  lvl_counts(S, n_act_, n_keys);
  const int count = (int)S.counters[use2 ? 1 : 2];
  const int32_t* list = use2 ? S.big2_list : S.big_list;
  __shared__ Ctl ctl;
  char* base = S.k.big_ws + (int64_t)blockIdx.x * S.k.slot_bytes;
  for (int i = blockIdx.x; i < count; i += gridDim.x) {
    const int cr = list[2 * i], c = list[2 * i + 1];
    const bool ok = decide_contig<kBlock, 0>(S, c, cr, level, base, S.k.slot_bytes, ctl, n_keys, false);
    if (!ok && threadIdx.x == 0) S.k.status[c] = WF_E_NOMEM;
    __syncthreads();
  }
}

#include "wf_sparse.h"
WF_STAMP_READER(sparse, g_sstamps, 16)
WF_STAMP_READER(big, g_bstamps, 48)

int bits_for(int64_t v) {   // bits to hold values 0..v
  int b = 1;
  while (b < 62 && (int64_t(1) << b) <= v) ++b;
  return b;
}

// Device scratch owned by one context's StagedState.  `drain` is the stream the context's
// kernels run on: it is drained before an allocation is replaced (queued kernels may still
// use the old one).  Per call, never a process global: contexts on different host threads
// must not drain -- or race on -- each other's streams.
struct Buf {
  void* p = nullptr;
  size_t n = 0;
  ~Buf() { if (p) (void)hipFree(p); }
  hipError_t ensure(hipStream_t drain, size_t bytes) {
    if (bytes <= n) return hipSuccess;
    if (p) {
      hipError_t e = hipStreamSynchronize(drain);
      if (e != hipSuccess) return e;
      (void)hipFree(p);
      p = nullptr;
      n = 0;
    }
    size_t want = std::max<size_t>(bytes + bytes / 4, 256);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) n = want;
    return e;
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

}  // namespace


// The roll-up launches of the first wave form and its level-0 launch over the triage's list
// take their contigs from a work-queue counter (a static XCD order left a few waves finishing
// last: roll-up 4.98 -> 4.35, list 2.36 -> 2.00 ms, r5j / r5k).  Levels whose largest contig
// has 4,097..8,192 attachments sort per contig in LDS (k_sort_radix), not with the device
// radix sort of the whole level.

struct StagedState {
  int device = 0;
  int cus = 256;
  Buf lut_off, lut, cnt, att_off, counters, pinned_dummy;
  Buf att_lo, att_hi, att_loc, att_clade, att_hit, att_sc;
  Buf keys0, keys1, vals0, vals1, flags, seg_id, seg_start, seg_crank, seg_mean;
  Buf cnt_leaves, red, seg_nleaf, leaf_off, leaf_seg, leaf_val, annot_best;
  Buf seg_rec, seg_cg, crank_first, satt_lohi, satt_sc, wave_list, lvl_ctr, seg_cnt, seg_len;
  Buf front;                      // k_front_radix: ticket, leaf count, per-rank look-back words
  Buf span_cnt, spans;                              // --write-details only
  unsigned long long* host_lvl = nullptr;         // pinned: count word of each level
  hipEvent_t lvl_ev[2] = {nullptr, nullptr};
  int sparse_big = 3;                // WF_OPT_SPARSE_BIG (2 all, 3 the open decisions; 0/1 retired)
  int sparse_res = -1;               // resident k_big_sparse waves per CU
  int two_res = -1;                  // resident k_dump_sparse<1> (compact tables) waves per CU
  int64_t att_limit = (int64_t(1) << 31) - 1;   // attachments per call (WF_OPT_ATT_LIMIT)
  int64_t dump_cap = 0;              // WF_OPT_DUMP_CAP (0: max(32 N, 65536))
  int triage = 1;                    // WF_OPT_TRIAGE: level-0 triage before the first wave form
  Buf tri_list, tri_cnt;             // the contigs the triage hands on, and their count
  Buf wq;                            // roll-up launches' work-queue counters
  Buf roll0, roll1, roll_cnt, anc;   // wave levels: contig lists, per-level counts, ancestors
  // per-phase timing (wf_phase): event pool, this call's spans (phase, begin, end)
  bool timing = false;
  std::vector<hipEvent_t> tev;
  int tev_used = 0;
  std::vector<int> tspans;
  double phase_ms[8] = {0};
  int64_t phase_n[8] = {0};
  Buf act0, act1, base0, base1, big_list, big2_list, two_list, one_list, big_ws, tmp, pend, act_l0;
  Buf sp_ws;                        // k_big_sparse scratch (kSpSlot per wave)
  Buf hkey;                         // wf_batch.hit_key when the caller passed none
  Buf dump_cg, dump_mean, dump_first, dump_list, dump_ctr, dump_um;   // hand-over (k_dump_sparse)
  bool level0 = true;               // wave kernels (wf_fast.hip) before the staged kernels
  bool rollup = false;              // ... carrying the roll-up levels too
  bool lut_ready = false;
  int64_t dec_lds = 32 * 1024;       // decision arena (grows with the data, see staged_score)
  bool dec_lds_fixed = false;        // set by wf_set_lds_bytes / WF_DEC_LDS
  unsigned long long* host_counters = nullptr;   // pinned
  // host-coherent mailbox: k_publish writes counts + a sequence word, the host spins on it
  unsigned long long* mbox = nullptr;
  unsigned long long* mbox_dev = nullptr;
  unsigned long long mbox_seq = 0;
  ~StagedState() {
    for (hipEvent_t e : tev) (void)hipEventDestroy(e);
    if (mbox) (void)hipHostFree(mbox);
    if (host_counters) (void)hipHostFree(host_counters);
    if (host_lvl) (void)hipHostFree(host_lvl);
    for (hipEvent_t e : lvl_ev)
      if (e) (void)hipEventDestroy(e);
  }
};

StagedState* staged_create(int device) {
  StagedState* st = new StagedState();
  st->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) st->cus = prop.multiProcessorCount;
  if (hipHostMalloc(reinterpret_cast<void**>(&st->host_counters), 16 * sizeof(unsigned long long)) != hipSuccess)
    st->host_counters = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&st->host_lvl), (kMaxIter + 2) * sizeof(unsigned long long)) !=
      hipSuccess)
    st->host_lvl = nullptr;
  for (hipEvent_t& e : st->lvl_ev)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) e = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&st->mbox), 16 * sizeof(unsigned long long),
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&st->mbox_dev), st->mbox, 0) != hipSuccess) {
    if (st->mbox) (void)hipHostFree(st->mbox);
    st->mbox = nullptr;
    st->mbox_dev = nullptr;
  }
  return st;
}

void staged_destroy(StagedState* st) { delete st; }

void staged_set_level0(StagedState* st, bool on, bool rollup) {
  st->level0 = on;
  st->rollup = rollup;
}

void staged_set_lds(StagedState* st, int64_t bytes) {
  st->dec_lds = bytes;
  st->dec_lds_fixed = true;
}

void staged_set_options(StagedState* st, int sparse_big, int64_t att_limit, int64_t dump_cap, int triage) {
  st->triage = triage;
  st->sparse_big = sparse_big;
  st->att_limit = att_limit;
  st->dump_cap = dump_cap;
}

void staged_timing(StagedState* st, bool on) {
  st->timing = on;
  for (int i = 0; i < 8; ++i) { st->phase_ms[i] = 0.0; st->phase_n[i] = 0; }
}

void staged_timing_read(const StagedState* st, double* ms, int64_t* spans, int n) {
  for (int i = 0; i < n && i < 8; ++i) { ms[i] = st->phase_ms[i]; spans[i] = st->phase_n[i]; }
}

// An event recorded on `s` (from the context's pool); -1 when timing is off or it failed.
static int t_mark(StagedState* st, hipStream_t s) {
  if (!st->timing) return -1;
  if (st->tev_used == (int)st->tev.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return -1;
    st->tev.push_back(e);
  }
  const int i = st->tev_used;
  if (hipEventRecord(st->tev[i], s) != hipSuccess) return -1;
  ++st->tev_used;
  return i;
}

static void t_span(StagedState* st, int phase, int b, int e) {
  if (b < 0 || e < 0) return;
  st->tspans.push_back(phase);
  st->tspans.push_back(b);
  st->tspans.push_back(e);
}

// this call's spans into the accumulators (the events are complete once the stream is)
static hipError_t t_collect(StagedState* st, hipStream_t s) {
  if (st->tspans.empty()) { st->tev_used = 0; return hipSuccess; }
  hipError_t e = hipStreamSynchronize(s);
  for (size_t i = 0; e == hipSuccess && i + 2 < st->tspans.size(); i += 3) {
    float ms = 0.f;
    e = hipEventElapsedTime(&ms, st->tev[st->tspans[i + 1]], st->tev[st->tspans[i + 2]]);
    st->phase_ms[st->tspans[i]] += ms;
    st->phase_n[st->tspans[i]] += 1;
  }
  st->tspans.clear();
  st->tev_used = 0;
  return e;
}

#define ST_TRY(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) { *err = std::string(#x) + ": " + hipGetErrorString(e_); return -2; } \
  } while (0)

static int build_lut(StagedState* st, hipStream_t s, std::string* err) {
  if (st->lut_ready) return 0;
  ST_TRY(st->lut_off.ensure(s, (kNpyBuf + 2) * sizeof(int32_t)));
  Buf counts;
  ST_TRY(counts.ensure(s, (kNpyBuf + 2) * sizeof(int32_t)));
  hipLaunchKernelGGL(k_lut_count, dim3((kNpyBuf + 256) / 256), dim3(256), 0, s, counts.as<int32_t>());
  ST_TRY(hipGetLastError());
  std::vector<int32_t> h(kNpyBuf + 2, 0);
  ST_TRY(hipMemcpyAsync(h.data(), counts.p, (kNpyBuf + 1) * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  ST_TRY(hipStreamSynchronize(s));
  std::vector<int32_t> off(kNpyBuf + 2, 0);
  for (int n = 0; n <= kNpyBuf; ++n) off[n + 1] = off[n] + h[n];
  ST_TRY(st->lut.ensure(s, (size_t)off[kNpyBuf + 1] * sizeof(int4)));
  ST_TRY(hipMemcpyAsync(st->lut_off.p, off.data(), (kNpyBuf + 2) * sizeof(int32_t), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_lut_fill, dim3((kNpyBuf + 256) / 256), dim3(256), 0, s, st->lut_off.as<int32_t>(),
                     st->lut.as<int4>());
  ST_TRY(hipGetLastError());
  ST_TRY(hipStreamSynchronize(s));
  st->lut_ready = true;
  return 0;
}

static inline unsigned grid_for(int64_t n, int block = 256) {
  return (unsigned)std::max<int64_t>(1, (n + block - 1) / block);
}

// Runs the whole path for one batch on stream `s` (synchronising on it between levels).
// `k` carries device pointers for batch, taxonomy, params and results.
// Host waits inside a pass: an event polled in a loop wakes the host within microseconds,
// where a blocking stream synchronisation took tens of microseconds per level.
// Exclusive scan of n ints by one workgroup (per-contig segment counts -> first segment):
// one launch with no host-side temp-storage query, where the device scan costs two
// launches and a host call that is slower than the scan itself.  Thread t owns a
// contiguous chunk; the chunk sums are scanned in LDS.
constexpr int kScanNT = 1024;
__global__ __launch_bounds__(kScanNT) void k_scan_small(const int32_t* in, int32_t* out, int n) {
  __shared__ int s_part[kScanNT];
  const int t = threadIdx.x;
  const int per = (n + kScanNT - 1) / kScanNT;
  const int b = min(n, t * per), e = min(n, b + per);
  int sum = 0;
  for (int i = b; i < e; ++i) sum += in[i];
  s_part[t] = sum;
  __syncthreads();
  for (int off = 1; off < kScanNT; off <<= 1) {
    const int v = t >= off ? s_part[t - off] : 0;
    __syncthreads();
    s_part[t] += v;
    __syncthreads();
  }
  int run = s_part[t] - sum;
  for (int i = b; i < e; ++i) {
    const int x = in[i];
    out[i] = run;
    run += x;
  }
}

// Counts to the host without a copy dispatch or an event: one thread stores them into the
// host-coherent mailbox, then (system-scope release) the sequence word the host spins on.
__global__ void k_publish(unsigned long long* box, unsigned long long seq,
                          const unsigned long long* a, int na, const unsigned long long* b, int nb) {
  if (threadIdx.x != 0) return;
  for (int i = 0; i < na; ++i) box[i] = a[i];
  for (int i = 0; i < nb; ++i) box[na + i] = b[i];
  __threadfence_system();
  __hip_atomic_store(&box[15], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static hipError_t publish_sync(StagedState* st, hipStream_t s, const void* a, int na, const void* b, int nb,
                               unsigned long long* out) {
  const unsigned long long seq = ++st->mbox_seq;
  hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, s, st->mbox_dev, seq,
                     static_cast<const unsigned long long*>(a), na,
                     static_cast<const unsigned long long*>(b), nb);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  volatile unsigned long long* box = st->mbox;
  for (unsigned it = 1; box[15] != seq; ++it) {
    if ((it & 4095u) == 0) {           // a failed stream must not spin forever
      e = hipStreamQuery(s);
      if (e != hipSuccess && e != hipErrorNotReady) return e;
      if (e == hipSuccess && box[15] != seq) return hipErrorUnknown;
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  for (int i = 0; i < na + nb; ++i) out[i] = box[i];
  return hipSuccess;
}

static hipError_t spin_sync(hipStream_t s, hipEvent_t ev) {
  hipError_t e = hipEventRecord(ev, s);
  if (e != hipSuccess) return e;
  while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
  }
  return e;
}

// --write-details: this level's evaluated contigs and segment records (gene scores =
// segment means, spans from k_seg_spans) to the host.  Synchronous; diagnostic output.
static hipError_t details_level(StagedState* st, const SArgs& sa, int level, int n_act, int64_t n_keys,
                                hipStream_t s, DetailsSink* det) {
  det->levels.emplace_back();
  DetailsLevel& L = det->levels.back();
  L.level = level;
  L.act.resize((size_t)n_act);
  hipError_t e = hipSuccess;
  if (level == 0) {
    for (int i = 0; i < n_act; ++i) L.act[i] = i;
  } else if (n_act > 0) {
    e = hipMemcpyAsync(L.act.data(), sa.act, (size_t)n_act * 4, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
  }
  int ns = 0;
  if (n_keys > 0) {
    e = hipMemcpyAsync(&ns, sa.seg_id + n_keys - 1, 4, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
  }
  e = hipStreamSynchronize(s);
  if (e != hipSuccess || ns == 0) return e;
  L.seg_start.resize((size_t)ns + 1);
  L.seg_crank.resize(ns);
  L.seg_cg.resize(2 * (size_t)ns);
  L.seg_mean.resize(ns);
  L.span_cnt.resize(ns);
  L.spans.resize(2 * (size_t)n_keys);
  const struct { void* dst; const void* src; size_t n; } cp[] = {
      {L.seg_start.data(), sa.seg_start, ((size_t)ns + 1) * 4},
      {L.seg_crank.data(), sa.seg_crank, (size_t)ns * 4},
      {L.seg_cg.data(), sa.seg_cg, (size_t)ns * 8},
      {L.seg_mean.data(), sa.seg_mean, (size_t)ns * 8},
      {L.span_cnt.data(), st->span_cnt.p, (size_t)ns * 4},
      {L.spans.data(), st->spans.p, (size_t)n_keys * 8}};
  for (const auto& c : cp) {
    e = hipMemcpyAsync(c.dst, c.src, c.n, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) return e;
  }
  return hipStreamSynchronize(s);
}


// ---- the contigs the wave kernels hand over (wf_fast.hip) -------------------------------
// pend[c]: 0 finished there, 1 staged from level 0, 2 evaluated and raised at level 0 there:
// a seed of staged level 1 (its attachments re-keyed here, its pair count in K.pair_evals).
struct PendIs {
  int v;
  __host__ __device__ bool operator()(int32_t p) const { return p == v; }
};
// pend 1 (staged from level 0) with at most `cap` attachments (the second wave form's slice)
struct PendFits {
  const int32_t* pend;
  const int64_t* cnt;
  int64_t cap;
  __host__ __device__ bool operator()(int i) const { return pend[i] == 1 && cnt[i] <= cap; }
};

// attachments of list[i] (0 at and past the device count *n): the exclusive scan of it gives
// each listed contig's compact key base, and its element N the list's key total
struct ListAtt {
  const int32_t* list;
  const int64_t* cnt;
  const int64_t* n;
  __host__ __device__ int64_t operator()(int i) const { return i < *n ? cnt[list[i]] : 0; }
};

__global__ void k_seed_info(int64_t* red, const int64_t* base0, const int64_t* base1, int n) {
  if (threadIdx.x == 0) {
    red[6] = base0[n];
    red[7] = base1[n];
  }
}

__global__ void k_set_word(unsigned long long* p, unsigned long long v) {
  if (threadIdx.x == 0) *p = v;
}

// the seeds' attachments to the parent clade (what the staged level 0 does on a raise)
__global__ void k_rekey_seeds(const int32_t* list, int n, const int64_t* catt_off, int32_t* att_clade,
                              const int32_t* parent) {
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const int c = list[i];
    const int64_t a1 = catt_off[c + 1];
    for (int64_t a = catt_off[c] + threadIdx.x; a < a1; a += blockDim.x) att_clade[a] = parent[att_clade[a]];
  }
}

// resident one-wave workgroups per CU of the segment-table kernels (k_big_sparse,
// k_dump_sparse: the same sp_level body) from the kernel's own VGPR and LDS use (the
// occupancy query returned 4 here: SQ_WAVES of the round-3 cfg5 profile): waves per SIMD =
// 512 / VGPRs (granule 8, at most 8), 4 SIMDs; LDS 160 KB per CU
static int resident_waves(const void* fn) {
  hipFuncAttributes fa{};
  int b = 8;
  if (hipFuncGetAttributes(&fa, fn) == hipSuccess) {
    const int vg = std::max(8, (fa.numRegs + 7) & ~7);
    const int by_vgpr = 4 * std::min(8, 512 / vg);
    const int by_lds = (int)((160 * 1024) / std::max<size_t>(1, fa.sharedSizeBytes));
    b = std::max(1, std::min(by_vgpr, by_lds));
  }
  return b;
}

static int sparse_waves(StagedState* st) {
  if (st->sparse_res < 0) st->sparse_res = resident_waves(reinterpret_cast<const void*>(&k_big_sparse));
  return st->sparse_res;
}

static int two_waves(StagedState* st) {
  if (st->two_res < 0) st->two_res = resident_waves(reinterpret_cast<const void*>(&k_dump_sparse<1>));
  return st->two_res;
}

template <class It>
static hipError_t scan_list(StagedState* st, hipStream_t s, It in, int64_t* out, int n) {
  size_t ts = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, ts, in, out, n, s);
  if (e != hipSuccess) return e;
  e = st->tmp.ensure(s, ts);
  if (e != hipSuccess) return e;
  ts = st->tmp.n;
  return hipcub::DeviceScan::ExclusiveSum(st->tmp.p, ts, in, out, n, s);
}

template <class Flags>
static hipError_t select_list(StagedState* st, hipStream_t s, Flags flags, int32_t* out, int64_t* count, int n) {
  size_t ts = 0;
  hipError_t e = hipcub::DeviceSelect::Flagged(nullptr, ts, hipcub::CountingInputIterator<int32_t>(0), flags, out,
                                               count, n, s);
  if (e != hipSuccess) return e;
  e = st->tmp.ensure(s, ts);
  if (e != hipSuccess) return e;
  ts = st->tmp.n;
  return hipcub::DeviceSelect::Flagged(st->tmp.p, ts, hipcub::CountingInputIterator<int32_t>(0), flags, out,
                                       count, n, s);
}

static int staged_run(StagedState* st, const KArgs& k, int n_tax, int max_loci, int max_hits, int64_t NH,
                      int64_t NL, hipStream_t s, std::string* err, DetailsSink* det) {
  const int N = k.n_contigs;
  if (N <= 0) return 0;
  if (!st->host_counters || !st->host_lvl || !st->lvl_ev[0] || !st->lvl_ev[1]) {
    *err = "pinned host allocation / event creation failed";
    return -2;
  }
  int rc = build_lut(st, s, err);
  if (rc) return rc;
  int64_t* hc = reinterpret_cast<int64_t*>(st->host_counters);   // pinned
  if (NH >= (int64_t(1) << 31) - 1) { *err = "too many hits for one batch (split it)"; return -1; }

  SArgs sa{};
  sa.k = k;
  sa.n_hits_i = (int)NH;
  sa.key_lb = bits_for(std::max(max_loci, 1));
  sa.key_tb = bits_for(std::max(n_tax, 1));
  sa.lut_off = st->lut_off.as<int32_t>();
  sa.lut = st->lut.as<int4>();
  sa.dec_lds_bytes = st->dec_lds;
  sa.force_big = st->sparse_big == 2 ? 1 : 0;
  sa.route_sparse = st->sparse_big >= 2 ? 1 : 0;
  sa.sparse_on = st->sparse_big != 0 ? 1 : 0;
  // kernels take SArgs by value (kernarg segment): no argument uploads, and the pointers
  // loaded from it are known to be global (global_* instead of flat_* memory operations)
  ST_TRY(st->counters.ensure(s, 8 * sizeof(unsigned long long)));
  sa.counters = st->counters.as<unsigned long long>();

  // contigs, hits -> attachments (per-contig counts, offsets, then the attachments)
  ST_TRY(st->cnt.ensure(s, (size_t)(N + 1) * sizeof(int64_t)));
  ST_TRY(st->cnt_leaves.ensure(s, (size_t)(N + 1) * sizeof(int64_t)));
  ST_TRY(st->att_off.ensure(s, (size_t)(N + 1) * sizeof(int64_t)));
  ST_TRY(st->red.ensure(s, 8 * sizeof(int64_t)));
  sa.catt_off = st->att_off.as<int64_t>();
  const unsigned agrid = (unsigned)std::min<int64_t>(N, (int64_t)st->cus * 32);   // waves per CU
  ST_TRY(hipMemsetAsync(st->red.p, 0, 8 * sizeof(int64_t), s));
  ST_TRY(hipMemsetAsync(st->cnt.as<int64_t>() + N, 0, sizeof(int64_t), s));
  ST_TRY(hipMemsetAsync(st->cnt_leaves.as<int64_t>() + N, 0, sizeof(int64_t), s));
  // Fused level 0 (wf_fast.hip) unless --write-details (per-level records of every contig)
  // or HBM annotation slots are needed.
  // (the wave kernels' 32-bit keys hold clade ids below 2^17)
  const bool level0 = st->level0 && !det && (int64_t)max_loci * k.n_sys <= kAnnSlots && sa.key_tb <= 17;
  hipLaunchKernelGGL(k_init, dim3(grid_for(N)), dim3(256), 0, s, sa.k);
  int t_waves = level0 ? t_mark(st, s) : -1;          // (the waves span: the wave launches alone)
  if (level0) {
    ST_TRY(st->pend.ensure(s, (size_t)N * 4));
    ST_TRY(st->act0.ensure(s, (size_t)N * 4));
    // The first form hands the contigs it leaves at explain_two (or at an unproven
    // assign-unknown row) over with their level-0 segment tables, every mean evaluated:
    // k_dump_sparse decides them from the table (pend 3 -> 0, 2 or 1)
    const bool dump = st->sparse_big != 0 && !st->rollup;
    // Wave levels: the first form also decides explain_two and carries the roll-up levels,
    // one launch per level over the contigs the level before raised
    const bool levels = dump;
    SArgs da = sa;
    unsigned long long* rcnt = nullptr;              // [kMaxIter + 2] per-level list counts, fail count
    if (dump) {
      int64_t cap = std::min<int64_t>(std::max<int64_t>((int64_t)N * 32, 1 << 16), (1ll << 31) - 4096);
      if (st->dump_cap > 0) cap = st->dump_cap;      // WF_OPT_DUMP_CAP (tests: the overflow branch)
      ST_TRY(st->dump_cg.ensure(s, (size_t)cap * 8)); ST_TRY(st->dump_mean.ensure(s, (size_t)cap * 8));
      ST_TRY(st->dump_first.ensure(s, ((size_t)N + 1) * 4)); ST_TRY(st->dump_list.ensure(s, (size_t)N * 8));
      ST_TRY(st->dump_ctr.ensure(s, 16));
      ST_TRY(hipMemsetAsync(st->dump_ctr.p, 0, 16, s));
      da.dump_cap = cap;
      da.dump_cg = st->dump_cg.as<int2>(); da.dump_mean = st->dump_mean.as<double>();
      da.dump_first = st->dump_first.as<int32_t>(); da.dump_list = st->dump_list.as<int32_t>();
      da.dump_ctr = st->dump_ctr.as<unsigned long long>();
      if (levels) {
        ST_TRY(st->dump_um.ensure(s, (size_t)N * 8));
        da.dump_um = st->dump_um.as<uint64_t>();
        ST_TRY(st->roll0.ensure(s, (size_t)N * 4)); ST_TRY(st->roll1.ensure(s, (size_t)N * 4));
        ST_TRY(st->roll_cnt.ensure(s, (kMaxIter + 3) * sizeof(unsigned long long)));
        ST_TRY(st->anc.ensure(s, (size_t)std::max(n_tax, 1) * 4));
        ST_TRY(hipMemsetAsync(st->roll_cnt.p, 0, (kMaxIter + 3) * sizeof(unsigned long long), s));
        rcnt = st->roll_cnt.as<unsigned long long>();
        da.n_tax = n_tax;
        da.wave_two = 1;
        da.roll_next = st->roll1.as<int32_t>();     // level L appends to roll[(L + 1) & 1]
        da.roll_next_n = rcnt + 1;
        da.fail_ctr = rcnt + kMaxIter + 2;
      }
    }
    if (levels || st->triage) {
      // work queues: [0] the level-0 list, [L] level L's launch
      ST_TRY(st->wq.ensure(s, (kMaxIter + 2) * sizeof(unsigned long long)));
      ST_TRY(hipMemsetAsync(st->wq.p, 0, (kMaxIter + 2) * sizeof(unsigned long long), s));
    }
    if (st->triage) {
      // the triage (wf_triage.hip) decides the contigs explain_one settles from their full
      // clades; the first wave form runs the rest from its list (count on the device)
      ST_TRY(st->tri_list.ensure(s, (size_t)N * 4));
      ST_TRY(st->tri_cnt.ensure(s, 8));
      if (!da.k.hkey) {                                  // no wf_batch.hit_key: packed here
        ST_TRY(st->hkey.ensure(s, (size_t)std::max<int64_t>(NH, 1) * 4));
        ST_TRY(pack_keys(da.k, NH, st->hkey.as<uint32_t>(), st->cus, s));
        da.k.hkey = st->hkey.as<uint32_t>();
        sa.k.hkey = da.k.hkey;                         // (k_att_contig reads it too)
      }
      const int t_tri0 = t_mark(st, s);                 // (the triage span: its launch alone)
      ST_TRY(launch_triage(da, st->cnt.as<int64_t>(), st->cnt_leaves.as<int64_t>(), st->pend.as<int32_t>(), max_hits,
                           st->cus, s));
      const int t_tri = t_mark(st, s);
      t_span(st, WF_PHASE_WAVES, t_waves, t_tri0);
      t_span(st, WF_PHASE_TRIAGE, t_tri0, t_tri);
      t_waves = t_tri;
      using PendItT = hipcub::TransformInputIterator<bool, PendIs, const int32_t*>;
      ST_TRY(select_list(st, s, PendItT(st->pend.as<int32_t>(), PendIs{kPendTriage}), st->tri_list.as<int32_t>(),
                         st->tri_cnt.as<int64_t>(), N));
      SArgs ta = da;                                   // (the list's contigs vary in cost as the roll-up lists')
      ta.wq = st->wq.as<unsigned long long>();
      ST_TRY(launch_fast_list(ta, st->cnt.as<int64_t>(), st->cnt_leaves.as<int64_t>(), st->pend.as<int32_t>(),
                              st->tri_list.as<int32_t>(), st->tri_cnt.as<int64_t>(), max_hits, st->cus, s));
    } else {
      ST_TRY(launch_fast(da, st->cnt.as<int64_t>(), st->cnt_leaves.as<int64_t>(), st->pend.as<int32_t>(), max_hits,
                         st->cus, s));
    }
    if (dump) {
      const int t_h0 = t_mark(st, s);
      t_span(st, WF_PHASE_WAVES, t_waves, t_h0);
      const int grid = st->cus * sparse_waves(st);
      ST_TRY(st->sp_ws.ensure(s, (size_t)grid * kSpSlot));
      da.sp_ws = st->sp_ws.as<char>();
      da.seg_cg = da.dump_cg; da.seg_mean = da.dump_mean; da.crank_first = da.dump_first;
      da.seed_pend = st->pend.as<int32_t>();
      if (levels) {
        da.anc = st->anc.as<int32_t>();               // (k_dump_sparse: ancestors of level 1)
        da.dump_ctr_next = da.dump_ctr + 1;
      }
      const int grid2 = st->cus * two_waves(st);
      if (levels)                                       // compact tables (and the level set-up)
        hipLaunchKernelGGL(k_dump_sparse<1>, dim3(grid2), dim3(64), 0, s, da, st->cnt.as<int64_t>(),
                           st->cnt_leaves.as<int64_t>(), 0);
      hipLaunchKernelGGL(k_dump_sparse<0>, dim3(grid), dim3(64), 0, s, da, st->cnt.as<int64_t>(),
                         st->cnt_leaves.as<int64_t>(), 0);
      ST_TRY(hipGetLastError());
      const int t_h1 = t_mark(st, s);
      t_span(st, WF_PHASE_HANDOVER, t_h0, t_h1);
      t_waves = t_h1;                                  // the waves span resumes here
      if (levels) {
        // levels 1, 2, ...: enqueued kLevelChunk at a time (a level with an empty list costs two
        // near-empty launches), then the next level's count is read back
        constexpr int kLevelChunk = 5;
        unsigned long long* dctr = st->dump_ctr.as<unsigned long long>();
        int32_t* roll[2] = {st->roll0.as<int32_t>(), st->roll1.as<int32_t>()};
        int L = 1;
        unsigned long long* hcnt = st->host_counters;
        for (;;) {
          const int L_end = std::min(L + kLevelChunk - 1, kMaxIter);
          for (; L <= L_end; ++L) {
            SArgs la = da;
            la.dump_ctr = dctr + (L & 1);
            la.dump_ctr_next = dctr + ((L + 1) & 1);
            la.roll_next = roll[(L + 1) & 1];
            la.roll_next_n = rcnt + L + 1;
            la.wq = st->wq.as<unsigned long long>() + L;
            ST_TRY(launch_level(la, st->cnt.as<int64_t>(), st->cnt_leaves.as<int64_t>(), st->pend.as<int32_t>(),
                                roll[L & 1], reinterpret_cast<const int64_t*>(rcnt + L), L, max_hits, st->cus, s));
            la.wq = nullptr;                             // (a queue for sp_two: r5t, 0.35 ms slower)
            hipLaunchKernelGGL(k_dump_sparse<1>, dim3(grid2), dim3(64), 0, s, la, st->cnt.as<int64_t>(),
                               st->cnt_leaves.as<int64_t>(), L);
            hipLaunchKernelGGL(k_dump_sparse<0>, dim3(grid), dim3(64), 0, s, la, st->cnt.as<int64_t>(),
                               st->cnt_leaves.as<int64_t>(), L);
            ST_TRY(hipGetLastError());
          }
          if (st->mbox) {
            ST_TRY(publish_sync(st, s, rcnt + L, 1, rcnt + kMaxIter + 2, 1, hcnt));
          } else {
            ST_TRY(hipMemcpyAsync(hcnt, rcnt + L, 8, hipMemcpyDeviceToHost, s));
            ST_TRY(hipMemcpyAsync(hcnt + 1, rcnt + kMaxIter + 2, 8, hipMemcpyDeviceToHost, s));
            ST_TRY(spin_sync(s, st->lvl_ev[0]));
          }
          if (hcnt[0] == 0 || L > kMaxIter) break;
        }
        const int t_r1 = t_mark(st, s);
        t_span(st, WF_PHASE_ROLLUP, t_h1, t_r1);
        t_waves = t_r1;
        if (hcnt[1] == 0) return 0;                    // every contig finished in the wave forms
      }
    }
    // the other contigs it handed over (pend 1) through the second wave form, its list and
    // count built on the device
    // (only those whose attachments fit the second form's slice: the others would load every
    // hit only to be handed on again)
    using FitIt = hipcub::TransformInputIterator<bool, PendFits, hipcub::CountingInputIterator<int>>;
    ST_TRY(select_list(st, s, FitIt(hipcub::CountingInputIterator<int>(0),
                                    PendFits{st->pend.as<int32_t>(), st->cnt.as<int64_t>(), max_hits <= 256 ? 256 : 512}),
                       st->act0.as<int32_t>(), st->red.as<int64_t>() + 3, N));
    ST_TRY(launch_full(sa, st->cnt.as<int64_t>(), st->cnt_leaves.as<int64_t>(), st->pend.as<int32_t>(),
                       st->act0.as<int32_t>(), st->red.as<int64_t>() + 3, max_hits, st->cus, st->rollup, s));
  } else {
    hipLaunchKernelGGL((k_att_contig<0, kAttNT>), dim3(agrid), dim3(kAttNT), 0, s, sa, st->cnt.as<int64_t>(),
                       st->cnt_leaves.as<int64_t>(),
                       reinterpret_cast<unsigned long long*>(st->red.as<int64_t>() + 1), nullptr, N);
  }
  ST_TRY(hipGetLastError());
  t_span(st, WF_PHASE_WAVES, t_waves, t_mark(st, s));
  const int t_attach = t_mark(st, s);
  {
    size_t t1 = 0, t2 = 0;
    ST_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, t1, st->cnt.as<int64_t>(),
                                            st->att_off.as<int64_t>(), (int)(N + 1), s));
    ST_TRY(hipcub::DeviceReduce::Sum(nullptr, t2, st->cnt_leaves.as<int64_t>(),
                                     st->red.as<int64_t>(), (int)(N + 1), s));
    size_t t3 = 0, t4 = 0;
    ST_TRY(hipcub::DeviceReduce::Max(nullptr, t3, st->cnt.as<int64_t>(), st->red.as<int64_t>() + 1,
                                     (int)(N + 1), s));
    if (level0)
      ST_TRY(hipcub::DeviceSelect::Flagged(nullptr, t4, hipcub::CountingInputIterator<int32_t>(0),
                                           st->pend.as<int32_t>(), st->act0.as<int32_t>(),
                                           st->red.as<int64_t>() + 2, N, s));
    ST_TRY(st->tmp.ensure(s, std::max(std::max(t1, t4), std::max(t2, t3))));
    size_t tb = st->tmp.n;
    ST_TRY(hipcub::DeviceScan::ExclusiveSum(st->tmp.p, tb, st->cnt.as<int64_t>(),
                                            st->att_off.as<int64_t>(), (int)(N + 1), s));
    tb = st->tmp.n;
    ST_TRY(hipcub::DeviceReduce::Sum(st->tmp.p, tb, st->cnt_leaves.as<int64_t>(),
                                     st->red.as<int64_t>(), (int)(N + 1), s));
    // largest contig (a reduction, not one global atomic per contig: those serialise)
    tb = st->tmp.n;
    ST_TRY(hipcub::DeviceReduce::Max(st->tmp.p, tb, st->cnt.as<int64_t>(), st->red.as<int64_t>() + 1,
                                     (int)(N + 1), s));
    if (level0) {                     // the contigs k_fast handed over, in contig order
      tb = st->tmp.n;
      ST_TRY(hipcub::DeviceSelect::Flagged(st->tmp.p, tb, hipcub::CountingInputIterator<int32_t>(0),
                                           st->pend.as<int32_t>(), st->act0.as<int32_t>(),
                                           st->red.as<int64_t>() + 2, N, s));
    }
  }
  if (level0) {
    // staged level 0 list (pend 1) and level 1 seeds (pend 2), each with compact key bases
    ST_TRY(st->act_l0.ensure(s, (size_t)N * 4)); ST_TRY(st->act1.ensure(s, (size_t)N * 4));
    ST_TRY(st->base0.ensure(s, (size_t)(N + 1) * 8)); ST_TRY(st->base1.ensure(s, (size_t)(N + 1) * 8));
    int64_t* red = st->red.as<int64_t>();
    using PendIt = hipcub::TransformInputIterator<bool, PendIs, const int32_t*>;
    const int32_t* pend = st->pend.as<int32_t>();
    ST_TRY(select_list(st, s, PendIt(pend, PendIs{1}), st->act_l0.as<int32_t>(), red + 4, N));
    ST_TRY(select_list(st, s, PendIt(pend, PendIs{2}), st->act1.as<int32_t>(), red + 5, N));
    using AttIt = hipcub::TransformInputIterator<int64_t, ListAtt, hipcub::CountingInputIterator<int>>;
    const int64_t* cnt = st->cnt.as<int64_t>();
    ST_TRY(scan_list(st, s, AttIt(hipcub::CountingInputIterator<int>(0), ListAtt{st->act_l0.as<int32_t>(), cnt, red + 4}),
                     st->base0.as<int64_t>(), N + 1));
    ST_TRY(scan_list(st, s, AttIt(hipcub::CountingInputIterator<int>(0), ListAtt{st->act1.as<int32_t>(), cnt, red + 5}),
                     st->base1.as<int64_t>(), N + 1));
    hipLaunchKernelGGL(k_seed_info, dim3(1), dim3(64), 0, s, red, st->base0.as<int64_t>(), st->base1.as<int64_t>(), N);
    ST_TRY(hipGetLastError());
  }
  const bool mailbox = st->mbox != nullptr;
  if (mailbox) {
    ST_TRY(publish_sync(st, s, st->att_off.as<int64_t>() + N, 1, st->red.p, 8,
                        reinterpret_cast<unsigned long long*>(&hc[2])));
  } else {
    ST_TRY(hipMemcpyAsync(&hc[2], st->att_off.as<int64_t>() + N, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    ST_TRY(hipMemcpyAsync(&hc[3], st->red.p, 8 * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    ST_TRY(spin_sync(s, st->lvl_ev[0]));
  }
  const int64_t A = hc[2], TLB = hc[3], max_att = hc[4];
  const int n_first = level0 ? (int)hc[5] : N;     // contigs handed over (their attachments)
  if (n_first == 0) return 0;                       // the wave kernels finished every contig
  const int n_l0 = level0 ? (int)hc[7] : N, n_seed = level0 ? (int)hc[8] : 0;
  const int64_t keys_l0 = level0 ? hc[9] : hc[2], keys_seed = level0 ? hc[10] : 0;
  // per-contig LDS sort when every contig's attachments fit one workgroup's LDS (else a
  // device radix sort of the whole level)
  sa.sort_cap = 0;
  if (max_att <= kSortMax && sa.key_tb + sa.key_lb + kSortIdxBits <= 64) {
    sa.sort_cap = 2;
    while (sa.sort_cap < max_att) sa.sort_cap <<= 1;
  } else if (max_att <= kRadixMax && sa.key_tb + sa.key_lb <= 32) {
    sa.sort_cap = (int)((max_att + 511) & ~int64_t(511));   // the LDS radix sort (k_sort_radix)
  }
  if (A >= st->att_limit || TLB >= (int64_t(1) << 31) - 1) {
    *err = "too many hit-locus attachments for one batch (split it)";
    return WF_E_TOOBIG;
  }
  const size_t A1 = (size_t)std::max<int64_t>(A, 1), T1 = (size_t)std::max<int64_t>(TLB, 1);
  ST_TRY(st->att_lo.ensure(s, A1 * 4)); ST_TRY(st->att_hi.ensure(s, A1 * 4));
  ST_TRY(st->att_loc.ensure(s, A1 * 4)); ST_TRY(st->att_clade.ensure(s, A1 * 4));
  ST_TRY(st->att_hit.ensure(s, A1 * 4)); ST_TRY(st->att_sc.ensure(s, A1 * 8));
  ST_TRY(st->keys0.ensure(s, A1 * 8)); ST_TRY(st->keys1.ensure(s, A1 * 8));
  ST_TRY(st->vals0.ensure(s, A1 * 4)); ST_TRY(st->vals1.ensure(s, A1 * 4));
  ST_TRY(st->flags.ensure(s, A1 * 4)); ST_TRY(st->seg_id.ensure(s, A1 * 4));
  ST_TRY(st->seg_start.ensure(s, (A1 + 1) * 4)); ST_TRY(st->seg_crank.ensure(s, A1 * 4));
  ST_TRY(st->seg_mean.ensure(s, A1 * 8));
  ST_TRY(st->seg_nleaf.ensure(s, (A1 + 1) * 4)); ST_TRY(st->leaf_off.ensure(s, (A1 + 1) * 4));
  ST_TRY(st->leaf_seg.ensure(s, T1 * 4)); ST_TRY(st->leaf_val.ensure(s, T1 * 8));
  ST_TRY(st->seg_rec.ensure(s, A1 * 16)); ST_TRY(st->seg_cg.ensure(s, A1 * 8));
  ST_TRY(st->wave_list.ensure(s, A1 * 4));
  ST_TRY(st->crank_first.ensure(s, ((size_t)N + 1) * 4));
  ST_TRY(st->seg_cnt.ensure(s, ((size_t)N + 1) * 4));
  ST_TRY(st->satt_lohi.ensure(s, A1 * 8)); ST_TRY(st->satt_sc.ensure(s, A1 * 8));
  ST_TRY(st->act0.ensure(s, (size_t)N * 4)); ST_TRY(st->act1.ensure(s, (size_t)N * 4));
  ST_TRY(st->base0.ensure(s, (size_t)(N + 1) * 8)); ST_TRY(st->base1.ensure(s, (size_t)(N + 1) * 8));
  ST_TRY(st->big_list.ensure(s, (size_t)N * 8));
  ST_TRY(st->big2_list.ensure(s, (size_t)N * 8));
  ST_TRY(st->two_list.ensure(s, (size_t)N * 8));
  ST_TRY(st->one_list.ensure(s, (size_t)N * 8));
  const int64_t n_annot = NL * k.n_sys;
  if (n_annot > 0) ST_TRY(st->annot_best.ensure(s, (size_t)n_annot * 8));
  {
    // temp storage for every primitive of this call, sized once (no reallocation between
    // enqueued kernels)
    size_t t1 = 0, t2 = 0, t3 = 0;
    hipcub::DoubleBuffer<uint64_t> kb0(st->keys0.as<uint64_t>(), st->keys1.as<uint64_t>());
    hipcub::DoubleBuffer<int32_t> vb0(st->vals0.as<int32_t>(), st->vals1.as<int32_t>());
    ST_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, t1, kb0, vb0, (int)A1, 0, 64, s));
    ST_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, t2, st->flags.as<int32_t>(),
                                            st->seg_id.as<int32_t>(), (int)A1, s));
    ST_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, t3, st->seg_nleaf.as<int32_t>(),
                                            st->leaf_off.as<int32_t>(), (int)A1 + 1, s));
    size_t t4 = 0;
    ST_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, t4, st->seg_cnt.as<int32_t>(),
                                            st->crank_first.as<int32_t>(), N + 1, s));
    ST_TRY(st->tmp.ensure(s, std::max(std::max(t1, t4), std::max(t2, t3))));
  }
  sa.att_lo = st->att_lo.as<int32_t>(); sa.att_hi = st->att_hi.as<int32_t>();
  sa.att_loc = st->att_loc.as<int32_t>(); sa.att_clade = st->att_clade.as<int32_t>();
  sa.att_hit = st->att_hit.as<int32_t>(); sa.att_sc = st->att_sc.as<double>();
  sa.flags = st->flags.as<int32_t>(); sa.seg_id = st->seg_id.as<int32_t>();
  sa.seg_start = st->seg_start.as<int32_t>(); sa.seg_crank = st->seg_crank.as<int32_t>();
  sa.seg_mean = st->seg_mean.as<double>();
  sa.seg_nleaf = st->seg_nleaf.as<int32_t>(); sa.leaf_off = st->leaf_off.as<int32_t>();
  sa.leaf_seg = st->leaf_seg.as<int32_t>(); sa.leaf_val = st->leaf_val.as<double>();
  sa.seg_rec = st->seg_rec.as<int4>();
  sa.seg_cg = st->seg_cg.as<int2>();
  sa.crank_first = st->crank_first.as<int32_t>();
  sa.seg_cnt = st->seg_cnt.as<int32_t>();
  ST_TRY(st->seg_len.ensure(s, A1 * 4));
  sa.seg_len = sa.sort_cap > 0 ? st->seg_len.as<int32_t>() : nullptr;   // set by k_seg_build
  sa.satt_lohi = st->satt_lohi.as<int2>(); sa.satt_sc = st->satt_sc.as<double>();
  sa.annot_best = st->annot_best.as<uint64_t>();
  sa.big_list = st->big_list.as<int32_t>();
  sa.big2_list = st->big2_list.as<int32_t>();
  sa.two_list = st->two_list.as<int32_t>();
  sa.wave_list = st->wave_list.as<int32_t>();
  if (n_annot > 0 && (int64_t)max_loci * k.n_sys > kAnnSlots) {   // HBM annotation slots
    ST_TRY(hipMemsetAsync(st->annot_best.p, 0, (size_t)n_annot * 8, s));
    ST_TRY(hipMemsetAsync(k.annot, 0xFF, (size_t)n_annot * 4, s));     // -1: no winner
  }
  if (max_hits >= kAttBigHits)
    hipLaunchKernelGGL((k_att_contig<1, kAttNTBig>), dim3(std::min<unsigned>(agrid, (unsigned)n_first)), dim3(kAttNTBig), 0,
                       s, sa, nullptr, nullptr, nullptr, level0 ? st->act0.as<int32_t>() : nullptr, n_first);
  else
    hipLaunchKernelGGL((k_att_contig<1, kAttNT>), dim3(std::min<unsigned>(agrid, (unsigned)n_first)), dim3(kAttNT), 0, s,
                       sa, nullptr, nullptr, nullptr, level0 ? st->act0.as<int32_t>() : nullptr, n_first);
  ST_TRY(hipGetLastError());
  t_span(st, WF_PHASE_ATTACH, t_attach, t_mark(st, s));

  // explain_one by one wave per contig (k_one); the dense workgroup (k_decide<3>) gets the
  // contigs it hands over and the ones it leaves open (explain_two)
  sa.one_list = st->one_list.as<int32_t>();
  // roll-up levels
  Buf* act[2] = {&st->act0, &st->act1};
  Buf* base[2] = {&st->base0, &st->base1};
  const unsigned leaf_grid = (unsigned)st->cus * 8u;   // k_leaf: persistent, 8 blocks per CU
  // Level counters: level L counts into block L of lvl_ctr; the host reads them after each
  // level through the mailbox
  const int n_lv = kMaxIter + 2;
  ST_TRY(st->lvl_ctr.ensure(s, (size_t)n_lv * 8 * sizeof(unsigned long long)));
  ST_TRY(hipMemsetAsync(st->lvl_ctr.p, 0, (size_t)n_lv * 8 * sizeof(unsigned long long), s));
  unsigned long long* lvl_ctr = st->lvl_ctr.as<unsigned long long>();
  sa.in_counts = nullptr;
  int n_act = n_l0;
  int64_t n_keys = keys_l0;
  int start = 0;
  if (n_seed > 0) {                     // level 1 begins with the seeds (level 0 appends)
    hipLaunchKernelGGL(k_set_word, dim3(1), dim3(64), 0, s, lvl_ctr,
                       ((unsigned long long)n_seed << 40) | (unsigned long long)keys_seed);
    hipLaunchKernelGGL(k_rekey_seeds, dim3(std::min(n_seed, st->cus * 8)), dim3(256), 0, s, st->act1.as<int32_t>(),
                       n_seed, sa.catt_off, sa.att_clade, k.parent);
    ST_TRY(hipGetLastError());
    if (n_l0 == 0) {
      start = 1;
      n_act = n_seed;
      n_keys = keys_seed;
    }
  }
  if (det) {
    det->levels.clear();
    ST_TRY(st->span_cnt.ensure(s, A1 * 4));
    ST_TRY(st->spans.ensure(s, A1 * 8));
  }
  if (st->dec_lds > 64 * 1024) {
    // per process, thread-safe initialisation (C++11 statics); every device is a gfx950
    static const hipError_t attr3 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_decide<3>),
                                                        hipFuncAttributeMaxDynamicSharedMemorySize,
                                                        160 * 1024 - 1024);
    ST_TRY(attr3);
  }
  for (int level = start; n_act > 0 && level <= kMaxIter; ++level) {
    sa.counters = lvl_ctr + 8 * level;
    const int cur = level & 1;
    sa.act = level == 0 ? (level0 ? st->act_l0.as<int32_t>() : nullptr) : act[cur]->as<int32_t>();
    sa.act_base = level == 0 && !level0 ? nullptr : base[cur]->as<int64_t>();
    sa.act_next = act[cur ^ 1]->as<int32_t>();
    sa.act_base_next = base[cur ^ 1]->as<int64_t>();
    const int cb = bits_for(n_act);
    const int end_bit = cb + sa.key_tb + sa.key_lb;
    if (end_bit > 64) { *err = "sort key wider than 64 bits"; return -1; }
    hipcub::DoubleBuffer<uint64_t> kbuf(st->keys0.as<uint64_t>(), st->keys1.as<uint64_t>());
    hipcub::DoubleBuffer<int32_t> vbuf(st->vals0.as<int32_t>(), st->vals1.as<int32_t>());
    sa.keys = nullptr;
    sa.vals = nullptr;
    const int t_seg = t_mark(st, s);
    if (n_keys > 0 && sa.sort_cap > kSortMax && !det) {
      // the stress contigs' whole front end in one launch (k_front_radix), then the rare
      // wave / leaf segments it listed
      static const hipError_t fattr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_front_radix<false>),
                                                          hipFuncAttributeMaxDynamicSharedMemorySize,
                                                          (int)radix_lds(kRadixMax));
      static const hipError_t pattr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_front_radix<true>),
                                                          hipFuncAttributeMaxDynamicSharedMemorySize,
                                                          (int)radix_lds(kRadixMax, true));
      ST_TRY(fattr);
      ST_TRY(pattr);
      const bool packed = sa.key_lb <= 6 && n_tax <= kPackTaxMax;
      const size_t fr_bytes = ((size_t)n_act + 4) * sizeof(unsigned long long);
      ST_TRY(st->front.ensure(s, fr_bytes));
      ST_TRY(hipMemsetAsync(st->front.p, 0, fr_bytes, s));
      unsigned long long* fr = st->front.as<unsigned long long>();
      const size_t lds = radix_lds(sa.sort_cap, packed);
      const int per_cu = std::max(1, (int)((160 * 1024) / (lds + 1024)));   // (+ its static LDS)
      if (packed)
        hipLaunchKernelGGL(k_front_radix<true>, dim3(std::min(n_act, st->cus * per_cu)), dim3(kRadixNT), lds, s, sa,
                           n_act, n_keys, n_tax, fr);
      else
        hipLaunchKernelGGL(k_front_radix<false>, dim3(std::min(n_act, st->cus * per_cu)), dim3(kRadixNT), lds, s, sa,
                           n_act, n_keys, n_tax, fr);
      hipLaunchKernelGGL(k_front_fin, dim3(1), dim3(64), 0, s, sa, n_act, fr);
      hipLaunchKernelGGL(k_seg_wave, dim3(st->cus * 32), dim3(64), 0, s, sa);
      hipLaunchKernelGGL(k_leaf, dim3(leaf_grid), dim3(256), 0, s, sa, n_keys);
      hipLaunchKernelGGL(k_seg_combine, dim3(st->cus * 4), dim3(256), 0, s, sa, n_keys);
      ST_TRY(hipGetLastError());
      sa.keys = kbuf.Current();
      sa.vals = vbuf.Current();
    } else if (n_keys > 0) {
      size_t need = st->tmp.n;
      if (sa.sort_cap > kSortMax) {
        static const hipError_t rattr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sort_radix),
                                                            hipFuncAttributeMaxDynamicSharedMemorySize,
                                                            (int)radix_lds(kRadixMax));
        ST_TRY(rattr);
        const size_t lds = radix_lds(sa.sort_cap);
        const int per_cu = std::max(1, (int)((160 * 1024) / lds));
        hipLaunchKernelGGL(k_sort_radix, dim3(std::min(n_act, st->cus * per_cu)), dim3(kRadixNT), lds, s, sa, n_act,
                           level, kbuf.Current(), vbuf.Current());
      } else if (sa.sort_cap > 0) {
        const size_t lds = (size_t)sa.sort_cap * 8;
        const int per_cu = std::min(32, std::max(1, (int)((160 * 1024) / lds)));
        // level 0: one wave per contig (10^4+ contigs fill the chip); later levels have
        // few contigs, so four waves shorten each contig's sort
        if (level == 0)
          hipLaunchKernelGGL(k_sort_contig<64>, dim3(std::min(n_act, st->cus * per_cu)), dim3(64), lds, s,
                             sa, n_act, level, kbuf.Current(), vbuf.Current());
        else
          hipLaunchKernelGGL(k_sort_contig<256>, dim3(std::min(n_act, st->cus * per_cu)), dim3(256), lds,
                             s, sa, n_act, level, kbuf.Current(), vbuf.Current());
      } else {
        hipLaunchKernelGGL(k_keys_active, dim3(std::min(n_act, st->cus * 8)), dim3(256), 0, s, sa,
                           n_act, kbuf.Current(), vbuf.Current());
        ST_TRY(hipGetLastError());
        ST_TRY(hipcub::DeviceRadixSort::SortPairs(st->tmp.p, need, kbuf, vbuf, (int)n_keys, 0, end_bit, s));
      }
      ST_TRY(hipGetLastError());
      sa.keys = kbuf.Current();
      sa.vals = vbuf.Current();
      if (sa.sort_cap > 0) {
        need = st->tmp.n;
        if (n_act < 32 * kScanNT)        // <= 32 items a thread: one workgroup
          hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(kScanNT), 0, s, sa.seg_cnt, sa.crank_first, n_act + 1);
        else
          ST_TRY(hipcub::DeviceScan::ExclusiveSum(st->tmp.p, need, sa.seg_cnt, sa.crank_first, n_act + 1, s));
        if (sa.sort_cap > kSortMax)                   // (the radix-sorted stress contigs)
          hipLaunchKernelGGL(k_seg_build_wide, dim3(std::min(n_act, st->cus * 4)), dim3(kRadixNT), 0, s, sa, n_act,
                             level, n_keys);
        else
          hipLaunchKernelGGL(k_seg_build, dim3(std::min(n_act, st->cus * 32)), dim3(64), 0, s, sa, n_act,
                             level, n_keys);
      } else {
        hipLaunchKernelGGL(k_seg_flags, dim3(grid_for(n_keys)), dim3(256), 0, s, sa, n_keys);
        need = st->tmp.n;
        ST_TRY(hipcub::DeviceScan::InclusiveSum(st->tmp.p, need, sa.flags, sa.seg_id, (int)n_keys, s));
        hipLaunchKernelGGL(k_segs, dim3(grid_for(n_keys)), dim3(256), 0, s, sa, n_keys);
        hipLaunchKernelGGL(k_gather, dim3(grid_for(n_keys)), dim3(256), 0, s, sa, n_keys);
        hipLaunchKernelGGL(k_crank_first, dim3(grid_for(n_keys + 1)), dim3(256), 0, s, sa, n_keys, n_act);
      }
      if (det)
        hipLaunchKernelGGL(k_seg_spans, dim3(grid_for(n_keys)), dim3(256), 0, s, sa, n_keys,
                           st->span_cnt.as<int32_t>(), st->spans.as<int32_t>());
      // short segments' means by one thread each; one wave per multi-attachment segment, a
      // serial envelope sweep (62 VGPRs, 2.8 KB LDS -> 32 waves per CU; roll-up levels have
      // ~10^5 such segments); the rest through the leaf kernels
      hipLaunchKernelGGL(k_seg_rec, dim3(grid_for(n_keys + 1)), dim3(256), 0, s, sa, n_keys);
      hipLaunchKernelGGL(k_seg_wave, dim3(st->cus * 32), dim3(64), 0, s, sa);
      need = st->tmp.n;
      ST_TRY(hipcub::DeviceScan::ExclusiveSum(st->tmp.p, need, sa.seg_nleaf, sa.leaf_off,
                                              (int)n_keys + 1, s));
      hipLaunchKernelGGL(k_leaf_expand, dim3(grid_for(n_keys)), dim3(256), 0, s, sa, n_keys);
      hipLaunchKernelGGL(k_leaf, dim3(leaf_grid), dim3(256), 0, s, sa, n_keys);
      hipLaunchKernelGGL(k_seg_combine, dim3(st->cus * 4), dim3(256), 0, s, sa, n_keys);
      ST_TRY(hipGetLastError());
    } else {
      sa.keys = kbuf.Current();
      sa.vals = vbuf.Current();
    }
    t_span(st, WF_PHASE_SEGMENTS, t_seg, t_mark(st, s));
    if (det) ST_TRY(details_level(st, sa, level, n_act, n_keys, s, det));
    const int t_dec = t_mark(st, s);
    const unsigned dgrid = (unsigned)std::min<int64_t>(n_act, (int64_t)st->cus * 16);
    hipLaunchKernelGGL(k_one, dim3(std::min<int64_t>(n_act, (int64_t)st->cus * 32)), dim3(64), 0, s, sa,
                       n_act, level, n_keys);
    // the dense decision for what k_one handed over whole (> 63 loci, more segments than it
    // holds, --weak-loci assign-unknown) and the > 63-loci contigs it left open (counts on
    // the device: a grid of rank-independent size, idle blocks exit at once): as many
    // one-wave workgroups as the arena and 3 waves/SIMD (VGPRs) allow
    const unsigned dec_per_cu =
        (unsigned)std::max<int64_t>(1, std::min<int64_t>(12, (160 * 1024) / std::max<int64_t>(st->dec_lds, 1)));
    hipLaunchKernelGGL(k_decide<3>, dim3(std::min<unsigned>(dgrid, (unsigned)st->cus * dec_per_cu)),
                       dim3(kDecNT), (size_t)st->dec_lds, s, sa, n_act, level, n_keys);
    ST_TRY(hipGetLastError());
    t_span(st, WF_PHASE_DECIDE, t_dec, t_mark(st, s));
    if (mailbox) {
      ST_TRY(publish_sync(st, s, sa.counters, 5, nullptr, 0, st->host_counters));
    } else {
      ST_TRY(hipMemcpyAsync(st->host_counters, sa.counters, 5 * sizeof(unsigned long long),
                            hipMemcpyDeviceToHost, s));
      ST_TRY(spin_sync(s, st->lvl_ev[0]));
    }
    if (st->host_counters[4]) {                      // (k_front_radix's look-back never completed)
      *err = "segment look-back timed out";
      return -2;
    }
    const int n_big = (int)st->host_counters[2];
    int n_dense = 0;                    // contigs that need the dense decision in an HBM slot
    const int t_big = n_big > 0 ? t_mark(st, s) : -1;
    if (n_big > 0 && st->sparse_big) {
      // the decision from the segment table, one wave per contig (wf_sparse.h): as many
      // waves as are resident at once (LDS-bound)
      const int grid = std::min(n_big, st->cus * sparse_waves(st));
      ST_TRY(st->sp_ws.ensure(s, (size_t)grid * kSpSlot));
      sa.sp_ws = st->sp_ws.as<char>();
      hipLaunchKernelGGL(k_big_sparse, dim3(grid), dim3(64), 0, s, sa, level, n_keys);
      ST_TRY(hipGetLastError());
      if (mailbox) {
        ST_TRY(publish_sync(st, s, sa.counters, 4, nullptr, 0, st->host_counters));
      } else {
        ST_TRY(hipMemcpyAsync(st->host_counters, sa.counters, 4 * sizeof(unsigned long long),
                              hipMemcpyDeviceToHost, s));
        ST_TRY(spin_sync(s, st->lvl_ev[0]));
      }
      n_dense = (int)st->host_counters[1];
    } else {
      n_dense = n_big;
    }
    if (n_dense > 0) {
      const int64_t slot = ((int64_t)st->host_counters[3] + 255) & ~int64_t(255);
      // HBM-slot workgroups: as many as are resident at once (135 VGPRs: 3 four-wave
      // workgroups per CU); cfg5 (30 k stress contigs, round 2) measured 234.7 ms/pass at 2
      // per CU, 222.8 at 3, 264.5 at 4 (a second, partial round), 230.2 at 8
      const int slots = std::min(n_dense, st->cus * 3);
      ST_TRY(st->big_ws.ensure(s, (size_t)slot * slots));
      sa.k.big_ws = st->big_ws.as<char>();
      sa.k.slot_bytes = slot;
      hipLaunchKernelGGL(k_decide_big, dim3(slots), dim3(kBlock), 0, s, sa, level, n_keys,
                         (n_big > 0 && st->sparse_big) ? 1 : 0);
      ST_TRY(hipGetLastError());
      ST_TRY(hipMemcpyAsync(st->host_counters, sa.counters, 4 * sizeof(unsigned long long),
                            hipMemcpyDeviceToHost, s));
      ST_TRY(spin_sync(s, st->lvl_ev[0]));
    }
    if (n_big > 0) t_span(st, WF_PHASE_BIG, t_big, t_mark(st, s));
    if (level == start && !st->dec_lds_fixed && n_dense * 50 > n_act && st->dec_lds < 48 * 1024)
      st->dec_lds += 8 * 1024;   // adaptive arena: grows while > 2% of a first level overflow
    n_act = (int)(st->host_counters[0] >> 40);
    n_keys = (int64_t)(st->host_counters[0] & ((1ull << 40) - 1));
  }
  return 0;
}

__global__ void k_ppot_strip(int64_t* ppot, int n) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n) ppot[c] &= (int64_t(1) << 40) - 1;
}

hipError_t finish_ppot(const KArgs& k, hipStream_t s) {
  if (!k.ppot || k.n_contigs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ppot_strip, dim3((unsigned)((k.n_contigs + 255) / 256)), dim3(256), 0, s, k.ppot, k.n_contigs);
  return hipGetLastError();
}

int staged_score(StagedState* st, const KArgs& k, int n_tax, int max_loci, int max_hits, int64_t NH, int64_t NL,
                 hipStream_t s, std::string* err, DetailsSink* det) {
  st->tspans.clear();
  st->tev_used = 0;
  int rc = staged_run(st, k, n_tax, max_loci, max_hits, NH, NL, s, err, det);
  const hipError_t e = t_collect(st, s);
  if (rc == 0 && e != hipSuccess) {
    *err = std::string("phase timing: ") + hipGetErrorString(e);
    rc = -2;
  }
  return rc;
}

WF_STAMP_READER(staged, g_stamps, 32)
}  // namespace wf
