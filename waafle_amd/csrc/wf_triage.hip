// Level-0 triage of the contig-scoring path (gfx950 / MI355X): the contigs explain_one
// settles from the clades present on every locus, decided without a sort.
//
// One wave64 per contig, alone in its workgroup (no barriers), persistent over the batch in
// the XCD-aware order of the wave kernels (wf_fast.hip).  Per contig (orgscorer.py:359-429,
// 447-461, 585-597, 621-631):
//   hits -> attachments     lane per hit, up to 4 batches of 64 held in registers; the loci
//                           (ascending, disjoint) in LDS, each hit's first candidate locus by
//                           binary search (orgscorer.py:359-369, calc_overlap utils.py:487-500)
//   full clades             the clades attached to locus 0 go into a small LDS hash table;
//                           every attachment ORs its locus into its clade's mask there; a clade
//                           whose mask holds every locus is "full".  An explain_one option has
//                           crit >= k1 > 0, so a nonzero gene score on every unmasked locus: with
//                           every locus unmasked, the options are full clades
//   their gene scores       lane per locus: the segment's envelope is one run (one attachment,
//                           or a whole-locus one dominating the rest), whose exact numpy mean has
//                           a closed form (pw_const_sum / pw_run_sum, wf_device.h)
//   weak-locus mask         every locus is unmasked when a full known clade's mean reaches kmin
//                           on it (orgscorer.py:420-427; --weak-loci penalize masks nothing)
//   explain_one + meld_one  crit = min, rank = numpy-order mean; best by (rank, clade) as the
//                           wave kernels; options within --range melded to their LCA
//   annotations             the last hit at the best score per (locus, system), :383-392
// Everything else -- no full clade (explain_two), a locus the full clades leave unsettled, a
// segment of several envelope runs, no option, more than 256 hits or 64 loci, overlapping or
// unordered loci, --min-overlap 0, --weak-loci assign-unknown -- is handed on untouched
// (pend = kPendTriage): the first wave form (k_wave<CAP, false>) runs exactly those contigs,
// from their hits, as it runs every contig without the triage.  Same arithmetic, so the same
// bits: the triage only skips the sort, the segment table and the pruning passes the wave
// form spends on the contigs explain_one settles at level 0 (~90% at cfg4).
#include "wf_device.h"
#include "wf_lanes.h"


namespace wf {

namespace {


constexpr int kTrHB = 4;               // hit batches of 64: contigs of up to 256 hits
constexpr int kTrLoc = 64;             // loci (64-bit locus masks)
constexpr int kTrTab = 128;            // candidate table: clades attached to locus 0
constexpr int kTrSeg = 64;             // full clades x loci evaluated (one lane each)
constexpr int kTrSpan = 26;            // loci one hit may attach to, from its first candidate
constexpr uint32_t kTrEmpty = 0xFFFFFFFFu;
constexpr int kTrXcds = 8;             // MI355X: 8 XCDs of 32 CUs, each with its own L2
constexpr int kTrWaves = 8;            // resident waves per SIMD (64 VGPRs, ~12 spilled; a 4.8 KB slice).
                                       // Same box (r5c): 3.66 ms per cfg4 pass against 3.85 at 6
                                       // waves per SIMD (75 VGPRs, none spilled)
constexpr int kTrBig = 512;            // more hits than any wave slice: k_count
constexpr int kCntR = 4;               // k_count: hit batches per round of loads

struct TriSmem {
  int lo[kTrLoc], hi[kTrLoc];          // locus site ranges (min, max of start/end)
  uint32_t tkey[kTrTab];               // candidate clade (kTrEmpty: free slot)
  uint64_t tmask[kTrTab];              // loci it is attached to
  uint64_t abest[kTrLoc];              // (locus, system): best annotation score bits
  int ahit[kTrLoc];                    // ... and the last hit at that score
  // the full clades' segments, slot i * G + g (full clade i, locus g): attachments, the last
  // attachment's site range, the best score of its attachments of a non-empty range and of
  // its whole-locus attachments (score bits: scores are >= 0)
  int scnt[kTrSeg];
  uint32_t slohi[kTrSeg];
  uint64_t spart[kTrSeg];
  uint64_t sfw[kTrSeg];
  int fcl[kTrSeg];                     // full clade i: its id
  int8_t tfull[kTrTab];                // table slot -> full clade index (-1: not full)
  int8_t st[kTrLoc];
};
static_assert(sizeof(TriSmem) <= 160 * 1024 / (4 * kTrWaves), "triage slice: kTrWaves per SIMD");

__device__ __forceinline__ uint32_t tr_hash(uint32_t clade) { return (clade * 0x9E3779B1u) >> 25; }   // 7 bits

// Site range [start, stop) of a hit on a locus (orgscorer.py:371-382, python slice rules),
// packed lo | hi << 16 (loci < 8192 sites here).
__device__ __forceinline__ uint32_t tr_lohi(int qlo, int qhi, int llo, int len) {
  const int h1s = max(0, qlo - llo);
  const int h2s = min(len - 1, qhi - llo);
  const int start = min(h1s, len);
  int stop = h2s + 1;
  if (stop < 0) { stop += len; if (stop < 0) stop = 0; }
  return (uint32_t)start | ((uint32_t)stop << 16);
}

// The packed hit word (wf_batch.hit_key, kKey* in wf_internal.h).  After the table pass the
// low 24 bits hold the clade's table slot + 1.

// wf_batch.hit_key when the caller passes none (include/waafle_hip.h)
__global__ void k_pack_keys(const KArgs K, int64_t n_hits, uint32_t* key) {
  for (int64_t h = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; h < n_hits; h += (int64_t)gridDim.x * blockDim.x)
    key[h] = (uint32_t)K.taxon[h] | (K.scov[h] >= K.p.min_scov ? kKeyScov : 0u) | (K.hstrand[h] == 1 ? kKeyMinus : 0u) |
             (K.n_sys > 0 ? (K.sysmask[h] & 63u) << kKeySys : 0u);
}

// SYSKEY: the annotation systems come from the key (n_systems <= 6); else from hit_sysmask.
template <bool SYSKEY>
__global__ __launch_bounds__(64, kTrWaves) void k_triage(const SArgs S_arg, int64_t* ccnt, int64_t* cleaves,
                                                         int32_t* pend) {
  __shared__ TriSmem F;
  const int lane = threadIdx.x;
  const int N = S_arg.k.n_contigs;
  // XCD-aware order (k_wave): XCD x's j-th workgroup takes contig (8 k + x) * B + j at step k
  const bool xmap = gridDim.x % kTrXcds == 0;
  const int xb = (int)gridDim.x / kTrXcds, xj = (int)blockIdx.x / kTrXcds, xx = (int)blockIdx.x % kTrXcds;
  for (int it = 0;; ++it) {
    const int c = xmap ? (it * kTrXcds + xx) * xb + xj : (int)blockIdx.x + it * (int)gridDim.x;
    if (c >= N) break;
    TLAP_MARK();
    const SArgs& S = kernarg_fresh<SArgs>(S_arg);
    const KArgs& K = S.k;
    const DevParams& P = K.p;
    const int nsys = K.n_sys;
    // a contig the triage does not decide goes on to the wave form
    auto hand_on = [&]() {
      if (lane == 0) pend[c] = kPendTriage;
    };
    const int64_t h0 = K.hit_off[c], h1 = K.hit_off[c + 1];
    const int64_t nh = h1 - h0;
    const int64_t hend = min(h1, h0 + 64 * kTrHB);
    // every field of the contig's hits, issued before the loci: 20 bytes a hit (range, the
    // packed key, score)
    int r_qlo[kTrHB], r_qhi[kTrHB];
    uint32_t r_k[kTrHB];
    double r_sc[kTrHB];
    uint32_t r_m[SYSKEY ? 1 : kTrHB];
#pragma unroll
    for (int b = 0; b < kTrHB; ++b) {
      const int64_t h = h0 + 64 * b + lane;
      r_qlo[b] = 0; r_qhi[b] = 0; r_k[b] = 0u; r_sc[b] = 0.0;
      if (!SYSKEY) r_m[b] = 0u;
      if (h < hend) {
        r_qlo[b] = K.qlo[h];
        r_qhi[b] = K.qhi[h];
        r_k[b] = K.hkey[h];
        r_sc[b] = K.score[h];
        if (!SYSKEY && nsys > 0) r_m[b] = K.sysmask[h];
      }
    }
    auto sysm = [&](int b) -> uint32_t { return SYSKEY ? r_k[b] >> kKeySys : r_m[b]; };
    const int64_t l0 = K.loc_off[c];
    const int G = (int)(K.loc_off[c + 1] - l0);
    int my_lo = 0, my_hi = -1, my_st = 0;
    if (lane < G && G <= kTrLoc) {
      const int a = K.lstart[l0 + lane], e = K.lend[l0 + lane];
      my_lo = min(a, e);
      my_hi = max(a, e);
      my_st = K.lstrand[l0 + lane];
    }
    const int prev_hi = __shfl_up(my_hi, 1, 64);
    // what the triage takes (else the wave form): loci ascending and disjoint (each hit's
    // loci found by binary search), every locus one numpy buffer, options only on full
    // clades (k1 > 0), the weak-locus mask from the full clades' means
    const bool take =
        nh > 0 && nh <= 64 * kTrHB && G > 0 && G <= kTrLoc && G * nsys <= kTrLoc && P.min_overlap > 0.0 &&
        P.k1 > 0.0 && P.weak != 2 &&
        __ballot(lane < G && ((lane >= 1 && my_lo <= prev_hi) || my_hi - my_lo + 1 >= kNpyBuf)) == 0ull;
    if (!take) {
      hand_on();
      continue;
    }
    const uint64_t allG = G >= 64 ? ~0ull : ((1ull << G) - 1ull);
    const int nann = G * nsys;
    const bool ann_on = nsys > 0;
    if (lane < G) { F.lo[lane] = my_lo; F.hi[lane] = my_hi; F.st[lane] = (int8_t)my_st; }
    F.tkey[lane] = kTrEmpty; F.tkey[lane + 64] = kTrEmpty;
    F.tmask[lane] = 0ull; F.tmask[lane + 64] = 0ull;
    F.abest[lane] = 0ull; F.ahit[lane] = -1;
    F.scnt[lane] = 0; F.sfw[lane] = 0ull; F.spart[lane] = 0ull;
    wave_sync();
    TLAP(0);                                           // (stamps: offsets, hits, loci, slice set-up)
    // ---- hits -> attachments (orgscorer.py:359-369): per batch, the first locus ending at or
    // after qlo, then the loci up to the one starting past qhi; attached loci relative to the
    // first: g0 | mask << 6 (0: none) ----
    uint32_t r_am[kTrHB];
    bool bad = false;
#pragma unroll
    for (int b = 0; b < kTrHB; ++b) {
      uint32_t am = 0u;
      if (h0 + 64 * b + lane < hend && (r_k[b] & kKeyScov)) {
        const int qlo = r_qlo[b], qhi = r_qhi[b];
        int g = 0;
#pragma unroll
        for (int k = 32; k > 0; k >>= 1) {
          const int gk = g + k;                      // (a select, not a branch per step)
          g = (gk <= G && F.hi[min(gk, G) - 1] < qlo) ? gk : g;
        }
        const int g0 = g;
        uint32_t rel = 0u;
        for (; g < G; ++g) {
          const int lo = F.lo[g];
          if (lo > qhi) break;
          if (attaches(P, qlo, qhi, (r_k[b] & kKeyMinus) ? 1 : 0, lo, F.hi[g] - lo + 1, F.st[g])) {
            if (g - g0 < kTrSpan) rel |= 1u << (g - g0);
            else bad = true;
          }
        }
        if (rel) {
          am = (uint32_t)g0 | (rel << 6);
          int cl = (int)(r_k[b] & kKeyTaxon);
          for (int j = 0; j < P.jump; ++j) cl = K.parent[cl];           // orgscorer.py:955-957
          r_k[b] = (r_k[b] & ~kKeyTaxon) | (uint32_t)cl;
        }
      }
      r_am[b] = am;
    }
    TLAP(1);                                           // (stamps: attachments)
    // ---- the candidates: clades attached to locus 0 ----
#pragma unroll
    for (int b = 0; b < kTrHB; ++b) {
      if ((r_am[b] & 0x7Fu) == 0x40u) {               // g0 == 0 and locus 0 attached
        const uint32_t cl = r_k[b] & kKeyTaxon;
        uint32_t slot = tr_hash(cl);
        for (int probes = 0;; ++probes) {
          if (probes == kTrTab) { bad = true; break; }
          const uint32_t old = atomicCAS(&F.tkey[slot], kTrEmpty, cl);
          if (old == kTrEmpty || old == cl) break;
          slot = (slot + 1) & (kTrTab - 1);
        }
      }
    }
    if (__ballot(bad) != 0ull) {
      hand_on();
      wave_sync();
      continue;
    }
    wave_sync();
    TLAP(2);                                           // (stamps: candidate inserts)
    // ---- every attachment ORs its loci into its clade's mask (the key's taxon bits become the
    // clade's table slot + 1, 0 outside the table); annotation pass 1 (:383-392) ----
#pragma unroll
    for (int b = 0; b < kTrHB; ++b) {
      const uint32_t am = r_am[b];
      int found = -1;
      if (am != 0u) {
        const int g0 = (int)(am & 63u);
        const uint64_t lm = (uint64_t)(am >> 6) << g0;
        const uint32_t cl = r_k[b] & kKeyTaxon;
        uint32_t slot = tr_hash(cl);
        for (int probes = 0; probes < kTrTab; ++probes) {
          const uint32_t k = F.tkey[slot];
          if (k == cl) { atomicOr(&F.tmask[slot], lm); found = (int)slot; break; }
          if (k == kTrEmpty) break;
          slot = (slot + 1) & (kTrTab - 1);
        }
        const uint32_t m = sysm(b);
        if (ann_on && m != 0u && r_sc[b] >= P.annot_ref)
          for (uint64_t bits = lm; bits; bits &= bits - 1) {
            const int g = __builtin_ctzll(bits);
            for (int s = 0; s < nsys; ++s)
              if ((m >> s) & 1u) atomicMax(&F.abest[g * nsys + s], dbits(r_sc[b]));
          }
      }
      r_k[b] = (r_k[b] & ~kKeyTaxon) | (uint32_t)(found + 1);
    }
    wave_sync();
    TLAP(3);                                           // (stamps: masks, annotation pass 1)
    // full clades (every locus in the mask), numbered in table order (lane i: slots i, i + 64)
    int nfull = 0;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int e = lane + 64 * half;
      const bool full = F.tkey[e] != kTrEmpty && F.tmask[e] == allG;
      const uint64_t fm = __ballot(full);
      const int fi = nfull + __popcll(fm & ((1ull << lane) - 1ull));
      F.tfull[e] = (int8_t)(full && fi * G < kTrSeg ? fi : -1);
      if (full && fi * G < kTrSeg) F.fcl[fi] = (int)F.tkey[e];
      nfull += __popcll(fm);
    }
    if (nfull == 0 || nfull * G > kTrSeg) {            // explain_two (no full clade), or the wave form
      hand_on();
      wave_sync();
      continue;
    }
    wave_sync();
    TLAP(4);                                           // (stamps: full-clade scan)
    // ---- the full clades' attachments per segment; annotation pass 2: the last hit (largest
    // index) at the best score ----
#pragma unroll
    for (int b = 0; b < kTrHB; ++b) {
      const uint32_t am = r_am[b];
      int fi = -1;
      if (am != 0u) {
        const int g0 = (int)(am & 63u);
        const int slot = (int)(r_k[b] & kKeyTaxon) - 1;
        fi = slot >= 0 ? (int)F.tfull[slot] : -1;
        if (fi >= 0)
          for (uint32_t rel = am >> 6; rel; rel &= rel - 1) {
            const int g = g0 + __builtin_ctz(rel);
            const int q = fi * G + g;
            const int llo = F.lo[g], len = F.hi[g] - llo + 1;
            const uint32_t lh = tr_lohi(r_qlo[b], r_qhi[b], llo, len);
            atomicAdd(&F.scnt[q], 1);
            F.slohi[q] = lh;
            // (k_wave's Fw: the best whole-locus score above 0.0; an attachment k_wave keeps
            // has a non-empty range and a score above it, so one exists iff spart > Fw)
            const int lo = (int)(lh & 0xFFFFu), hi = (int)(lh >> 16);
            if (lo < hi) atomicMax(&F.spart[q], dbits(r_sc[b]));
            if (lo <= 0 && hi >= len && r_sc[b] > 0.0) atomicMax(&F.sfw[q], dbits(r_sc[b]));
          }
        const uint32_t m = sysm(b);
        if (ann_on && m != 0u && r_sc[b] >= P.annot_ref) {
          const int h = (int)(h0 + 64 * b + lane);
          for (uint64_t bits = (uint64_t)(am >> 6) << g0; bits; bits &= bits - 1) {
            const int g = __builtin_ctzll(bits);
            for (int s = 0; s < nsys; ++s)
              if (((m >> s) & 1u) && F.abest[g * nsys + s] == dbits(r_sc[b])) atomicMax(&F.ahit[g * nsys + s], h);
          }
        }
      }
    }
    wave_sync();
    TLAP(5);                                           // (stamps: segments, annotation pass 2)
    // ---- gene scores (:399-406), lane per segment: one envelope run, exact numpy mean ----
    const int nseg = nfull * G;
    const int my_g = lane % G, my_f = lane / G;
    double mean = 0.0;
    bool fail = false;
    if (lane < nseg) {
      const int n = F.scnt[lane];
      const int len = F.hi[my_g] - F.lo[my_g] + 1;
      int lo = 0, hi = len;
      double v = 0.0;
      const double vp = __longlong_as_double((long long)F.spart[lane]);
      const double vw = __longlong_as_double((long long)F.sfw[lane]);
      if (n == 1) {                                    // (an empty range sums to 0.0 at any v)
        const uint32_t lh = F.slohi[lane];
        lo = (int)(lh & 0xFFFFu); hi = (int)(lh >> 16); v = vp;
      } else if (!(vp > vw)) {
        v = vw;                                        // dominated by a whole-locus run
      } else {
        fail = true;                                   // several envelope runs: the wave form
      }
      hi = max(hi, lo);
      // (a whole-locus run -- the usual owner hit -- by the shorter closed form; pw_run_sum
      // gives the same bits there, tests/test_pw_const.py)
      const double sum = (lo <= 0 && hi >= len) ? pw_const_sum(len, v) : pw_run_sum(len, lo, hi, v);
      mean = (0.0 + sum) / (double)len;
    }
    TLAP(6);                                           // (stamps: gene scores)
    // every locus unmasked (:420-427): a full known clade's mean >= kmin on it (penalize and
    // kmin <= 0 mask nothing)
    const bool sure_l = lane < nseg && F.fcl[my_f] != K.unknown && mean >= P.kmin;
    const uint64_t sure = wave_or_dpp(sure_l ? 1ull << my_g : 0ull);
    const bool um_all = P.weak != 0 || P.kmin <= 0.0;
    if (__ballot(fail) != 0ull || (!um_all && sure != allG)) {
      hand_on();
      wave_sync();
      continue;
    }
    // crit = min, rank = numpy's mean over the G loci (np_sum_seq order), full clade i on lane i
    double my_r = -__builtin_inf(), my_c = 0.0;
    for (int i = 0; i < nfull; ++i) {
      const int base = i * G;
      const int m8 = G < 8 ? 0 : G - (G & 7);
      double r0 = 0.0, r1 = 0.0, r2 = 0.0, r3 = 0.0, r4 = 0.0, r5 = 0.0, r6 = 0.0, r7 = 0.0;
      double mn = __builtin_inf();
      for (int u = 0; u < m8; u += 8) {                // (u % 8 -> accumulator, in order: straight-line)
        const double x0 = lane_bcast(mean, base + u), x1 = lane_bcast(mean, base + u + 1);
        const double x2 = lane_bcast(mean, base + u + 2), x3 = lane_bcast(mean, base + u + 3);
        const double x4 = lane_bcast(mean, base + u + 4), x5 = lane_bcast(mean, base + u + 5);
        const double x6 = lane_bcast(mean, base + u + 6), x7 = lane_bcast(mean, base + u + 7);
        r0 += x0; r1 += x1; r2 += x2; r3 += x3; r4 += x4; r5 += x5; r6 += x6; r7 += x7;
        mn = x0 < mn ? x0 : mn; mn = x1 < mn ? x1 : mn; mn = x2 < mn ? x2 : mn; mn = x3 < mn ? x3 : mn;
        mn = x4 < mn ? x4 : mn; mn = x5 < mn ? x5 : mn; mn = x6 < mn ? x6 : mn; mn = x7 < mn ? x7 : mn;
      }
      double res = m8 > 0 ? leaf_tree(r0, r1, r2, r3, r4, r5, r6, r7) : 0.0;
      for (int u = m8; u < G; ++u) {
        const double x = lane_bcast(mean, base + u);
        mn = x < mn ? x : mn;
        res += x;
      }
      if (lane == i) { my_r = (0.0 + res) / (double)G; my_c = mn; }
    }
    TLAP(7);                                           // (stamps: mask, crit and rank)
    // ---- explain_one (:585-597): options = full clades with crit >= k1; best by (rank, clade) ----
    const bool mine = lane < nfull;
    const int my_cl = mine ? F.fcl[lane] : -1;
    const bool opt = mine && my_c >= P.k1;
    double br = opt ? my_r : -__builtin_inf(), bcrit = opt ? my_c : 0.0;
    long long bk = opt ? my_cl : -1;
    each_stride([&](auto J) {
      const double r2 = xor_lanes<decltype(J)::value>(br), c2 = xor_lanes<decltype(J)::value>(bcrit);
      const long long k2 = xor_lanes<decltype(J)::value>(bk);
      if (better(r2, k2, br, bk)) { br = r2; bk = k2; bcrit = c2; }
    });
    if (bk < 0) {                                      // no option: explain_two (the wave form)
      hand_on();
      wave_sync();
      continue;
    }
    // meld_one (:621-631): options within --range of the best, LCA of their clades
    int nm = 0, lca = (int)bk;
    const bool in = P.dis1 == 1 && opt && (br - my_r) <= P.range;
    const uint64_t inm = __ballot(in);
    if (P.dis1 == 1) {
      nm = __popcll(inm);
      if (nm == 0) {                                   // negative --range: the wave form's status
        hand_on();
        wave_sync();
        continue;
      }
      if (nm > 1) {                                    // (one option: its own clade)
        int acc = in ? my_cl : -1;
        each_stride([&](auto J) { acc = lca2(K, acc, xor_lanes<decltype(J)::value>(acc)); });
        lca = acc;
      }
      // melded clades in ascending id order (the wave form's segment order)
      int pos = 0;
      for (uint64_t rest = inm; rest; rest &= rest - 1) pos += lane_bcast(my_cl, __builtin_ctzll(rest)) < my_cl ? 1 : 0;
      if (in) K.meld[2 * h0 + 2 * (int64_t)c + pos] = my_cl;
    }
    // ---- the record (set_synteny_one: every locus 'A') ----
    if (lane < G) K.syn[l0 + lane] = 'A';
    if (ann_on && lane < nann) K.annot[l0 * nsys + lane] = F.ahit[lane];
    if (lane == 0) {
      K.call[c] = WF_CALL_NO_LGT;
      K.crit[c] = bcrit;
      K.rank[c] = br;
      K.c1[c] = lca;
      K.c2[c] = -1;
      K.nm1[c] = nm;
      K.iters[c] = 1;
      K.pair_evals[c] = 0;
      ccnt[c] = 0;
      cleaves[c] = 0;
      pend[c] = 0;
    }
    wave_sync();                                       // the slice is reused by the next contig
    TLAP(8);                                           // (stamps: explain_one, meld_one, record)
    WF_STAMPS_ONLY(if (tsamp_ && lane == 0) atomicAdd(&g_tstamps[15], 1ull));
  }
}

// The staged path's counts of the contigs of more hits than any wave slice (the cfg5 stress
// shape; k_triage hands them on): attachments and numpy leaves (k_wave's ccnt /
// cleaves, with the ordered-loci binary search), pend 1 -- straight to the staged kernels,
// where the wave forms would load every hit only to find the contig does not fit.
// Unordered or overlapping loci, more than 64, --min-overlap 0: left to the wave form
// (pend kPendTriage).  Launched after k_triage, only when the batch has such contigs.
__global__ __launch_bounds__(64) void k_count(const SArgs S, int64_t* ccnt, int64_t* cleaves, int32_t* pend) {
  __shared__ int s_lo[kTrLoc], s_hi[kTrLoc], s_nl[kTrLoc];
  __shared__ int8_t s_st[kTrLoc];
  const KArgs& K = S.k;
  const DevParams& P = K.p;
  const int lane = threadIdx.x;
  unsigned long long n_staged = 0;
  auto leaves = [&](int len) {                       // numpy leaves of a locus (the LUT's counts)
    return (len / kNpyBuf) * (S.lut_off[kNpyBuf + 1] - S.lut_off[kNpyBuf]) +
           (S.lut_off[len % kNpyBuf + 1] - S.lut_off[len % kNpyBuf]);
  };
  for (int c = blockIdx.x; c < K.n_contigs; c += gridDim.x) {
    const int64_t h0 = K.hit_off[c], h1 = K.hit_off[c + 1];
    if (h1 - h0 <= kTrBig) continue;                 // (k_triage handed it on: pend kPendTriage)
    const int64_t l0 = K.loc_off[c];
    const int G = (int)(K.loc_off[c + 1] - l0);
    int clo = 0, chi = -1, cst = 0;
    if (lane < G && G <= kTrLoc) {
      const int a = K.lstart[l0 + lane], e = K.lend[l0 + lane];
      clo = min(a, e);
      chi = max(a, e);
      cst = K.lstrand[l0 + lane];
    }
    const int cprev = __shfl_up(chi, 1, 64);
    if (!(G > 0 && G <= kTrLoc && P.min_overlap > 0.0 && __ballot(lane < G && lane >= 1 && clo <= cprev) == 0ull))
      continue;
    if (lane < G) { s_lo[lane] = clo; s_hi[lane] = chi; s_st[lane] = (int8_t)cst; s_nl[lane] = leaves(chi - clo + 1); }
    wave_sync();
    long long n_att = 0, nl = 0;
    for (int64_t hb = h0; hb < h1; hb += 64 * kCntR) {   // kCntR batches' loads issued together
      uint32_t r_k[kCntR];
      int r_qlo[kCntR], r_qhi[kCntR];
#pragma unroll
      for (int r = 0; r < kCntR; ++r) {
        const int64_t h = hb + 64 * r + lane;
        r_k[r] = 0u; r_qlo[r] = 0; r_qhi[r] = 0;
        if (h < h1) { r_k[r] = K.hkey[h]; r_qlo[r] = K.qlo[h]; r_qhi[r] = K.qhi[h]; }
      }
#pragma unroll
      for (int r = 0; r < kCntR; ++r) {
        if (hb + 64 * r + lane >= h1 || !(r_k[r] & kKeyScov)) continue;
        const int qlo = r_qlo[r], qhi = r_qhi[r], hs = (r_k[r] & kKeyMinus) ? 1 : 0;
        int g = 0;
#pragma unroll
        for (int k = 32; k > 0; k >>= 1)
          if (g + k <= G && s_hi[g + k - 1] < qlo) g += k;
        for (; g < G; ++g) {
          const int lo = s_lo[g];
          if (lo > qhi) break;
          const int len = s_hi[g] - lo + 1;
          if (attaches(P, qlo, qhi, hs, lo, len, s_st[g])) {
            ++n_att;
            nl += s_nl[g];                             // (per locus, staged above: no table loads here)
          }
        }
      }
    }
    n_att = wave_sum_dpp(n_att);
    nl = wave_sum_dpp(nl);
    if (lane == 0) {
      ccnt[c] = n_att;
      cleaves[c] = nl;
      pend[c] = 1;                                   // staged from level 0
    }
    ++n_staged;
    wave_sync();
  }
  if (lane == 0 && n_staged && S.fail_ctr) atomicAdd(S.fail_ctr, n_staged);   // (one add per wave)
}


}  // namespace

WF_STAMP_READER(triage, g_tstamps, 16)

template <bool SYSKEY>
int triage_per_cu() {
  static const int per_cu = [] {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, reinterpret_cast<const void*>(&k_triage<SYSKEY>), 64, 0) !=
            hipSuccess || b < 1)
      b = 1;
    return b;
  }();
  return per_cu;
}

hipError_t pack_keys(const KArgs& k, int64_t n_hits, uint32_t* key, int cus, hipStream_t s) {
  if (n_hits > 0)
    hipLaunchKernelGGL(k_pack_keys, dim3((unsigned)std::min<int64_t>((n_hits + 255) / 256, (int64_t)cus * 16)),
                       dim3(256), 0, s, k, n_hits, key);
  return hipGetLastError();
}

hipError_t launch_triage(const SArgs& sa, int64_t* ccnt, int64_t* cleaves, int32_t* pend, int max_hits, int cus,
                         hipStream_t s) {
  const int N = sa.k.n_contigs;
  if (sa.k.n_sys <= 6) {
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(N, (int64_t)cus * triage_per_cu<true>()));
    hipLaunchKernelGGL(k_triage<true>, dim3(grid), dim3(64), 0, s, sa, ccnt, cleaves, pend);
  } else {
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(N, (int64_t)cus * triage_per_cu<false>()));
    hipLaunchKernelGGL(k_triage<false>, dim3(grid), dim3(64), 0, s, sa, ccnt, cleaves, pend);
  }
  if (max_hits > kTrBig)
    hipLaunchKernelGGL(k_count, dim3((unsigned)std::min<int64_t>(N, (int64_t)cus * 32)), dim3(64), 0, s, sa, ccnt,
                       cleaves, pend);
  return hipGetLastError();
}

}  // namespace wf
