// Per-contig wave kernels of the contig-scoring path (gfx950 / MI355X).
//
// One wave64 carries one contig through the whole path, alone: each workgroup is a single
// wave with its own LDS slice, so no wave ever waits on another (no workgroup barrier) and
// a CU holds as many independent contigs as the slices allow.  Per contig:
//   attachments (orgscorer.py:359-392)        lane per hit, loci in LDS, wave scan for slots
//   (clade, locus) sort (:394-406)            bitonic in registers: R keys per lane, strides
//                                             < 64 by shuffles, >= 64 inside the lane
//   segment means (:399-406)                  lane per segment (numpy closed forms), the wave
//                                             together for multi-run segments
//   maxes, weak loci, Contig.score, explain_one, meld_one (:407-429, :447-461, :585-597,
//                                             :621-631)   lane per clade run
// Two forms of the same kernel:
//   k_wave<CAP, false>  every contig, level 0, explain_one only (small slice, high occupancy)
//   k_wave<CAP, true>   the contigs the first one handed over: explain_two (:599-619), the
//                       LGT checks and meld_two (:633-744, eval_two of wf_device.h), and the
//                       roll-up loop (:431-445, :566-583) -- attachments re-keyed to the parent
//                       clade in LDS, level after level
//   k_wave<CAP, false, true> (ROLL)  roll-up level L >= 1 of the contigs the level before
//                       raised (WF_MODE_LEVEL0): hits re-attached with clade anc[taxon]
// In WF_MODE_LEVEL0 the first form hands a contig explain_one leaves open to k_dump_sparse
// with its segment table (explain_two there; a raised contig joins the next ROLL launch's
// list).  A contig no wave form can finish (more attachments than a slice holds, more
// than 64 loci, a leaf table, segment or explain_two state the slice cannot hold) is handed
// to the staged path (wf_staged.hip) with its attachment and leaf counts; the staged level
// 0 then runs on those contigs only.  Contigs finished here never write attachments, keys
// or segment records to HBM: their traffic is the hits and loci read once plus the record.
#include <algorithm>
#include <cstdlib>

#include "wf_device.h"
#include "wf_lanes.h"

namespace wf {

namespace {

constexpr int kSlotBits = 9;         // key = clade << 15 | locus << 9 | attachment slot
constexpr int kCladeShift = 15;
constexpr uint32_t kSlotMask = (1u << kSlotBits) - 1;
constexpr int kLoc0 = 64;            // loci per contig (locus bitmasks are 64-bit)
constexpr int kLut0 = 256;           // packed leaf-table entries of the contig's loci
constexpr int kAnn0 = 64;            // (locus, system) annotation slots
constexpr int kRuns0 = 64;           // envelope runs of a multi-attachment segment ...
constexpr int kMultiAtt0 = 32;       // ... so at most 32 attachments (2 * 32 - 1 runs);
constexpr int kRunsL0 = 32;          // the level-0 form: 16 attachments (a 10 KB slice:
constexpr int kMultiAttL0 = 16;      // 16 waves per CU, see WaveSmem)
constexpr int kXcds = 8;             // MI355X: 8 XCDs of 32 CUs, each with its own L2
// resident waves per SIMD of the roll-up launches: 4 (128 VGPRs, some spilled) beat 3 (168,
// none) by 0.35 ms of roll-up per cfg4 pass on one box (r4f: their few contigs per wave
// want occupancy more than registers; again r5u: 3 waves +0.45 ms)
constexpr int kRollWaves = 4;
constexpr int kPot0 = 64;            // potential clades of an in-slice explain_two ...
constexpr int kS0 = 640;          // ... and their score rows (potential clades x loci;
                                     // 640 = 64 x 10 and a 20 KB slice: 8 waves per CU)

// One wave's LDS slice.  `scr` is reused phase by phase (offsets in the accessors):
//   attachments:  hit[CAP] | sm[CAP] | abest[64] | ahit[64]      (annotations)
//   means:        v[CAP] | runs | list[CAP] | rc[CAP]            (multi-run segments; the
//                 level-0 pruning: segments to evaluate, clade-run sizes -- !FULL only)
//   explain_one:  v | rank[CAP] (FULL; else in sc) | mem[CAP] | mx[64]
//   explain_two:  v | cl[CAP] | sib[CAP] | hm[CAP] | S[kS0] | masks, loci lists (FULL only)
// key, lohi and sc (by attachment slot) live across roll-up levels.  Keys are 32-bit:
// clade << 15 | locus << 9 | slot (clade ids < 2^17, checked on the host).
// LDS per slice sets the occupancy (160 KB per CU): CAP 224, level-0 form = 10,096 B -> 16
// waves per CU (the VGPR limit too); the FULL form at CAP 256 = 20,296 B -> 8.
template <int CAP, bool FULL>
struct WaveSmem {
  static constexpr int cmax(int a, int b) { return a > b ? a : b; }
  static constexpr int kRunsN = FULL ? kRuns0 : kRunsL0;
  using Runs = WaveRunsT<kRunsN>;
  static constexpr int kRunsB = (int)sizeof(Runs);
  static constexpr int kScr = FULL ? 24 * CAP + 8 * kS0 + 2048
                                   : cmax(cmax(8 * CAP + 768, 8 * CAP + kRunsB + 3 * CAP), 12 * CAP + 512);
  uint32_t key[CAP];                 // keys by slot, then in sorted order
  uint32_t lohi[CAP];                // by slot: site range lo | hi << 16
  double sc[CAP];                    // by slot: score
  uint32_t seg[CAP + 2];             // per segment: its head key, slot field = first sorted position
  uint32_t lut[kLut0];               // packed leaf tables, locus g at lbase[g]
  int lo[kLoc0], len[kLoc0];
  int16_t lbase[kLoc0], nl1[kLoc0];
  int8_t st[kLoc0];
  alignas(16) char scr[kScr];
  __device__ int* hit() { return reinterpret_cast<int*>(scr); }
  __device__ int* sm() { return reinterpret_cast<int*>(scr) + CAP; }
  __device__ unsigned long long* abest() { return reinterpret_cast<unsigned long long*>(scr + 8 * CAP); }
  __device__ int* ahit() { return reinterpret_cast<int*>(scr + 8 * CAP + 8 * kAnn0); }
  __device__ double* v() { return reinterpret_cast<double*>(scr); }
  __device__ Runs& runs() { return *reinterpret_cast<Runs*>(scr + 8 * CAP); }
  __device__ uint16_t* list() { return reinterpret_cast<uint16_t*>(scr + 8 * CAP + kRunsB); }       // !FULL
  __device__ uint8_t* rc() { return reinterpret_cast<uint8_t*>(scr + 8 * CAP + kRunsB + 2 * CAP); }  // !FULL
  __device__ double* rank() { return FULL ? reinterpret_cast<double*>(scr + 8 * CAP) : sc; }
  __device__ int* mem() { return reinterpret_cast<int*>(scr + (FULL ? 16 : 8) * CAP); }
  __device__ unsigned long long* mx() { return reinterpret_cast<unsigned long long*>(scr + (FULL ? 20 : 12) * CAP); }
  __device__ int* cl() { return reinterpret_cast<int*>(scr + 8 * CAP); }
  __device__ int* sib() { return reinterpret_cast<int*>(scr + 12 * CAP); }
  __device__ uint64_t* hm() { return reinterpret_cast<uint64_t*>(scr + 16 * CAP); }
  __device__ double* S() { return reinterpret_cast<double*>(scr + 24 * CAP); }
  __device__ uint64_t* pmask() { return reinterpret_cast<uint64_t*>(scr + 24 * CAP + 8 * kS0); }   // [kPot0]
  __device__ int* ign() { return reinterpret_cast<int*>(scr + 24 * CAP + 8 * kS0 + 8 * kPot0); }  // [64]
  __device__ int* um() { return ign() + 64; }
  __device__ int* loc_len() { return ign() + 128; }
  __device__ uint8_t* best_syn() { return reinterpret_cast<uint8_t*>(ign() + 192); }    // [64]
};

static_assert(sizeof(WaveSmem<224, false>) <= 160 * 1024 / 16, "level-0 slice: 16 waves per CU");
static_assert(sizeof(WaveSmem<256, true>) <= 160 * 1024 / 8, "FULL slice: 8 waves per CU");

__device__ __forceinline__ int leaves_for(const SArgs& S, int len) {
  return (len / kNpyBuf) * (S.lut_off[kNpyBuf + 1] - S.lut_off[kNpyBuf]) +
         (S.lut_off[len % kNpyBuf + 1] - S.lut_off[len % kNpyBuf]);
}

__device__ __forceinline__ uint64_t lanes_below() { return (1ull << lane_id()) - 1ull; }

// (every lane active: wf_lanes.h)
__device__ __forceinline__ int wave_excl_scan(int v, int* total) { return wave_excl_scan_dpp(v, total); }

__device__ __forceinline__ int wave_lca(const KArgs& K, int acc) {
  each_stride([&](auto J) { acc = lca2(K, acc, xor_lanes<decltype(J)::value>(acc)); });
  return acc;
}

// Ascending bitonic sort of N = 64 * R keys, element lane + 64 r in x[r].  The merge
// size k is a runtime loop (the unrolled network of every R and key width would not fit
// the instruction cache); the strides j inside it are static, so in-lane partners are
// static register indices and lane partners static shuffles.
// Ascending bitonic sort of N = 64 * R keys, element R * lane + r in x[r] (lane-major: the
// strides below R stay inside a lane, element stride j >= R is lane stride j / R, so the
// most frequent strides -- every merge runs 1, 2, 4, ... -- are register swaps and one-DPP
// exchanges).  The merge size k is a runtime loop (the unrolled network would not fit the
// instruction cache); the strides inside it are static.
template <int R, class T>
__device__ __forceinline__ void wave_sort(T (&x)[R]) {
  const int lane = lane_id();
  constexpr int N = 64 * R;
#pragma unroll 1
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
    for (int jl = 32; jl >= 1; jl >>= 1) {           // element strides jl * R: partner lane ^ jl
      if (jl * R >= k) continue;
      // i & (jl * R) and i & k (k > jl * R >= R) depend on the lane alone
      const bool keep_min = ((lane & jl) == 0) == (((lane * R) & k) == 0);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const T y = xor_lanes_rt(x[r], jl);
        const T lo = y < x[r] ? y : x[r], hi = y < x[r] ? x[r] : y;
        x[r] = keep_min ? lo : hi;
      }
    }
#pragma unroll
    for (int j = R / 2; j >= 1; j >>= 1) {           // strides below R: element r ^ j, same lane
      if (j >= k) continue;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r & j) continue;
        const bool asc = (((lane * R) | r) & k) == 0;
        const T a = x[r], b = x[r | j];
        const T lo = a < b ? a : b, hi = a < b ? b : a;
        x[r] = asc ? lo : hi;
        x[r | j] = asc ? hi : lo;
      }
    }
  }
}

// The slice's keys in sorted order (one network of 64 * R 32-bit keys, lane-major), and the
// attachments' ranges and scores moved along: afterwards attachment t's lohi / sc sit at t
// and its key's slot field is t, so every later read goes straight to position t (no
// key -> slot hop: the loads of a segment's attachments issue together).  Nothing reads
// the insertion order after the first sort (F.hit / F.sm: annotation pass 2, before it).
//
// PERMUTE = false (level 0): keys only, attachments reached through the keys' slot fields.
template <int R, bool PERMUTE = true, class SM>
__device__ __forceinline__ void sort_slice(SM& F, int n_att) {
  const int lane = lane_id();
  uint32_t y[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int t = R * lane + r;
    y[r] = t < n_att ? F.key[t] : ~0u;
  }
  wave_sort<R>(y);
  if (!PERMUTE) {
    wave_sync();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int t = R * lane + r;
      if (t < n_att) F.key[t] = y[r];
    }
    wave_sync();
    return;
  }
  uint32_t lh[R];
  double sv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int t = R * lane + r;
    lh[r] = 0u;
    sv[r] = 0.0;
    if (t < n_att) {
      const int slot = (int)(y[r] & kSlotMask);
      lh[r] = F.lohi[slot];
      sv[r] = F.sc[slot];
    }
  }
  wave_sync();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int t = R * lane + r;
    if (t < n_att) {
      F.key[t] = (y[r] & ~kSlotMask) | (uint32_t)t;
      F.lohi[t] = lh[r];
      F.sc[t] = sv[r];
    }
  }
  wave_sync();
}

// Segment s: (clade, locus) and its sorted attachment range [seg_first(s), seg_first(s+1)).
template <class SM>
__device__ __forceinline__ int2 cg_of(SM& F, int s) {
  const uint32_t w = F.seg[s];
  return make_int2((int)(w >> kCladeShift), (int)((w >> kSlotBits) & (kLoc0 - 1)));
}
template <class SM>
__device__ __forceinline__ int seg_first(SM& F, int s) { return (int)(F.seg[s] & kSlotMask); }
__device__ __forceinline__ int lo16(uint32_t w) { return (int)(w & 0xFFFFu); }
__device__ __forceinline__ int hi16(uint32_t w) { return (int)(w >> 16); }

// The slice's attachments for SegAttT (wf_device.h): sorted position t -> range, score (at
// t since sort_slice).
struct SliceSrc {
  const uint32_t* key;
  const uint32_t* lohi;
  const double* sc;
  __device__ __forceinline__ int idx(int t) const { return t; }
  __device__ __forceinline__ void att(int a, int& l, int& h, double& v) const {
    const uint32_t w = lohi[a];
    l = lo16(w); h = hi16(w); v = sc[a];
  }
};
// Level 0 without the data move: sorted position t -> its key's slot field -> range, score.
struct SliceSrcKey {
  const uint32_t* key;
  const uint32_t* lohi;
  const double* sc;
  __device__ __forceinline__ int idx(int t) const { return (int)(key[t] & kSlotMask); }
  __device__ __forceinline__ void att(int a, int& l, int& h, double& v) const {
    const uint32_t w = lohi[a];
    l = lo16(w); h = hi16(w); v = sc[a];
  }
};

// Exact mean of one segment (sorted attachments [kb, ke), any count) by one lane: every
// numpy leaf by SegAttT::leaf (closed forms, else the envelope's runs), folded in tree
// order on a register stack.  For the roll-up levels, where many segments per block have
// several attachments and one lane each beats one wave each.
template <class Src, class LT>
__device__ __noinline__ double lane_seg_mean(Src src, int kb, int ke, LT lt, int nl, int len) {
  SegAttT<Src> at;
  at.load(src, kb, ke);
  SumStack stk;
  for (int q = 0; q < nl; ++q) {
    const int4 e = lt(q);
    stk.push(at.leaf(src, e.x, e.y));
    for (int a = 0; a < e.z; ++a) stk.add_top();
  }
  return (0.0 + stk.s0) / (double)len;
}

// Exact means of the multi-attachment segments of one 64-segment chunk (lanes of `mlist`,
// each with its segment's sorted attachments [kb, ke), leaf count nl <= 64, locus length
// len and packed leaf table lut), one numpy LEAF per lane rather than one segment per lane:
// whole segments are packed into rounds of at most 64 leaves (a lane-order prefix sum of
// nl), lane i of a round evaluates leaf i - start of the segment whose leaves start at or
// below it (SegAttT::leaf, as lane_seg_mean), and the segment's own lane folds its leaves in
// tree order (SumStack) from W.lv.  Same leaf values, same fold, so the same bits as
// lane_seg_mean; a round costs one leaf per lane instead of a whole segment.  W.z maps a
// round's start position to its segment's lane.  Returns the mean on the segment's lane.
template <int R, class Src>
__device__ __forceinline__ double flat_leaf_means(Src src, const uint32_t* lut, uint64_t mlist, int kb, int ke,
                                               int nl, int len, WaveRunsT<R>& W) {
  const int lane = lane_id();
  double mean = 0.0;
  for (uint64_t rem = mlist; rem;) {
    const bool mine = (rem >> lane) & 1ull;
    const int my_nl = mine ? nl : 0;
    int total = 0;
    const int start = wave_excl_scan_dpp(my_nl, &total);
    const bool take = mine && start + my_nl <= 64;
    const uint64_t tk = __ballot(take);
    if (take) W.z[start] = lane;
    const uint64_t starts = wave_or_dpp(take ? 1ull << start : 0ull);
    const int last = 63 - __clzll(tk);
    const int used = lane_bcast(start + my_nl, last);  // leaves of this round
    wave_sync();
    const uint64_t le = lane == 63 ? ~0ull : (2ull << lane) - 1ull;
    const uint64_t st_le = starts & le;
    const int p = st_le ? 63 - __clzll(st_le) : 0;
    const int own = lane < used ? W.z[p] : last;
    // the owner's segment (all lanes active for the permutes)
    const int okb = __shfl(kb, own, 64), oke = __shfl(ke, own, 64);
    const uintptr_t olut = (uintptr_t)__shfl((long long)(uintptr_t)lut, own, 64);
    if (lane < used) {
      const int4 e = PackedLut{reinterpret_cast<const uint32_t*>(olut)}(lane - p);
      SegAttT<Src, 1> at;                             // (multi segments: read from LDS)
      at.load(src, okb, oke);
      W.lv[lane] = at.leaf(src, e.x, e.y);
    }
    wave_sync();
    if (take) {
      SumStack stk;
      const PackedLut lt{lut};
      for (int q = 0; q < nl; ++q) {
        stk.push(W.lv[start + q]);
        const int z = lt(q).z;
        for (int a = 0; a < z; ++a) stk.add_top();
      }
      mean = (0.0 + stk.s0) / (double)len;
    }
    wave_sync();                                      // (W.lv, W.z: the next round's)
    rem &= ~tk;
  }
  return mean;
}

// Contig.score of the clade run starting at segment t (orgscorer.py:447-461): crit = min
// and rank = np.mean over the Gu unmasked loci of the clade's row, whose entries are the
// run's segment means and 0.0 elsewhere.  numpy's order (np_sum_seq): fewer than 8 values
// are added in order from 0.0; else value u goes to accumulator u % 8 while u < Gu - Gu % 8,
// the eight are combined as a tree and the rest added in order.  Scores are >= 0, so the
// 0.0 entries change no partial sum and only the run's segments are visited.
template <class SM>
__device__ __forceinline__ void sparse_score(SM& F, const double* v, int t, int ns, int clade, uint64_t um,
                                             int Gu, double& crit, double& rank) {
  const int m8 = Gu < 8 ? 0 : Gu - (Gu & 7);
  double r0 = 0.0, r1 = 0.0, r2 = 0.0, r3 = 0.0, r4 = 0.0, r5 = 0.0, r6 = 0.0, r7 = 0.0;
  double mn = 0.0;
  int cnt = 0;
  int q = t;
  for (; q < ns; ++q) {                              // the accumulators (Gu >= 8)
    const int2 cq = cg_of(F, q);
    if (cq.x != clade) break;
    if (!((um >> cq.y) & 1ull)) continue;
    const double x = v[q];
    mn = (cnt == 0 || x < mn) ? x : mn;
    ++cnt;
    const int u = __popcll(um & ((1ull << cq.y) - 1ull));
    if (u >= m8) continue;
    const int a = u & 7;
    r0 = a == 0 ? r0 + x : r0; r1 = a == 1 ? r1 + x : r1;
    r2 = a == 2 ? r2 + x : r2; r3 = a == 3 ? r3 + x : r3;
    r4 = a == 4 ? r4 + x : r4; r5 = a == 5 ? r5 + x : r5;
    r6 = a == 6 ? r6 + x : r6; r7 = a == 7 ? r7 + x : r7;
  }
  double res = m8 > 0 ? leaf_tree(r0, r1, r2, r3, r4, r5, r6, r7) : 0.0;
  for (int p = t; p < q; ++p) {                      // the rest, in order
    const int2 cp = cg_of(F, p);
    if (!((um >> cp.y) & 1ull)) continue;
    if (__popcll(um & ((1ull << cp.y) - 1ull)) >= m8) res += v[p];
  }
  crit = cnt < Gu ? 0.0 : mn;
  rank = (0.0 + res) / (double)Gu;
}

// Contig.score of the clade run starting at segment t (t uniform; orgscorer.py:447-461) by
// the whole wave: lane i holds segment t + i (a run has at most 64 segments, one per locus).
// crit = the min over the run's unmasked segments (0.0 when fewer than Gu); the rank only
// when crit >= k1 (an option then has a segment on every unmasked locus, so the u-th
// unmasked locus is the u-th used lane), summed in sparse_score's numpy order by a uniform
// walk over the used lanes.  Returns the run's clade.
template <class SM>
__device__ __forceinline__ int wave_run_score(SM& F, const double* v, int t, int ns, uint64_t um, int Gu,
                                              double k1, double& crit, double& rank) {
  const int lane = lane_id();
  const int clade = (int)(F.seg[t] >> kCladeShift);
  const int q = t + lane;
  bool in = false;
  int g = 0;
  double x = 0.0;
  if (q < ns) {
    const uint32_t w = F.seg[q];
    in = (int)(w >> kCladeShift) == clade;
    g = (int)((w >> kSlotBits) & (kLoc0 - 1));
    x = v[q];
  }
  const uint64_t out = __ballot(!in);                // the run: lanes below the first other clade
  const int len = out ? __builtin_ctzll(out) : 64;
  const bool use = lane < len && ((um >> g) & 1ull);
  const uint64_t used = __ballot(use);
  const int cnt = __popcll(used);
  double mn = use ? x : __builtin_inf();
  mn = wave_butterfly(mn, [](double a, double b) { return b < a ? b : a; });
  crit = (cnt < Gu || cnt == 0) ? 0.0 : mn;
  rank = 0.0;
  if (crit >= k1) {
    const int m8 = Gu < 8 ? 0 : Gu - (Gu & 7);
    double r0 = 0.0, r1 = 0.0, r2 = 0.0, r3 = 0.0, r4 = 0.0, r5 = 0.0, r6 = 0.0, r7 = 0.0;
    uint64_t rest = used;
    for (int u = 0; u < m8; ++u, rest &= rest - 1) {  // value u -> accumulator u % 8, in order
      const double xu = lane_bcast(x, __builtin_ctzll(rest));
      switch (u & 7) {
        case 0: r0 += xu; break;
        case 1: r1 += xu; break;
        case 2: r2 += xu; break;
        case 3: r3 += xu; break;
        case 4: r4 += xu; break;
        case 5: r5 += xu; break;
        case 6: r6 += xu; break;
        default: r7 += xu; break;
      }
    }
    double res = m8 > 0 ? leaf_tree(r0, r1, r2, r3, r4, r5, r6, r7) : 0.0;
    for (; rest; rest &= rest - 1) res += lane_bcast(x, __builtin_ctzll(rest));   // the rest, in order
    rank = (0.0 + res) / (double)Gu;
  }
  return clade;
}

// explain_two + LGT filters + meld_two for one level in the slice (decide_two's arithmetic,
// orgscorer.py:599-619, 633-744; eval_two / pair_rank / pair_crit of wf_device.h on a
// Contig whose rows are the potential clades first, then the others).  Returns kDecDone
// (written), kDecStop, kDecRaise, or -1 when the state does not fit (staged path).
// eval_two inlined into wave_two: out of line, every call spilled the caller's live VGPRs
// to scratch (cfg4: the FULL form 8.56 -> 8.35 ms inlined)
__device__ __forceinline__ OptEval eval_two_call(const KArgs& K, const Contig& C, int Pcount, int pa, int pb,
                                              const uint8_t* best, uint8_t* out) {
  return eval_two(K, C, Pcount, pa, pb, best, out);
}

template <int CAP>
__device__ __noinline__ int wave_two(const SArgs& S, WaveSmem<CAP, true>& F, int c, int64_t h0, int64_t l0, int G,
                                     int ns, uint64_t um, int Gu, int iteration, int64_t& pair_evals) {
  const KArgs& K = S.k;
  const DevParams& P = K.p;
  const int lane = lane_id();
  const double* v = F.v();
  const uint64_t allG = G >= 64 ? ~0ull : ((1ull << G) - 1ull);
  // a clade run starting at segment t: max score over all G loci (missing loci are 0.0),
  // loci at or above the sister threshold, loci present
  auto run_scan = [&](int t, int clade, double& mx, uint64_t& hmask, uint64_t& present) {
    mx = -__builtin_inf();
    hmask = 0;
    present = 0;
    for (int q = t; q < ns; ++q) {
      const int2 cq = cg_of(F, q);
      if (cq.x != clade) break;
      const double x = v[q];
      mx = x > mx ? x : mx;
      present |= 1ull << cq.y;
      if (x >= P.sister_thr) hmask |= 1ull << cq.y;
    }
    if (present != allG) {
      mx = 0.0 > mx ? 0.0 : mx;
      if (0.0 >= P.sister_thr) hmask |= allG & ~present;
    }
  };
  // pass A: clades, potential clades (:603-605), root present
  int Pn = 0, Pp = 0;
  bool root = false;
  for (int t0 = 0; t0 < ns; t0 += 64) {
    const int t = t0 + lane;
    bool head = false, pot = false;
    if (t < ns) {
      const int clade = cg_of(F, t).x;
      head = t == 0 || cg_of(F, t - 1).x != clade;
      if (head) {
        double mx;
        uint64_t hmk, pres;
        run_scan(t, clade, mx, hmk, pres);
        pot = mx >= P.k2;
        root = root || clade == K.root;
      }
    }
    Pn += __popcll(__ballot(head));
    Pp += __popcll(__ballot(pot));
  }
  root = __ballot(root) != 0ull;
  pair_evals += (int64_t)Pp * (Pp - 1) / 2;
  if (lane == 0) note_ppot(K, c, iteration, Pp);
  if (Pp > kPot0 || Pp * G > kS0 || Pn > CAP) return -1;
  // pass B: rows (potential clades first, clade order), S rows, sister data
  double* Sm = F.S();
  for (int i = lane; i < Pp * G; i += 64) Sm[i] = 0.0;
  wave_sync();
  int prow = 0, nrow = Pp;
  for (int t0 = 0; t0 < ns; t0 += 64) {
    const int t = t0 + lane;
    bool head = false, pot = false;
    int clade = -1;
    double mx = 0.0;
    uint64_t hmk = 0, pres = 0;
    if (t < ns) {
      clade = cg_of(F, t).x;
      head = t == 0 || cg_of(F, t - 1).x != clade;
      if (head) {
        run_scan(t, clade, mx, hmk, pres);
        pot = mx >= P.k2;
      }
    }
    const uint64_t pm = __ballot(pot), nm = __ballot(head && !pot);
    if (head) {
      const int row = pot ? prow + __popcll(pm & lanes_below()) : nrow + __popcll(nm & lanes_below());
      F.cl()[row] = clade;
      F.sib()[row] = K.sibp[clade];
      F.hm()[row] = hmk;
      if (pot)
        for (int q = t; q < ns; ++q) {
          const int2 cq = cg_of(F, q);
          if (cq.x != clade) break;
          Sm[row * G + cq.y] = v[q];
        }
    }
    prow += __popcll(pm);
    nrow += __popcll(nm);
  }
  if (lane < G) {
    F.ign()[lane] = ((um >> lane) & 1ull) ? 0 : 1;
    F.loc_len()[lane] = F.len[lane];
    if ((um >> lane) & 1ull) F.um()[__popcll(um & lanes_below())] = lane;
  }
  wave_sync();
  Contig C;
  C.l0 = l0;
  C.G = G;
  C.h0 = h0;
  C.mbase = 2 * h0 + 2 * (int64_t)c;
  C.S = Sm;
  C.ign = F.ign();
  C.um = F.um();
  C.loc_len = F.loc_len();
  C.cl_id = F.cl();
  C.sib_of = F.sib();
  C.hm = F.hm();
  const uint64_t full = Gu >= 64 ? ~0ull : ((1ull << Gu) - 1ull);
  for (int i = lane; i < Pp; i += 64) {             // "crit >= k2" masks over the unmasked loci
    uint64_t m = 0;
    for (int u = 0; u < Gu; ++u)
      if (Sm[i * G + C.um[u]] >= P.k2) m |= 1ull << u;
    F.pmask()[i] = m;
  }
  wave_sync();
  const uint64_t* pmask = F.pmask();
  // pass 1: best pair over all pairs clade1 < clade2 (rows in name order), ties -> later pair
  double br = -__builtin_inf();
  long long bk = -1;
  for (int i = 0; i + 1 < Pp; ++i) {
    const uint64_t mi = pmask[i];
    for (int j = i + 1 + lane; j < Pp; j += 64) {
      if ((mi | pmask[j]) != full) continue;
      const double r = pair_rank(C, i, j, Gu);
      const long long key = (long long)i * Pp + j;
      if (better(r, key, br, bk)) { br = r; bk = key; }
    }
  }
  each_stride([&](auto J) {
    const double r2 = xor_lanes<decltype(J)::value>(br);
    const long long k2 = xor_lanes<decltype(J)::value>(bk);
    if (better(r2, k2, br, bk)) { br = r2; bk = k2; }
  });
  if (bk >= 0) {
    const int bi = (int)(bk / Pp), bj = (int)(bk % Pp);
    int b_ok = 0, b_dir = 0, b_c1p = 0, b_c2p = 0;
    double bcrit = 0.0;
    if (lane == 0) {
      const OptEval e = eval_two_call(K, C, Pn, bi, bj, nullptr, F.best_syn());
      b_ok = e.ok; b_dir = e.dir; b_c1p = e.c1p; b_c2p = e.c2p;
      bcrit = pair_crit(C, bi, bj, Gu);
    }
    b_ok = lane_bcast(b_ok, 0); b_dir = lane_bcast(b_dir, 0);
    b_c1p = lane_bcast(b_c1p, 0); b_c2p = lane_bcast(b_c2p, 0);
    bcrit = lane_bcast(bcrit, 0);
    wave_sync();
    // pass 2: options within --range of the best get the LGT filters (:636-639)
    int n_in = 0;
    bool all_ok = true, all_same = true;
    uint64_t b1 = 0, b2 = 0;
    for (int i = 0; i + 1 < Pp; ++i) {
      const uint64_t mi = pmask[i];
      for (int j = i + 1 + lane; j < Pp; j += 64) {
        if ((mi | pmask[j]) != full) continue;
        const double r = pair_rank(C, i, j, Gu);
        if (!((br - r) <= P.range)) continue;
        const OptEval e = eval_two_call(K, C, Pn, i, j, F.best_syn(), nullptr);
        ++n_in;
        all_ok = all_ok && e.ok;
        all_same = all_same && e.same;
        b1 |= 1ull << e.c1p;
        b2 |= 1ull << e.c2p;
      }
    }
    n_in = wave_sum_dpp(n_in);
    b1 = wave_or_dpp(b1);
    b2 = wave_or_dpp(b2);
    all_ok = __ballot(!all_ok) == 0ull;
    all_same = __ballot(!all_same) == 0ull;
    // meld_two (:640-669): 0 none, 1 best as is, 2 meld, 3 unchecked best, 4 upstream crash
    int kind;
    if (n_in == 0) kind = (P.dis2 == 0) ? 3 : (P.dis2 == 1 ? 0 : 4);   // --range < 0
    else if (n_in == 1 || P.dis2 == 0) kind = 1;
    else if (P.dis2 == 1) kind = 0;
    else kind = (all_ok && all_same) ? 2 : 0;
    if (kind == 4) {
      if (lane == 0) K.status[c] = WF_E_BADINPUT;
      return kDecDone;
    }
    bool have_ok = false;
    int lca1 = -1, lca2v = -1;
    const int m1 = __popcll(b1), m2 = __popcll(b2);
    if (kind == 2) {
      const bool in1 = lane < Pp && ((b1 >> lane) & 1ull), in2 = lane < Pp && ((b2 >> lane) & 1ull);
      lca1 = wave_lca(K, in1 ? F.cl()[lane] : -1);
      lca2v = wave_lca(K, in2 ? F.cl()[lane] : -1);
      bool keep = true;
      if (!P.allow_lca) {
        const int nl = lca2(K, lca1, lca2v);
        keep = !(nl == lca1 || nl == lca2v);
      }
      have_ok = keep;                                // melded options are all OK
      if (have_ok) {
        if (in1) K.meld[C.mbase + __popcll(b1 & lanes_below())] = F.cl()[lane];
        if (in2) K.meld[C.mbase + m1 + __popcll(b2 & lanes_below())] = F.cl()[lane];
      }
    } else if (kind == 1) {
      have_ok = b_ok != 0;
    } else if (kind == 3) {
      have_ok = true;
    }
    if (have_ok) {
      if (lane < G) K.syn[l0 + lane] = F.best_syn()[lane];
      if (lane == 0) {
        K.call[c] = WF_CALL_LGT;
        K.crit[c] = bcrit;
        K.rank[c] = br;
        K.dir[c] = (int8_t)b_dir;
        K.c1[c] = (kind == 2) ? lca1 : F.cl()[b_c1p];
        K.c2[c] = (kind == 2) ? lca2v : F.cl()[b_c2p];
        K.nm1[c] = (kind == 2) ? m1 : 0;
        K.nm2[c] = (kind == 2) ? m2 : 0;
        K.iters[c] = (int16_t)iteration;
        K.pair_evals[c] = pair_evals;
      }
      return kDecDone;
    }
  }
  return (Pn == 0 || root) ? kDecStop : kDecRaise;
}

template <int CAP, bool FULL, bool ROLL = false>
// rollup (FULL, WF_MODE_WAVES): carry a contig through its roll-up levels in the slice;
// else (the FULL form's fallback duty in WF_MODE_LEVEL0) hand a raised contig to the staged
// kernels as a level-1 seed.  In WF_MODE_LEVEL0 the roll-up levels run as first-form ROLL
// launches (below), one per level.
// S_arg must stay the first parameter: kernarg_fresh reads the argument block at kernarg
// offset 0.  ROLL (first form only): roll-up level start_level > 0 of the contigs in `list`
// (the wave levels, S.anc set) -- its own instantiation, so profiles tell the level-0 pass
// from the roll-up passes and level 0 carries none of their code.
__global__ __launch_bounds__(64, FULL ? 2 : (ROLL ? kRollWaves : 4)) void k_wave(const SArgs S_arg, int64_t* ccnt, int64_t* cleaves, int32_t* pend,
                                             const int32_t* list, int n_list, const int64_t* n_dev, int rollup,
                                             int start_level_arg) {
  static_assert(!(FULL && ROLL), "the roll-up passes are first-form launches");
  const int start_level = ROLL ? start_level_arg : 0;   // (ROLL: always >= 1)
  if (n_dev) n_list = (int)*n_dev;                   // the list's length, counted on the device
  // a queue hands out n_list contigs in all: waves past that many take none and leave before
  // touching its counter (a short roll-up list over ~4 k waves spent ~50 us in their claims;
  // the static order below deals contigs to every block, so it has no such exit)
  if (S_arg.wq && (int)blockIdx.x >= n_list) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  WaveSmem<CAP, FULL>& F = *reinterpret_cast<WaveSmem<CAP, FULL>*>(smem);
  const int lane = threadIdx.x;
  // XCD-aware contig order.  Workgroups are dealt to the 8 XCDs round-robin (blockIdx % 8),
  // so a plain grid stride puts neighbouring contigs on different XCDs, and the record
  // fields of 8 neighbours (1-8 B each, one array per field) share cache lines that 8 L2s
  // write back partially.  Instead XCD x's j-th workgroup takes contig (8 k + x) * B + j at
  // step k (B = grid / 8): each XCD walks runs of B consecutive contigs.
  const bool xmap = gridDim.x % kXcds == 0;
  const int xb = (int)gridDim.x / kXcds, xj = (int)blockIdx.x / kXcds, xx = (int)blockIdx.x % kXcds;
  for (int it = 0;; ++it) {
    int ci;
    if (S_arg.wq) {
      // a work queue: a wave takes the list's next contig when it finishes one (the roll-up
      // lists are ~20 k contigs of very different cost over ~4 k waves: static striding left
      // the launches tail-bound)
      unsigned long long q = 0;
      if (lane == 0) q = atomicAdd(S_arg.wq, 1ull);
      ci = __builtin_amdgcn_readfirstlane((int)q);
    } else {
      ci = xmap ? (it * kXcds + xx) * xb + xj : (int)blockIdx.x + it * (int)gridDim.x;
    }
    if (ci >= n_list) break;
    const int c = list ? list[ci] : ci;
    WLAP_MARK();
    // The argument block (~1 KB: some 40 array pointers and the parameters) is re-read per
    // contig through an opaque copy of the kernarg pointer (scalar loads, constant cache):
    // held across the whole persistent loop its fields overflowed the SGPR file (204 SGPRs
    // spilled to VGPR lanes, a v_readlane + wait states per use).
    const SArgs& S = kernarg_fresh<SArgs>(S_arg);
    const KArgs& K = S.k;
    const DevParams& P = K.p;
    const int nsys = K.n_sys;
    const bool ann_on = !ROLL && nsys > 0;            // annotations: level 0 only (never raised, :383-392)
    // --weak-loci assign-unknown: the second form leaves every contig the first one handed
    // over to the staged kernels (its pend / counts stand); they carry the virtual row
    if (FULL && P.weak == 2) continue;
    const int64_t h0 = K.hit_off[c], h1 = K.hit_off[c + 1];
    // the first round of hits: every field of up to kHB batches of 64, issued before the loci
    // (their chain -- offsets, loci, leaf counts -- then overlaps these loads)
    constexpr int kHB = 4;
    int r_qlo[kHB], r_qhi[kHB], r_hs[kHB], r_cl[kHB];
    double r_scv[kHB], r_sc[kHB];
    uint32_t r_m[kHB];
    auto load_round = [&](int64_t hq) {
#pragma unroll
      for (int b = 0; b < kHB; ++b) {
        const int64_t h = hq + 64 * b + lane;
        r_qlo[b] = 0; r_qhi[b] = 0; r_hs[b] = 0; r_cl[b] = 0;
        r_scv[b] = 0.0; r_sc[b] = 0.0; r_m[b] = 0u;
        if (h < h1) {
          r_scv[b] = K.scov[h];
          r_qlo[b] = K.qlo[h];
          r_qhi[b] = K.qhi[h];
          if (P.stranded) r_hs[b] = K.hstrand[h];      // (the strand only matters --stranded)
          r_cl[b] = K.taxon[h];
          r_sc[b] = K.score[h];
          if (ann_on) r_m[b] = K.sysmask[h];
        }
      }
    };
    load_round(h0);
    const int64_t l0 = K.loc_off[c];
    const int G = (int)(K.loc_off[c + 1] - l0);
    const int Gs = min(G, kLoc0);
    // ---- loci (lane g), leaf-table bases ----
    int nl1 = 0;
    int my_lo = 0, my_hi = -1;
    if (lane < Gs) {
      const int a = K.lstart[l0 + lane], b = K.lend[l0 + lane];
      const int len = max(a, b) - min(a, b) + 1;
      my_lo = min(a, b);
      my_hi = max(a, b);
      F.lo[lane] = my_lo;
      F.len[lane] = len;
      F.st[lane] = K.lstrand[l0 + lane];
      if (len < kNpyBuf) nl1 = S.lut_off[len + 1] - S.lut_off[len];
      F.nl1[lane] = (int16_t)nl1;
    }
    // loci ascending and disjoint (the usual GFF): with min_overlap > 0 a hit attaches only
    // to the loci it overlaps (a disjoint pair scores 0 < min_overlap), which are a run found
    // by binary search -- the attach loop then visits those, in GFF order, instead of every
    // locus per hit
    const int prev_hi = __shfl_up(my_hi, 1, 64);
    const bool ordered = G <= kLoc0 && P.min_overlap > 0.0 &&
                         __ballot(lane >= 1 && lane < Gs && my_lo <= prev_hi) == 0ull;
    int lut_total;
    const int lb = wave_excl_scan(nl1, &lut_total);
    F.lbase[lane] = (int16_t)min(lb, 32767);
    const int nann = Gs * nsys;
    F.abest()[lane] = 0ull;
    F.ahit()[lane] = -1;
    const bool long_locus = __ballot(lane < Gs && F.len[lane] > 65535) != 0ull;   // lohi is 16-bit
    bool staged = G > kLoc0 || lut_total > kLut0 || nann > kAnn0 || long_locus;
    wave_sync();
    // packed leaf tables, one flat batch of loads -- only once a segment needs them (a run
    // that does not cover its locus, or several runs): whole-locus runs have a closed form
    bool lut_ready = false;
    auto load_lut = [&]() {
      for (int i = lane; i < lut_total; i += 64) {
        int g = 0;                                   // last locus whose table starts at or before i
        for (int b = 32; b > 0; b >>= 1)
          if (g + b < Gs && F.lbase[g + b] <= i) g += b;
        F.lut[i] = pack_leaf(S.lut[S.lut_off[F.len[g]] + (i - F.lbase[g])]);
      }
      wave_sync();
      lut_ready = true;
    };

    WLAP(0);
    // ---- hits -> attachments, in (hit, locus) order (orgscorer.py:359-382) ----
    int n_att = 0;
    long long nl_sum = 0;
    // kHB batches of 64 hits per round: every field of all of them is loaded up front (one
    // global round trip per round instead of one per batch); the batches take their slots in
    // order, each picking its fields from the round's registers by a uniform select.  (Finding
    // every batch's loci before the first takes its slots spilled: 0.15 ms slower, r4c.)
    for (int64_t hq = h0; hq < h1; hq += 64 * kHB) {
      if (hq != h0) load_round(hq);
    for (int bq = 0; bq < kHB && hq + 64 * bq < h1; ++bq) {
      const int64_t hb = hq + 64 * bq;
      const int64_t h = hb + lane;
      int qlo = r_qlo[0], qhi = r_qhi[0], hs = r_hs[0], clade = r_cl[0];
      double scv = r_scv[0], sc = r_sc[0];
      uint32_t m = r_m[0];
      int n = 0;
      uint64_t am = 0ull;
#pragma unroll
      for (int b = 1; b < kHB; ++b)
        if (bq == b) {
          qlo = r_qlo[b]; qhi = r_qhi[b]; hs = r_hs[b]; clade = r_cl[b];
          scv = r_scv[b]; sc = r_sc[b]; m = r_m[b];
        }
      if (ordered && h < h1 && scv >= P.min_scov) {
        int g = 0;                                   // first locus ending at or after qlo
#pragma unroll
        for (int k = 32; k > 0; k >>= 1) {
          const int i = min(g + k, Gs) - 1;
          if (g + k <= Gs && F.lo[i] + F.len[i] - 1 < qlo) g += k;
        }
        for (; g < Gs; ++g) {
          const int lo = F.lo[g], len = F.len[g];
          if (lo > qhi) break;
          if (attaches(P, qlo, qhi, hs, lo, len, F.st[g])) {
            ++n;
            nl_sum += len < kNpyBuf ? F.nl1[g] : leaves_for(S, len);
            am |= 1ull << g;
          }
        }
        if (ROLL && n > 0) clade = S.anc[clade];   // parent^(jump + level), :431-445
      } else if (!ordered && h < h1 && scv >= P.min_scov) {
        for (int g = 0; g < G; ++g) {
          int lo, len, st;
          if (g < kLoc0) {
            lo = F.lo[g]; len = F.len[g]; st = F.st[g];
          } else {                                   // counted only (the contig goes staged)
            const int a = K.lstart[l0 + g], b = K.lend[l0 + g];
            lo = min(a, b); len = max(a, b) - lo + 1; st = K.lstrand[l0 + g];
          }
          if (attaches(P, qlo, qhi, hs, lo, len, st)) {
            ++n;                                     // leaves: the LDS count below 8192 sites
            nl_sum += (g < kLoc0 && len < kNpyBuf) ? F.nl1[g] : leaves_for(S, len);
            if (g < kLoc0) am |= 1ull << g;
          }
        }
        if (ROLL && n > 0) clade = S.anc[clade];   // parent^(jump + level), :431-445
      }
      int total;
      const int o = wave_excl_scan(n, &total);
      if (!staged && n > 0 && n_att + o + n <= CAP) {
        if (!ROLL)
          for (int j = 0; j < P.jump; ++j) clade = K.parent[clade];   // orgscorer.py:955-957
        const bool ann = m != 0 && sc >= P.annot_ref;
        int slot = n_att + o;
        for (uint64_t bits = am; bits; bits &= bits - 1, ++slot) {
          const int g = __builtin_ctzll(bits);
          const int len = F.len[g];
          const int h1s = max(0, qlo - F.lo[g]);
          const int h2s = min(len - 1, qhi - F.lo[g]);
          const int start = min(h1s, len);
          int stop = h2s + 1;                        // site[h1:h2+1], python slice rules
          if (stop < 0) { stop += len; if (stop < 0) stop = 0; }
          F.key[slot] = ((uint32_t)clade << kCladeShift) | ((uint32_t)g << kSlotBits) | (uint32_t)slot;
          F.lohi[slot] = (uint32_t)start | ((uint32_t)stop << 16);
          F.sc[slot] = sc;
          F.hit()[slot] = (int)h;
          F.sm()[slot] = (int)m;
          if (ann)                                   // annotation pass 1: best score bits (:383-392)
            for (int b = 0; b < nsys; ++b)
              if ((m >> b) & 1u) atomicMax(&F.abest()[g * nsys + b], dbits(sc));
        }
      }
      n_att += total;
    }
    }
    nl_sum = wave_sum_dpp(nl_sum);
    staged = staged || n_att > CAP;
    wave_sync();
    WLAP(1);
    WSTAT(16, 1);
    WSTAT(17, n_att);
    WSTAT(23, h1 - h0);
    if (!staged && G > 0 && ann_on) {
      // annotation pass 2: the last hit (largest index) at the best score per (locus, system)
      for (int t = lane; t < n_att; t += 64) {
        const uint32_t m = (uint32_t)F.sm()[t];
        const double sc = F.sc[t];
        if (m == 0 || !(sc >= P.annot_ref)) continue;
        const int g = (int)((F.key[t] >> kSlotBits) & (kLoc0 - 1));
        const int h = F.hit()[t];
        for (int b = 0; b < nsys; ++b)
          if (((m >> b) & 1u) && F.abest()[g * nsys + b] == dbits(sc)) atomicMax(&F.ahit()[g * nsys + b], h);
      }
      wave_sync();
      if (lane < nann) K.annot[l0 * nsys + lane] = F.ahit()[lane];
    }
    WLAP(2);
    // ---- levels: sort, segments, means, explain_one [, explain_two, roll-up] ----
    int64_t pair_evals = (ROLL && lane == 0) ? K.pair_evals[c] : 0;
    pair_evals = lane_bcast((uint64_t)pair_evals, 0);
    bool seed = false;                                 // raised at level 0: staged level 1 seed
    bool dumped = false;                               // segment table handed to k_dump_sparse
    // level 0: keys sorted alone, attachments reached through the keys' slot fields (its few
    // multi-attachment segments do not repay moving the data: r4w, 9.19 / 9.25 ms against
    // 9.25 / 9.26 moved); the roll-up launches move ranges and scores with the keys.  (Keeping
    // the roll-up attachments in descending-score order for early exits saved what its extra
    // sort cost, r4j, and was removed.)
    constexpr bool kKeyOrder = !FULL && !ROLL;
    using Src = typename std::conditional<kKeyOrder, SliceSrcKey, SliceSrc>::type;
    auto slot_at = [&](int t) -> int { return kKeyOrder ? (int)(F.key[t] & kSlotMask) : t; };
    for (int level = start_level; !staged && G > 0 && h1 > h0; ++level) {   // else: never evaluated (:959)
      const int iteration = level + 1;
      if (level > start_level) {                     // roll up (:431-445): re-key to the parent clade
        for (int t = lane; t < n_att; t += 64) {
          const uint32_t k0 = F.key[t];
          const int parent = K.parent[(int)(k0 >> kCladeShift)];
          F.key[t] = ((uint32_t)parent << kCladeShift) | (k0 & ((1u << kCladeShift) - 1));
        }
        wave_sync();
      }
      sort_slice<(CAP + 63) / 64, !kKeyOrder>(F, n_att);   // one network: code size
      WLAP(3);
      // ---- segments = runs of equal (clade, locus) ----
      int ns = 0;
      for (int t0 = 0; t0 < n_att; t0 += 64) {
        const int t = t0 + lane;
        const bool head = t < n_att && (t == 0 || (F.key[t] >> kSlotBits) != (F.key[t - 1] >> kSlotBits));
        const uint64_t hm = __ballot(head);
        if (head) F.seg[ns + __popcll(hm & lanes_below())] = (F.key[t] & ~kSlotMask) | (uint32_t)t;
        ns += __popcll(hm);
      }
      if (lane == 0) F.seg[ns] = (uint32_t)n_att;    // end of the last segment (n_att <= CAP)
      wave_sync();
      WLAP(4);
      WSTAT(18, ns);
      // ---- segment means (numpy pairwise order, exact), evaluated pass by pass ----
      // Only what the decision can use is evaluated (exact for k1 > 0):
      //  - explain_one: an option has crit >= k1 > 0, so a segment on every unmasked locus;
      //    the weak-locus mask needs, per locus, one known clade's mean >= kmin, or proof that
      //    none reaches it -- a segment's mean is at most its best attachment score (times
      //    1 + 2e-15 for the rounded sum), so segments scoring below kmin * (1 - 1e-12) are
      //    never evaluated;
      //  - explain_two (FULL, k2 > 0 and a positive sister threshold): a potential clade has
      //    a mean >= k2 (bound as above); its whole row is evaluated; the sister checks read
      //    clades whose listed parent is the parent of a potential clade, at scores >= the
      //    sister threshold (bound as above).
      // Passes: 0 clades on every locus, 1 the best-scoring segment of each open locus, 7 the
      // other segments that may settle a locus still open, 2 clades on every unmasked locus,
      // 3 every segment (not pruned), 4 potential-clade candidates, 5 potential rows + sister
      // candidates, 6 every segment not yet evaluated.
      double* v = F.v();
      bool fail = false;
      const bool prune = P.k1 > 0.0;
      const bool prune2 = FULL && prune && P.k2 > 0.0 && (!P.sister_on || P.sister_thr > 0.0);
      // first form, hand-over to k_dump_sparse after explain_one found no option: only what
      // its explain_two can read is evaluated (passes 4 and 5 as in the FULL form); the rest
      // goes over as 0.0.  Exact because (a) the unmasked-locus set it rebuilds is this one
      // (every locus in it holds an evaluated known-clade mean >= kmin, every other locus has
      // none), (b) with no option here, zeros create none there, (c) a clade none of whose
      // segments can reach k2 is no potential clade either way, and potential clades' rows
      // are evaluated whole, (d) the sister counts read only clades listed under a potential
      // clade's parent, at scores >= the threshold (bound as in pass 5).  More than 64
      // potential clades (the parent list's size) evaluate everything (pass 6).
      const bool prune2d = !FULL && prune && P.k2 > 0.0 && (!P.sister_on || P.sister_thr > 0.0) && P.weak != 2;
      const uint64_t allG = G >= 64 ? ~0ull : ((1ull << G) - 1ull);
      uint64_t um = 0;
      uint8_t* rc = F.rc();                            // per segment: its clade run's size / flag
      int* pp = reinterpret_cast<int*>(F.mx());        // parents of the potential clades (FULL)
      int npp = 0;
      // segments of the clade run starting at t that lie on loci of `mask`
      auto run_count = [&](int t, uint64_t mask) -> int {
        const int clade = cg_of(F, t).x;
        int cnt = 0;
        for (int q = t; q < ns; ++q) {
          const int2 cq = cg_of(F, q);
          if (cq.x != clade) break;
          cnt += (int)((mask >> cq.y) & 1ull);
        }
        return cnt;
      };
      // per-locus bits of evaluated known-clade segments with mean >= kmin
      auto sure_bits = [&]() -> uint64_t {
        uint64_t b = 0;
        for (int t = lane; t < ns; t += 64) {
          const int2 cg = cg_of(F, t);
          if (cg.x != K.unknown && v[t] >= 0.0 && v[t] >= P.kmin) b |= 1ull << cg.y;
        }
        b = wave_or_dpp(b);
        return b;
      };
      // Upper bound of segment t's mean, computed once per segment in the prune setup and
      // kept in the not-evaluated marker, v[t] = -1 - ub (any v < 0 is "not evaluated";
      // -1 - (-1 - ub) may lose ub's bits below 2^-52, far inside the bounds' 1e-12 slack).
      // The best attachment score bounds any envelope's mean; a one-attachment segment's
      // mean is its score times its run's share of the locus up to numpy's rounding (a
      // pairwise sum of <= 8191 equal terms: relative error < 1e-14), so score x share x
      // (1 + 2e-12) bounds it too and rules out the partial decoy hits the explain_two
      // passes (4, 5) would otherwise evaluate.  (With the triage, the first form's level-0
      // contigs are the explain_two ones: every one of them asks.)
      auto scan_best = [&](int t) -> double {
        const int kb = seg_first(F, t), ke = t + 1 < ns ? seg_first(F, t + 1) : n_att;
        double ub = 0.0;
        if (ke - kb == 1) {
          const int slot = slot_at(kb);
          const uint32_t x = F.lohi[slot];
          const double sc = F.sc[slot];
          const int len = F.len[cg_of(F, t).y];
          const int run = max(0, hi16(x) - lo16(x));
          return fmin(sc, sc * ((double)run / (double)len) * (1.0 + 2e-12));
        }
        for (int q = kb; q < ke; ++q) ub = fmax(ub, F.sc[slot_at(q)]);
        return ub;
      };
      auto best_score = [&](int t) -> double {       // (callers: v[t] < 0)
        return FULL ? scan_best(t) : -1.0 - v[t];
      };
      // Hand-over (lower bounds): a pass-4 candidate whose mean is surely >= every threshold the
      // table's non-member readers compare it with (k2, the sister threshold, kmin) -- some
      // attachment's run alone gives the envelope a mean >= score x share, numpy's rounding
      // inside the 2e-12 slack -- is not evaluated in pass 4 (rc bit 0x80); its clade's mask
      // and potential flag count it, a member's row evaluates it in pass 5, and otherwise the
      // table carries lb_thr in its place (the same answer to every such comparison).
      const double lb_thr = fmax(fmax(P.k2, P.sister_on ? P.sister_thr : 0.0), P.kmin);
      auto lb_mean = [&](int t) -> double {
        const int kb = seg_first(F, t), ke = t + 1 < ns ? seg_first(F, t + 1) : n_att;
        const double len = (double)F.len[cg_of(F, t).y];
        double lb = 0.0;
        for (int q = kb; q < ke; ++q) {
          const int slot = slot_at(q);
          const uint32_t x = F.lohi[slot];
          const int run = max(0, hi16(x) - lo16(x));
          lb = fmax(lb, F.sc[slot] * ((double)run / len) * (1.0 - 2e-12));
        }
        return lb;
      };
      auto lb_sure = [&](int t) -> bool { return lb_mean(t) >= lb_thr; };
      // Unmasked loci settled by lower bounds: a known clade's segment whose bound
      // reaches kmin unmasks its locus (:420-427) without its mean.  Only where the contig's
      // hand-over is sure to be the compact table (whose explain_two takes um from the header;
      // a whole table would rebuild um from the values it holds) or everything gets evaluated
      // (pass 6), and explain_one reads only the means of the clades it ranks.
      const bool lb_um = !FULL && prune2d && S.wave_two && S.dump_cap > 0 && G <= kE2MaxG &&
                         ns <= kE2Seg && P.weak == 0 && P.kmin > 0.0;
      auto lb_um_bits = [&](uint64_t open_) -> uint64_t {
        uint64_t b = 0;
        for (int t = lane; t < ns; t += 64) {
          const int2 cg = cg_of(F, t);
          if (cg.x != K.unknown && ((open_ >> cg.y) & 1ull) && v[t] < 0.0 && -1.0 - v[t] >= P.kmin &&
              lb_mean(t) >= P.kmin * (1.0 + 1e-12))
            b |= 1ull << cg.y;
        }
        return wave_or_dpp(b);
      };
      int n_pass0 = -1;                                // pass 0's list, built with the run sizes
      if (prune) {
        // every segment's clade-run size, from the run heads' ballot masks: a lane's run
        // starts at the last head at or before it and ends at the next head after it
        constexpr int kCh = (CAP + 63) / 64;
        uint64_t hd[kCh];
#pragma unroll
        for (int i = 0; i < kCh; ++i) {
          const int t = 64 * i + lane;
          hd[i] = __ballot(t < ns && (t == 0 || (F.seg[t - 1] >> kCladeShift) != (F.seg[t] >> kCladeShift)));
        }
        const uint64_t le = lane == 63 ? ~0ull : (2ull << lane) - 1ull;   // lanes <= this one
        int rs[kCh];
        int carry = 0;
#pragma unroll
        for (int i = 0; i < kCh; ++i) {                // run starts, chunk by chunk
          const uint64_t m = hd[i] & le;
          rs[i] = m ? 64 * i + 63 - __clzll(m) : carry;
          carry = hd[i] ? 64 * i + 63 - __clzll(hd[i]) : carry;
        }
        carry = ns;
        int rsz[kCh];
#pragma unroll
        for (int i = kCh - 1; i >= 0; --i) {           // run ends, backwards
          const int t = 64 * i + lane;
          const uint64_t m = hd[i] & ~le;
          const int re = m ? 64 * i + __ffsll((unsigned long long)m) - 1 : carry;
          carry = hd[i] ? 64 * i + __ffsll((unsigned long long)hd[i]) - 1 : carry;
          rsz[i] = re - rs[i];
          if (t < ns) {
            v[t] = FULL ? -1.0 : -1.0 - scan_best(t);  // not evaluated (first form: its bound)
            rc[t] = (uint8_t)rsz[i];
          }
        }
        // pass 0's list (segments of clades on every locus), in segment order
        uint16_t* lst = F.list();
        n_pass0 = 0;
#pragma unroll
        for (int i = 0; i < kCh; ++i) {
          const int t = 64 * i + lane;
          const bool in = t < ns && rsz[i] == G;
          const uint64_t im = __ballot(in);
          if (in) lst[n_pass0 + __popcll(im & lanes_below())] = (uint16_t)t;
          n_pass0 += __popcll(im);
        }
        wave_sync();
      }
      const double bound = P.kmin * (1.0 - 1e-12), bound2 = P.k2 * (1.0 - 1e-12);
      const double bound_s = P.sister_thr * (1.0 - 1e-12);
      uint64_t open = 0;
      int outcome = 0;                                 // 2: decided (or stopped) by explain_one
      bool compact_ok = false;                         // passes 4, 5 ran: explain_two's inputs only
      // first form: the level's decision goes to k_dump_sparse with the whole segment table
      // (pass 6 evaluates the rest) instead of the staged kernels
      bool dump = false;
      const bool can_dump = !FULL && S.dump_cap > 0;
      WLAP(5);
      for (int pass = prune ? 0 : 3;;) {
        WLAP(8);
        WSTAT(19, 1);
        WSTAT(24 + pass, 1);
        int n = ns;
        const uint16_t* list = nullptr;
        if (pass == 1) {                               // per open locus: its best attachment score
          F.mx()[lane] = 0ull;
          wave_sync();
          for (int t = lane; t < ns; t += 64) {
            const int2 cg = cg_of(F, t);
            if (v[t] < 0.0 && cg.x != K.unknown && ((open >> cg.y) & 1ull))
              atomicMax(&F.mx()[cg.y], dbits(best_score(t)));
          }
          wave_sync();
        }
        if (pass == 0 && n_pass0 >= 0) {
          n = n_pass0;
          list = F.list();
        } else if (pass != 3) {                        // compact this pass's segments
          uint16_t* lst = F.list();
          const int gu = __popcll(um);
          n = 0;
          for (int t0 = 0; t0 < ns; t0 += 64) {
            const int t = t0 + lane;
            bool in = false;
            if (t < ns) {
              const int2 cg = cg_of(F, t);
              if (pass == 0) {
                in = (int)rc[t] == G;
              } else if (pass == 1 || pass == 7) {
                in = v[t] < 0.0 && cg.x != K.unknown && ((open >> cg.y) & 1ull) && best_score(t) >= bound;
                if (pass == 1 && in) {                 // first only the best-scoring one per locus
                  const double ub = best_score(t);
                  in = false;
                  const unsigned long long want = ((unsigned long long)dbits(ub) << 0);
                  in = F.mx()[cg.y] == want;
                }
              } else if (pass == 2) {
                in = v[t] < 0.0 && ((um >> cg.y) & 1ull) && (int)rc[t] == gu;
              } else if (pass == 4) {
                in = v[t] < 0.0 && best_score(t) >= bound2;
                if (!FULL && in && lb_sure(t)) {
                  in = false;
                  rc[t] |= 0x80;                       // (run sizes < 0x80: pass 4's post replaces them)
                }
              } else if (pass == 5) {
                if (v[t] < 0.0) {
                  in = (rc[t] & 3) == 1;               // a (member) potential clade's row
                  if (!in && P.sister_on && best_score(t) >= bound_s) {
                    const int sp = K.sibp[cg.x];
                    for (int i = 0; i < npp && !in; ++i) in = pp[i] == sp;
                  }
                }
              } else {
                in = v[t] < 0.0;
              }
            }
            const uint64_t im = __ballot(in);
            if (in) lst[n + __popcll(im & lanes_below())] = (uint16_t)t;
            n += __popcll(im);
          }
          wave_sync();
          list = lst;
        }
        WLAP(6);
        WSTAT(20, n);
        WSTAT(40 + pass, n);                          // (segments listed per pass)
        for (int s0 = 0; s0 < n; s0 += 64) {
          const int s = s0 + lane < n ? (list ? (int)list[s0 + lane] : s0 + lane) : ns;
          bool multi = false, big = false;               // big: too many attachments for the wave path
          int g = 0, len = 0, nl = 0;
          bool one_run = false;                          // one envelope run [lo, hi) of value vv
          int lo = 0, hi = 0;
          double vv = 0.0;
          if (s < ns) {
            const int kb = seg_first(F, s), ke = s + 1 < ns ? seg_first(F, s + 1) : n_att, na = ke - kb;
            g = cg_of(F, s).y;
            len = F.len[g];
            nl = F.nl1[g];
            const bool thread_ok = len < kNpyBuf && nl <= kThreadLeaves;
            if (na == 1) {
              if (thread_ok) {
                const int slot = slot_at(kb);
                lo = lo16(F.lohi[slot]); hi = hi16(F.lohi[slot]); vv = F.sc[slot];
                one_run = true;
              }
            } else if (na <= kPruneMax) {
              double Fw = 0.0;                           // best whole-locus attachment
              for (int t = kb; t < ke; ++t) {
                const int slot = slot_at(t);
                const uint32_t x = F.lohi[slot];
                const double sc = F.sc[slot];
                if (lo16(x) <= 0 && hi16(x) >= len && sc > Fw) Fw = sc;
              }
              int kept = 0;                              // attachments the envelope still needs
              for (int t = kb; t < ke; ++t) {
                const int slot = slot_at(t);
                const uint32_t x = F.lohi[slot];
                kept += (lo16(x) < hi16(x) && F.sc[slot] > Fw) ? 1 : 0;
              }
              if (kept == 0 && thread_ok) { lo = 0; hi = len; vv = Fw; one_run = true; }
            }
            if (one_run) {
            } else if ((FULL || ROLL || na <= kMultiAttL0) && nl <= 64 && len < kNpyBuf) {
              multi = true;
              big = na > (FULL ? kMultiAtt0 : kMultiAttL0);   // (beyond the envelope buffer)
            }
            else
              fail = true;                               // the staged leaf kernels take it
          }
          if (!lut_ready && __ballot(multi) != 0ull) load_lut();   // (one runs: closed forms)
          WLAP(15);
          if (one_run) v[s] = one_run_mean(PackedLut{F.lut + F.lbase[g]}, nl, len, lo, hi, vv);
          WLAP(pass == 0 ? 7 : (pass == 6 ? 11 : 14));
          uint64_t mlist = __ballot(multi);
          constexpr bool kFlat = ROLL;                   // (its only multi path: the others compile out)
          if constexpr (kFlat) {
            // roll-up levels, where a segment gathers the attachments of many clades: one
            // numpy leaf per lane over all of the chunk's multi-attachment segments
            if (mlist != 0ull) {
              int kb = 0, ke = 0;
              if (multi) { kb = seg_first(F, s); ke = s + 1 < ns ? seg_first(F, s + 1) : n_att; }
              const double m = flat_leaf_means(Src{F.key, F.lohi, F.sc}, F.lut + F.lbase[multi ? g : 0], mlist,
                                               kb, ke, nl, len, F.runs());
              if (multi) v[s] = m;
            }
            mlist = 0;
          } else if ((FULL || ROLL) && (__popcll(mlist) >= 3 || __ballot(big) != 0ull)) {
            // several multi-attachment segments: one lane each, not the whole wave per segment
            if (multi) {
              const int kb = seg_first(F, s), ke = s + 1 < ns ? seg_first(F, s + 1) : n_att;
              v[s] = lane_seg_mean(Src{F.key, F.lohi, F.sc}, kb, ke, PackedLut{F.lut + F.lbase[g]}, nl, len);
            }
            mlist = 0;
          }
          if constexpr (!kFlat)
          for (uint64_t mm = mlist; mm; mm &= mm - 1) {  // the wave, one segment each
            const int src = __builtin_ctzll(mm);
            const int s2 = lane_bcast(s, src);
            const int kb = seg_first(F, s2), na = (s2 + 1 < ns ? seg_first(F, s2 + 1) : n_att) - kb;
            const int g2 = lane_bcast(g, src), len2 = lane_bcast(len, src), nl2 = lane_bcast(nl, src);
            int lo = 0, hi = 0;
            double sc = 0.0;
            if (lane < na) {
              const int slot = slot_at(kb + lane);
              const uint32_t x = F.lohi[slot];
              if (lo16(x) < hi16(x)) { lo = lo16(x); hi = hi16(x); sc = F.sc[slot]; }
            }
            const double mean = wave_seg_mean(PackedLut{F.lut + F.lbase[g2]}, nl2, len2, lo, hi, sc, F.runs());
            if (lane == 0) v[s2] = mean;
          }
          WLAP(pass == 0 ? 12 : 13);
        }
        wave_sync();
        WLAP(7);
        // after the pass: the weak-locus mask, explain_one, the next pass
        bool e1_now = false;
        if (pass == 0) {
          if (P.weak != 0 || P.kmin <= 0.0) {
            um = allG;                                 // penalize: no mask; kmin <= 0: nothing masked
            e1_now = true;                             // (every locus unmasked: pass 0 had the options)
          } else {
            um = sure_bits();
            open = allG & ~um;                         // loci no full clade settles
            if (open && lb_um) {
              um |= lb_um_bits(open);
              open = allG & ~um;
            }
            if (open) { pass = 1; continue; }
            e1_now = true;
          }
        } else if (pass == 1 || pass == 7) {
          um |= sure_bits();
          if (pass == 1 && (open & ~um)) {             // loci the best segments did not settle
            open &= ~um;
            pass = 7;
            continue;
          }
          if (um != allG && um != 0ull) {
            for (int t = lane; t < ns; t += 64)        // clade runs' sizes on the unmasked loci
              if (t == 0 || cg_of(F, t - 1).x != cg_of(F, t).x) {
                const int cnt = run_count(t, ~0ull), cu = run_count(t, um);
                for (int q = t; q < t + cnt; ++q) rc[q] = (uint8_t)cu;
              }
            wave_sync();
            pass = 2;
            continue;
          }
          e1_now = true;
        } else if (pass == 2) {
          e1_now = true;
        } else if (pass == 3) {
          // weak loci from every mean: ignore -> mask (:420-427), penalize -> none (:413-414)
          F.mx()[lane] = 0ull;
          wave_sync();
          for (int t = lane; t < ns; t += 64) {        // per-locus max over known clades
            const int2 cg = cg_of(F, t);
            const double x = v[t];
            if (cg.x != K.unknown && x > 0.0) atomicMax(&F.mx()[cg.y], dbits(x));
          }
          wave_sync();
          const double mxl = __longlong_as_double((long long)F.mx()[lane]);
          um = __ballot(lane < G && (P.weak != 0 || mxl >= P.kmin));
          e1_now = true;
        } else if (pass == 4) {                        // potential clades: a mean >= k2 (:603-605)
          // One walk per clade run: its size, whether it is potential, and (hand-over) its
          // loci >= k2 on the unmasked set.  Hand-over: only potential clades that form a
          // candidate pair (crit >= k2 <=> (m_i | m_j) == um: exact here, every segment that
          // can reach k2 was evaluated by pass 4) have their rows read by explain_two's ranks
          // and LGT checks; the others (rc 2) keep what pass 4 evaluated -- enough to find them
          // potential and to build their masks -- and count as sisters through pass 5's sister
          // candidates like any other clade.  Lane i: potential clade i's run (<= 64 of them,
          // else pass 6 below).
          const bool members = !FULL;
          int ph = -1, pcnt = 0, np0 = 0;
          uint64_t pm = 0;
          for (int t0 = 0; t0 < ns; t0 += 64) {
            const int t = t0 + lane;
            const bool head = t < ns && (t == 0 || cg_of(F, t - 1).x != cg_of(F, t).x);
            bool pot = false;
            uint64_t m = 0;
            int cnt = 0;
            if (head) {
              const int clade = cg_of(F, t).x;
              for (int q = t; q < ns; ++q) {
                const int2 cq = cg_of(F, q);
                if (cq.x != clade) break;
                ++cnt;
                if (v[q] >= P.k2 || (rc[q] & 0x80)) { pot = true; m |= 1ull << cq.y; }
              }
              for (int q = t; q < t + cnt; ++q) rc[q] = (uint8_t)((rc[q] & 0x80) | (pot ? 1 : 0));
            }
            m &= um;
            const uint64_t im = __ballot(head && pot);
            if (members)
              for (uint64_t r = im; r; r &= r - 1) {     // potential clade np0 + k -> lane np0 + k
                const int src = __builtin_ctzll(r);
                const int dst = np0 + __popcll(im & ((1ull << src) - 1ull));
                const int hs = lane_bcast(t, src), hc = lane_bcast(cnt, src);
                const uint64_t ms = lane_bcast(m, src);
                if (lane == dst) { ph = hs; pcnt = hc; pm = ms; }
              }
            np0 += __popcll(im);
          }
          wave_sync();
          if (members && np0 <= 64) {
            bool member = false;
            for (int j = 0; j < np0; ++j) {
              const uint64_t mj = lane_bcast(pm, j);
              member = member || (lane != j && (pm | mj) == um);
            }
            if (lane < np0 && !member)
              for (int q = ph; q < ph + pcnt; ++q) rc[q] = (uint8_t)((rc[q] & 0x80) | 2);
            wave_sync();
          }
          npp = 0;                                     // their parents (sister checks, :717-744)
          int npot = 0;
          for (int t0 = 0; t0 < ns; t0 += 64) {
            const int t = t0 + lane;
            const bool in = t < ns && (rc[t] & 3) && (t == 0 || cg_of(F, t - 1).x != cg_of(F, t).x);
            const uint64_t im = __ballot(in);
            const bool mem_in = in && (rc[t] & 3) == 1;  // (the parents of candidate-pair members)
            const uint64_t mm = __ballot(mem_in);
            // the sisters of X are the clades listed under parent(X) (get_sisters, utils.py:428-434):
            // pass 5 evaluates clades whose listed parent is one of these.  (Not sibp(X): an
            // unlisted X has sibp -1 but parent r__Root, whose listed children are its sisters.)
            if (mem_in && npp + __popcll(mm & lanes_below()) < 64)
              pp[npp + __popcll(mm & lanes_below())] = K.parent[cg_of(F, t).x];
            npp = min(npp + __popcll(mm), 64);
            npot += __popcll(im);
          }
          wave_sync();
          pass = (!FULL && npot > 64) ? 6 : 5;         // (hand-over: the parent list overflowed)
          compact_ok = pass == 5;
          continue;
        } else {
          break;                                       // passes 5 / 6: explain_two's inputs
        }
        if (!e1_now) break;
        WLAP(32);                                      // (stamps: sure bits, pass choice)
        if (__ballot(fail) != 0ull) { staged = __ballot(fail) != 0ull; outcome = 2; break; }
        // ---- explain_one (k_one's arithmetic, orgscorer.py:407-429, 447-461, 585-597) ----
        const int Gu = __popcll(um);
        if (Gu == 0) {                                 // level 0: skipped contig (:959)
          if (level > 0 && lane == 0) {                // later: np.min of an empty array upstream
            K.iters[c] = (int16_t)min(iteration, 32767);
            K.pair_evals[c] = pair_evals;
            K.status[c] = WF_E_EMPTYMASK;
          }
          outcome = 2;
          break;
        }
          double br = -__builtin_inf(), bcrit = 0.0;
          long long bk = -1;
          double* rank = F.rank();
          // the rank of the option whose clade run starts at t, or -1 (crit: its crit)
          auto option_rank = [&](int t, double& crit) -> double {
            const int clade = cg_of(F, t).x;
            // (assign-unknown: a real "Unknown" run is replaced by the virtual row, below)
            if ((t == 0 || cg_of(F, t - 1).x != clade) && (!prune || (int)rc[t] == Gu) &&
                !(P.weak == 2 && clade == K.unknown)) {
              double rnk;                                  // (pruned: only runs on every unmasked locus)
              sparse_score(F, v, t, ns, clade, um, Gu, crit, rnk);
              if (crit >= P.k1) return rnk;
            }
            return -1.0;
          };
          // Option ranks for meld_one.  FULL: by segment (-1: none).  The first form's rank
          // array would be the attachment scores' (sc), which a hand-over to k_dump_sparse
          // still needs (pass 6): its options are compacted instead, ranks into the mx
          // region and clades into the mem region (meld_one compacts them in place), or --
          // past 64 options -- recomputed there
          double* opt_r = reinterpret_cast<double*>(F.mx());
          int* opt_c = F.mem();
          int nopt = 0;
          if (!FULL && prune) {
            // the candidates (run heads whose run counts Gu segments on the unmasked loci, in
            // segment order), each scored by the whole wave: the best option stays uniform
            for (int t0 = 0; t0 < ns; t0 += 64) {
              const int t = t0 + lane;
              bool cand = false;
              if (t < ns) {
                const int clade = (int)(F.seg[t] >> kCladeShift);
                cand = (t == 0 || (int)(F.seg[t - 1] >> kCladeShift) != clade) && (int)rc[t] == Gu &&
                       !(P.weak == 2 && clade == K.unknown);
              }
              for (uint64_t cm = __ballot(cand); cm; cm &= cm - 1) {
                const int tt = t0 + __builtin_ctzll(cm);
                double crit, rk;
                const int clade = wave_run_score(F, v, tt, ns, um, Gu, P.k1, crit, rk);
                if (crit >= P.k1) {
                  if (better(rk, clade, br, bk)) { br = rk; bk = clade; bcrit = crit; }
                  if (nopt < 64 && lane == 0) { opt_r[nopt] = rk; opt_c[nopt] = clade; }
                  ++nopt;
                }
              }
            }
            WLAP(33);                                    // (stamps: option scan)
          } else {
          for (int t0 = 0; t0 < ns; t0 += 64) {
            const int t = t0 + lane;
            double crit = 0.0;
            const double rk = t < ns ? option_rank(t, crit) : -1.0;
            const int clade = t < ns ? cg_of(F, t).x : 0;
            if (rk >= 0.0 && better(rk, clade, br, bk)) { br = rk; bk = clade; bcrit = crit; }
            if (FULL) {
              if (t < ns) rank[t] = rk;
            } else {
              const uint64_t im = __ballot(rk >= 0.0);
              const int pos = nopt + __popcll(im & lanes_below());
              if (rk >= 0.0 && pos < 64) { opt_r[pos] = rk; opt_c[pos] = clade; }
              nopt += __popcll(im);
            }
          }
          WLAP(33);                                      // (stamps: option scan)
          each_stride([&](auto J) {
            const double r2 = xor_lanes<decltype(J)::value>(br), c2 = xor_lanes<decltype(J)::value>(bcrit);
            const long long k2 = xor_lanes<decltype(J)::value>(bk);
            if (better(r2, k2, br, bk)) { br = r2; bk = k2; bcrit = c2; }
          });
          }
          if (P.weak == 2) {
            // assign-unknown (:416-418): the row "Unknown" = 1 - maxes is no option iff some
            // locus has 1 - max < k1; a known clade's evaluated mean bounds that locus's max
            // from below (1 - x is monotone), so one such locus settles it.  Otherwise -- or
            // without a known option -- the staged kernels decide with the row.
            bool settles = false;
            for (int t = lane; t < ns; t += 64) {
              const int2 cg = cg_of(F, t);
              if (cg.x != K.unknown && v[t] >= 0.0 && (1.0 - v[t]) < P.k1) settles = true;
            }
            if (bk < 0 || __ballot(settles) == 0ull) {
              if (can_dump) {
                dump = true;
                if (pass == 3) break;
                pass = 6;
                continue;
              }
              staged = true;
              outcome = 2;
              break;
            }
          }
          WLAP(34);                                      // (stamps: reduction)
          if (bk >= 0) {
            wave_sync();
            int nm = 0;                                    // meld_one (:621-631): options within --range
            if (!FULL && P.dis1 == 1 && nopt <= 64) {      // (options in segment order)
              const bool in = lane < nopt && (br - opt_r[lane]) <= P.range;
              const int clade = in ? opt_c[lane] : 0;      // read by every lane before the writes
              const uint64_t im = __ballot(in);
              if (in) F.mem()[__popcll(im & lanes_below())] = clade;
              nm = __popcll(im);
            } else if (P.dis1 == 1)
              for (int t0 = 0; t0 < ns; t0 += 64) {
                const int t = t0 + lane;
                double crit_unused;
                const double rk = t < ns ? (FULL ? rank[t] : option_rank(t, crit_unused)) : -1.0;
                const bool in = rk >= 0.0 && (br - rk) <= P.range;
                const uint64_t im = __ballot(in);
                if (in) F.mem()[nm + __popcll(im & lanes_below())] = cg_of(F, t).x;
                nm += __popcll(im);
              }
            wave_sync();
            if (P.dis1 == 1 && nm == 0) {                  // negative --range upstream crash
              if (lane == 0) K.status[c] = WF_E_BADINPUT;
              outcome = 2;
              break;
            }
            int lca = (int)bk;
            if (P.dis1 == 1) {
              int acc = -1;
              for (int i = lane; i < nm; i += 64) acc = lca2(K, acc, F.mem()[i]);
              lca = wave_lca(K, acc);
            }
            WLAP(35);                                      // (stamps: meld_one + LCA)
            const int64_t mbase = 2 * h0 + 2 * (int64_t)c;
            for (int i = lane; i < nm; i += 64) K.meld[mbase + i] = F.mem()[i];
            if (lane < G) K.syn[l0 + lane] = ((um >> lane) & 1ull) ? 'A' : '~';   // set_synteny_one
            if (lane == 0) {
              K.call[c] = WF_CALL_NO_LGT;
              K.crit[c] = bcrit;
              K.rank[c] = br;
              K.c1[c] = lca;
              K.c2[c] = -1;
              K.nm1[c] = nm;
              K.iters[c] = (int16_t)iteration;
              K.pair_evals[c] = pair_evals;
            }
            outcome = 2;
            break;
          }
        if (!FULL) {                                   // explain_two (:570): the next kernel
          if (can_dump) {
            dump = true;
            if (pass == 3) break;
            pass = prune2d ? 4 : 6;
            continue;
          }
          staged = true;
          outcome = 2;
          break;
        }
        if (pass == 3) break;                          // every mean is there already
        pass = prune2 ? 4 : 6;
      }
      staged = staged || __ballot(fail) != 0ull;
      wave_sync();
      WLAP(8);
      if (dump && !staged) {
        // The compact form (WF_OPT_WAVE_TWO; passes 4 and 5 ran, <= 64 potential clades):
        // only what explain_two reads -- the potential clades' rows (rc) and the segments at
        // or above the sister threshold -- plus the unmasked loci and whether r__Root is
        // present; k_dump_sparse decides from it (sp_two).  Else the whole table (sp_level).
        bool compact = !FULL && compact_ok && S.wave_two && G <= kE2MaxG && P.weak != 2;
        int n_out = ns;
        bool rootp = false;
        // (rc 2: a potential clade in no candidate pair -- its evaluated segments only)
        auto want = [&](int t) {
          const int k = rc[t] & 3;
          return k == 1 || (k == 2 && (v[t] >= 0.0 || (rc[t] & 0x80))) || (P.sister_on && v[t] >= P.sister_thr);
        };
        // (not evaluated: lb_thr for a pass-4 segment known >= it, else 0.0 -- see prune2d)
        auto out_v = [&](int t) { return v[t] >= 0.0 ? v[t] : ((rc[t] & 0x80) ? lb_thr : 0.0); };
        if (compact) {
          int n2 = 0;
          for (int t0 = 0; t0 < ns; t0 += 64) {
            const int t = t0 + lane;
            bool w = false;
            if (t < ns) {
              w = want(t);
              rootp = rootp || cg_of(F, t).x == K.root;
            }
            n2 += __popcll(__ballot(w));
          }
          rootp = __ballot(rootp) != 0ull;
          compact = n2 <= kE2Seg;
          if (compact) n_out = n2;
        }
        // the table: one 64-bit atomic gives the slot (high bits) and its first entry (low
        // 40), so slot k's entries start where slot k - 1's end
        unsigned long long old = 0;
        if (lane == 0) old = atomicAdd(S.dump_ctr, (1ull << 40) | (unsigned long long)n_out);
        old = lane_bcast((uint64_t)old, 0);
        const int slot = (int)(old >> 40);
        const int64_t base = (int64_t)(old & ((1ull << 40) - 1));
        dumped = base + n_out <= S.dump_cap;         // else: the staged kernels (pend 1)
        if (dumped && compact) {
          int o = 0;
          for (int t0 = 0; t0 < ns; t0 += 64) {
            const int t = t0 + lane;
            const bool w = t < ns && want(t);
            const uint64_t wm = __ballot(w);
            if (w) {
              const int q = o + __popcll(wm & lanes_below());
              S.dump_cg[base + q] = cg_of(F, t);
              S.dump_mean[base + q] = out_v(t);      // (member rows are whole)
            }
            o += __popcll(wm);
          }
        } else if (dumped) {
          for (int t = lane; t < ns; t += 64) {
            S.dump_cg[base + t] = cg_of(F, t);
            S.dump_mean[base + t] = out_v(t);
          }
        }
        if (lane == 0) {
          S.dump_first[slot] = (int)(base < INT32_MAX ? base : INT32_MAX);
          S.dump_first[slot + 1] = (int)(base + n_out < INT32_MAX ? base + n_out : INT32_MAX);
          S.dump_list[2 * slot] = compact ? 1 : 0;   // the table's form
          S.dump_list[2 * slot + 1] = dumped ? c : -1;
          if (compact) S.dump_um[slot] = um | (rootp ? (1ull << 63) : 0ull);
        }
        staged = true;                                 // (its attachment counts stand)
        WSTAT(21, 1);
        WLAP(9);
        break;
      }
      WLAP(9);
      if (staged || outcome == 2) break;
      const int Gu = __popcll(um);
      wave_sync();
      int dec = -1;
      if constexpr (FULL) dec = wave_two(S, F, c, h0, l0, G, ns, um, Gu, iteration, pair_evals);
      if (dec < 0) {
        staged = true;
        break;
      }
      if (dec == kDecDone) break;
      if (dec == kDecRaise && iteration + 1 <= kMaxIter) {
        if (!rollup) {                                 // the staged kernels start at level 1
          staged = true;
          seed = iteration == 1;
          if (lane == 0) K.pair_evals[c] = pair_evals;
          break;
        }
        wave_sync();
        continue;
      }
      if (lane == 0) {                                 // unclassified after evaluation
        K.iters[c] = (int16_t)min(dec == kDecRaise ? iteration + 1 : iteration, 32767);
        K.pair_evals[c] = pair_evals;
        K.status[c] = dec == kDecRaise ? WF_E_RUNAWAY : 0;
      }
      break;
    }
    if (lane == 0) {
      ccnt[c] = staged ? n_att : 0;
      cleaves[c] = staged ? nl_sum : 0;
      const int pd = staged ? (dumped ? 3 : (seed ? 2 : 1)) : 0;
      pend[c] = pd;
      if (pd == 1 && S.fail_ctr) atomicAdd(S.fail_ctr, 1ull);   // (wave levels: staged from level 0)
    }
    WSTAT(22, staged ? 1 : 0);
    wave_sync();                                       // the slice is reused by the next contig
    WLAP(10);
  }
}

// Resident k_wave workgroups per CU.  One value per process (every device is a gfx950 with
// the same kernel image); the static's initialisation is thread-safe (C++11), so contexts on
// several host threads may call this concurrently.
template <int CAP, bool FULL, bool ROLL = false>
int blocks_per_cu() {
  static const int n = [] {
    const int bytes = (int)sizeof(WaveSmem<CAP, FULL>);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_wave<CAP, FULL, ROLL>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, reinterpret_cast<const void*>(&k_wave<CAP, FULL, ROLL>), 64,
                                                     bytes) != hipSuccess || b < 1)
      b = 1;
    return b;
  }();
  return n;
}

// n_list: the list length, or (n_dev set) an upper bound for the grid
template <int CAP, bool FULL, bool ROLL = false>
hipError_t launch_cap(const SArgs& sa, int64_t* ccnt, int64_t* cleaves, int32_t* pend, const int32_t* list,
                      int n_list, const int64_t* n_dev, int cus, int rollup, hipStream_t s, int start_level = 0) {
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(n_list, (int64_t)cus * blocks_per_cu<CAP, FULL, ROLL>()));
  hipLaunchKernelGGL((k_wave<CAP, FULL, ROLL>), dim3(grid), dim3(64), sizeof(WaveSmem<CAP, FULL>), s, sa, ccnt, cleaves, pend,
                     list, n_list, n_dev, rollup, start_level);
  return hipGetLastError();
}

}  // namespace

WF_STAMP_READER(fast, g_wstamps, 48)

hipError_t launch_fast(const SArgs& sa, int64_t* ccnt, int64_t* cleaves, int32_t* pend, int max_hits, int cus,
                       hipStream_t s) {
  const int N = sa.k.n_contigs;
  if (max_hits <= 224) return launch_cap<224, false>(sa, ccnt, cleaves, pend, nullptr, N, nullptr, cus, 0, s);
  return max_hits <= 256 ? launch_cap<256, false>(sa, ccnt, cleaves, pend, nullptr, N, nullptr, cus, 0, s)
                         : launch_cap<512, false>(sa, ccnt, cleaves, pend, nullptr, N, nullptr, cus, 0, s);
}

hipError_t launch_fast_list(const SArgs& sa, int64_t* ccnt, int64_t* cleaves, int32_t* pend, const int32_t* list,
                            const int64_t* n_dev, int max_hits, int cus, hipStream_t s) {
  const int N = sa.k.n_contigs;
  if (max_hits <= 224) return launch_cap<224, false>(sa, ccnt, cleaves, pend, list, N, n_dev, cus, 0, s);
  return max_hits <= 256 ? launch_cap<256, false>(sa, ccnt, cleaves, pend, list, N, n_dev, cus, 0, s)
                         : launch_cap<512, false>(sa, ccnt, cleaves, pend, list, N, n_dev, cus, 0, s);
}

hipError_t launch_level(const SArgs& sa, int64_t* ccnt, int64_t* cleaves, int32_t* pend, const int32_t* list,
                        const int64_t* n_dev, int level, int max_hits, int cus, hipStream_t s) {
  const int N = sa.k.n_contigs;
  if (max_hits <= 224) return launch_cap<224, false, true>(sa, ccnt, cleaves, pend, list, N, n_dev, cus, 0, s, level);
  return max_hits <= 256 ? launch_cap<256, false, true>(sa, ccnt, cleaves, pend, list, N, n_dev, cus, 0, s, level)
                         : launch_cap<512, false, true>(sa, ccnt, cleaves, pend, list, N, n_dev, cus, 0, s, level);
}

hipError_t launch_full(const SArgs& sa, int64_t* ccnt, int64_t* cleaves, int32_t* pend, const int32_t* list,
                       const int64_t* n_dev, int max_hits, int cus, bool rollup, hipStream_t s) {
  const int N = sa.k.n_contigs;
  return max_hits <= 256 ? launch_cap<256, true>(sa, ccnt, cleaves, pend, list, N, n_dev, cus, rollup, s)
                         : launch_cap<512, true>(sa, ccnt, cleaves, pend, list, N, n_dev, cus, rollup, s);
}

}  // namespace wf
