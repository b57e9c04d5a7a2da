// One roll-up level for contigs with many clade rows, straight from the segment table
// (orgscorer.py:407-429, 566-744), one wave per contig.  Included by wf_staged.hip inside
// its anonymous namespace.
//
// The dense decision (decide_contig) materialises the gene-score matrix S (clades x loci)
// and reads it many times; at the stress shape (~5,000 clades x 20 loci)
// that matrix is ~0.8 MB per contig in an HBM slot.  Here S is never built.  A clade's row
// is its run of segments (the segment table is sorted by clade, then locus; a locus without
// a segment scores 0), and every quantity the level needs is either a per-row bit summary
// taken while streaming the runs, or comes from the few rows that can still form an option:
//
//   pass 1  segment-parallel: per-locus maxes over known clades (:407-411), root present
//           -> weak loci (:420-427), the unmasked-locus set `keep`
//   pass 2  row-parallel (lane per clade run, runs in clade order): explain_one's test
//           crit >= k1 <=> every kept locus >= k1 (bit summary), its rank only for options;
//           potential clades (max over all loci >= k2, :603-605) counted in order and their
//           ">= k2 on kept loci" masks entered into a class table in LDS
//   classes crit(c1,c2) >= k2 <=> (m1 | m2) == keep: the test runs on class pairs; the
//           passing class pairs hold exactly the reference's candidate pairs
//   pass 3  row-parallel: the clades of those classes ("members": potential index, run
//           start, sister mask, listed parent) into the wave's HBM scratch, grouped by class
//   pass 4  row-parallel, --sister-penalty on: for every parent of a member, per locus, how
//           many present clades listed under it score >= the threshold (saturating at 3:
//           one pair removes at most its two clades, get_sisters(c1) - {c2}, :717-744)
//   pairs   the passing class pairs' members: rank (numpy order), best by (rank, pair
//           index), eval_two and meld_two exactly as decide_two, rows read from the runs
//
// The passes stage the contig's segments through LDS 256 at a time (plus 64 ahead: a run
// has at most 63 segments), so a run is walked in LDS and each step of a pass waits on one
// batch of coalesced loads.  --weak-loci assign-unknown (:416-418): the "Unknown" row is
// 1 - maxes on every locus, kept in LDS and entered in clade order (a real "Unknown"
// clade's run is replaced by it).  A contig whose classes or class pairs outgrow the LDS
// tables, whose members outgrow the scratch, or with > 63 loci goes on to the dense
// decision (k_decide_big) instead.
constexpr int kSpCls = 128;      // mask-class hash slots (at most 3/4 used)
constexpr int kSpPairs = 128;    // passing class pairs
constexpr int kSpMemG = 2048;    // member clades per contig (HBM scratch)
constexpr int kSpParG = 4096;    // parent hash slots (HBM scratch), >= 2 * members
constexpr int kSpDense = 16384;  // dense member rows (members x loci doubles, HBM scratch)
constexpr int kSpWin = 256;      // segments staged per step (128: 0.04 ms slower, s6a)
constexpr int kSpMaxG = 63;      // loci per contig (mask bits; ~0 marks an empty class slot)
constexpr int kSpP1 = 8;         // pass 1: 64-segment chunks per step (one round trip each)

struct SpMember {                // 32 B
  int rs, cl, pi, sp;            // run start (-1: the virtual "Unknown" row), clade,
                                 // potential index, listed parent
  int h, pad;                    // class slot
  unsigned long long hm;         // loci >= the sister threshold (all loci)
};
struct SpParent {                // 32 B: parent id (~0: empty), clades >= threshold at a
  unsigned long long key, c1, c2, c3;   // locus: >= 1, >= 2, >= 3 (bit per locus)
};
// parent-table slots held in LDS (up to 32 members: at cfg5 a contig has 2); more go to the
// wave's HBM scratch.  Pass 4 probes the table once per clade run of the contig (~5,000 at
// the stress shape): in HBM each probe was a dependent global load.
constexpr int kSpLPar = 64;
static_assert(kSpLPar * 32 == kSpCls * (8 + 4 + 4), "lpar overlays the class table");
// per-wave scratch: members (in the order found) | their positions grouped by class | parents
// | the members' dense rows | the virtual "Unknown" row | the melded-member bit sets (the
// last two kept out of LDS: k_big_sparse's LDS sets its residency, 13 waves per CU at 12 KB)
constexpr int64_t kSpOffGidx = (int64_t)kSpMemG * sizeof(SpMember);
constexpr int64_t kSpOffPar = kSpOffGidx + (int64_t)kSpMemG * sizeof(int);
constexpr int64_t kSpOffDense = kSpOffPar + (int64_t)kSpParG * sizeof(SpParent);
constexpr int64_t kSpOffUrow = kSpOffDense + (int64_t)kSpDense * sizeof(double);
constexpr int64_t kSpOffBm = kSpOffUrow + 64 * sizeof(double);
constexpr int64_t kSpSlot = kSpOffBm + 2 * (kSpMemG / 32) * sizeof(unsigned);

struct SpShared {
  // (wcg and wv are contiguous: after pass 4 they hold the members' dense rows, kSpLdsRows)
  int2 wcg[kSpWin + 64];                     // staged segments: (clade, locus) ...
  double wv[kSpWin + 64];                    // ... and gene score
  unsigned long long mx[64];                 // per-locus max score bits (known clades)
  union {
    struct {                                 // the class table (passes 2, 3) ...
      unsigned long long ckey[kSpCls];       // class mask (~0: empty)
      int cmany[kSpCls];                     // the class has at least 2 potential clades
      int cint[kSpCls];                      // class is in a passing pair
    };
    SpParent lpar[kSpLPar];                  // ... then (pass 4 on) the parent table, when it fits
  };
  int ccnt[kSpCls];                          // members of a passing class (pass 3)
  int cls[kSpCls];                           // occupied slots, compacted
  int coff[kSpCls], cfill[kSpCls];           // members of the class: first, filled
  int pair[kSpPairs];                        // passing class pairs: a | b << 16 (a <= b)
  int pref[kSpPairs + 1];                    // candidate-pair prefix
  double row[64];                            // one dense row (explain_one's best)
  int len[64];                               // locus lengths (ambiguous fraction)
  uint8_t syn[64];                           // best option's synteny
  int n_used, n_pairs, n_in, all_ok, all_same, cnt, over;
};

constexpr int kSpLdsRows = 2 * (kSpWin + 64);      // doubles over wcg + wv
static_assert(offsetof(SpShared, wv) == sizeof(int2) * (kSpWin + 64), "wcg, wv contiguous");

__device__ __forceinline__ int sp_hash(uint64_t m, int cap) {
  return (int)((m * 0x9E3779B97F4A7C15ull) >> 40) & (cap - 1);
}

// Value of clade run `cl` at locus g (0 without a segment), from the segment table in HBM,
// or of the virtual row `vrow` (run start < 0); calls in ascending g.
struct SpCursor {
  int t, cl, se;
  const double* vrow;
  __device__ __forceinline__ double at(const SArgs& S, int g) {
    if (vrow) return vrow[g];
    while (t < se) {
      const int2 cg = S.seg_cg[t];
      if (cg.x != cl || cg.y >= g) break;
      ++t;
    }
    if (t < se) {
      const int2 cg = S.seg_cg[t];
      if (cg.x == cl && cg.y == g) return S.seg_mean[t];
    }
    return 0.0;
  }
};

// A member's row for the pair evaluations: its dense copy in the scratch when the members'
// rows fit it (independent loads), else read from the run (dependent loads).
struct SpRowAcc {
  const double* d;
  SpCursor c;
  __device__ __forceinline__ double at(const SArgs& S, int g) { return d ? d[g] : c.at(S, g); }
};

// Bit summary of the run staged at window index w: loci at or above k1 / k2 / the sister
// threshold (a locus without a segment scores 0.0 and is compared as such).
struct SpRow {
  uint64_t mk1, mk2, mhs;
};

__device__ __forceinline__ SpRow sp_row(const SpShared& sh, const DevParams& P, int w, int cl, uint64_t allg) {
  uint64_t cov = 0, k1 = 0, k2 = 0, hs = 0;
  for (; sh.wcg[w].x == cl; ++w) {
    const double v = sh.wv[w];
    const uint64_t bit = 1ull << sh.wcg[w].y;
    cov |= bit;
    if (v >= P.k1) k1 |= bit;
    if (v >= P.k2) k2 |= bit;
    if (v >= P.sister_thr) hs |= bit;
  }
  const uint64_t z = allg & ~cov;
  SpRow r;
  r.mk1 = k1 | (0.0 >= P.k1 ? z : 0ull);
  r.mk2 = k2 | (0.0 >= P.k2 ? z : 0ull);
  r.mhs = hs | (0.0 >= P.sister_thr ? z : 0ull);
  return r;
}

// numpy-order mean over the kept loci of the run staged at w (Contig.score, :447-461)
__device__ __forceinline__ double sp_rank_w(const SpShared& sh, int w, int cl, uint64_t keep, int Gu) {
  uint64_t m = keep;
  auto next = [&]() -> double {
    const int g = __builtin_ctzll(m);
    m &= m - 1;
    while (sh.wcg[w].x == cl && sh.wcg[w].y < g) ++w;
    return (sh.wcg[w].x == cl && sh.wcg[w].y == g) ? sh.wv[w] : 0.0;
  };
  return (0.0 + np_sum_seq(Gu, next)) / (double)Gu;
}

// Runs of the contig's segments [so, se) in clade order, one per lane: f(is_start, t, w, cl)
// is called by every lane of the wave for each 64-segment chunk (is_start false on lanes
// that hold no run start; t the segment, w its window index), so f may use wave operations.
// The window holds kSpWin segments plus 64 ahead (clade -2 past the contig's end).
// The next window's loads are issued before this one is walked (registers, then LDS at the
// next step), so each step's global round trip overlaps the previous step's run walks
// instead of stalling the wave (a stress contig is ~20 windows per pass, four passes).
template <class F>
__device__ __forceinline__ void sp_rows(const SArgs& S, SpShared& sh, int so, int se, F f) {
  const int lane = threadIdx.x & 63;
  int carry = -1;
  int2 cg[kSpWin / 64 + 1];
  double v[kSpWin / 64 + 1];
  auto fetch = [&](int base) {
#pragma unroll
    for (int j = 0; j < kSpWin / 64 + 1; ++j) {
      const int t = base + 64 * j + lane;
      cg[j] = t < se ? S.seg_cg[t] : make_int2(-2, 0);
      v[j] = t < se ? S.seg_mean[t] : 0.0;
    }
  };
  if (so < se) fetch(so);
  for (int base = so; base < se; base += kSpWin) {
    __syncthreads();                                 // the previous window is consumed
#pragma unroll
    for (int j = 0; j < kSpWin / 64 + 1; ++j) {
      sh.wcg[64 * j + lane] = cg[j];
      sh.wv[64 * j + lane] = v[j];
    }
    __syncthreads();
    if (base + kSpWin < se) fetch(base + kSpWin);    // (in flight while this window is walked)
#pragma unroll 1
    for (int j = 0; j < kSpWin / 64; ++j) {
      const int w = 64 * j + lane;
      const int cl = sh.wcg[w].x;
      const int prev = w == 0 ? carry : sh.wcg[w - 1].x;
      f(base + w < se && cl != prev, base + w, w, cl);
    }
    carry = sh.wcg[kSpWin - 1].x;
  }
  __syncthreads();
}

// sp_rows with one dependent global load per run start hoisted out of the run walks:
// pre(t, cl) is evaluated for the window's four 64-segment chunks first (their loads issue
// together), then f(is_start, t, w, cl, pre value) per chunk.  Chunks unrolled (the
// prefetched values stay in registers).
template <class Pre, class F>
__device__ __forceinline__ void sp_rows_pf(const SArgs& S, SpShared& sh, int so, int se, Pre pre, F f) {
  const int lane = threadIdx.x & 63;
  int carry = -1;
  int2 cg[kSpWin / 64 + 1];
  double v[kSpWin / 64 + 1];
  auto fetch = [&](int base) {
#pragma unroll
    for (int j = 0; j < kSpWin / 64 + 1; ++j) {
      const int t = base + 64 * j + lane;
      cg[j] = t < se ? S.seg_cg[t] : make_int2(-2, 0);
      v[j] = t < se ? S.seg_mean[t] : 0.0;
    }
  };
  if (so < se) fetch(so);
  for (int base = so; base < se; base += kSpWin) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kSpWin / 64 + 1; ++j) {
      sh.wcg[64 * j + lane] = cg[j];
      sh.wv[64 * j + lane] = v[j];
    }
    __syncthreads();
    if (base + kSpWin < se) fetch(base + kSpWin);
    int pv[kSpWin / 64];
    bool st[kSpWin / 64];
#pragma unroll
    for (int j = 0; j < kSpWin / 64; ++j) {
      const int w = 64 * j + lane;
      const int cl = sh.wcg[w].x;
      const int prev = w == 0 ? carry : sh.wcg[w - 1].x;
      st[j] = base + w < se && cl != prev;
      pv[j] = pre(st[j], cl);
    }
#pragma unroll
    for (int j = 0; j < kSpWin / 64; ++j) {
      const int w = 64 * j + lane;
      f(st[j], base + w, w, sh.wcg[w].x, pv[j]);
    }
    carry = sh.wcg[kSpWin - 1].x;
  }
  __syncthreads();
}

// (rank, crit) of a clade pair over the kept loci: numpy-order mean and min of the
// per-locus max (orgscorer.py:447-461), rows read from the segment table.
__device__ __forceinline__ double sp_pair_rank(const SArgs& S, SpRowAcc a, SpRowAcc b, uint64_t keep, int Gu) {
  uint64_t m = keep;
  auto next = [&]() -> double {
    const int g = __builtin_ctzll(m);
    m &= m - 1;
    const double x = a.at(S, g), y = b.at(S, g);
    return x < y ? y : x;
  };
  return (0.0 + np_sum_seq(Gu, next)) / (double)Gu;
}

__device__ __forceinline__ double sp_pair_crit(const SArgs& S, SpRowAcc a, SpRowAcc b, uint64_t keep) {
  double m = 0.0;
  bool first = true;
  for (uint64_t r = keep; r; r &= r - 1) {
    const int g = __builtin_ctzll(r);
    const double x = a.at(S, g), y = b.at(S, g);
    const double v = x < y ? y : x;
    m = (first || v < m) ? v : m;
    first = false;
  }
  return m;
}

// parent table (open addressing, capacity pcap, a power of 2)
__device__ __forceinline__ const SpParent* sp_par_find(const SpParent* tab, int pcap, int p) {
  for (int h = sp_hash((uint64_t)p, pcap), n = 0; n < pcap; h = (h + 1) & (pcap - 1), ++n) {
    const unsigned long long k = tab[h].key;
    if (k == (unsigned long long)p) return &tab[h];
    if (k == ~0ull) return nullptr;
  }
  return nullptr;
}

// Loci where a clade listed under parent entry e, other than clades X and Y, scores >= the
// sister threshold: the saturating counts minus X's and Y's own contributions.
__device__ __forceinline__ uint64_t sp_sisters(const SpParent* e, int p, const SpMember& X, const SpMember& Y) {
  if (!e) return 0ull;
  const uint64_t dx = X.sp == p ? X.hm : 0ull, dy = Y.sp == p ? Y.hm : 0ull;
  const uint64_t sub2 = dx & dy, sub1 = dx ^ dy;
  return e->c3 | (e->c2 & ~sub2) | (e->c1 & ~sub1 & ~sub2);
}

// eval_two (wf_device.h, G <= 64 form) for members A (potential index i) and B (j > i):
// the synteny masks from the two runs, swap rule, direction, LGT filters, sister penalty.
// c1p / c2p of the result are 0 (A) or 1 (B).
__device__ __forceinline__ OptEval sp_eval_two(const SArgs& S, const SpShared& sh, const SpMember& A,
                                               const SpMember& B, SpRowAcc a, SpRowAcc b, const SpParent* par,
                                               int pcap, int G, uint64_t ign, bool cmp, uint8_t* out) {
  const KArgs& K = S.k;
  const DevParams& P = K.p;
  const bool unk = A.cl == K.unknown || B.cl == K.unknown;
  uint64_t mm = 0, ma = 0, mb = 0;
  for (int g = 0; g < G; ++g) {
    const uint64_t bit = 1ull << g;
    const double s1 = a.at(S, g), s2 = b.at(S, g);
    const double mn = s2 < s1 ? s2 : s1;
    if (ign & bit) continue;
    if (mn >= P.k_amb && !unk) mm |= bit;
    else if (s1 >= P.k2) ma |= bit;
    else if (s2 >= P.k2) mb |= bit;
  }
  OptEval e;
  const uint64_t ab = ma | mb;                     // "^[^A]*B" -> swap (:537-540)
  e.swapped = (ab && ((mb >> __builtin_ctzll(ab)) & 1ull)) ? 1 : 0;
  const uint64_t mA = e.swapped ? mb : ma, mB = e.swapped ? ma : mb;
  e.same = 1;
  int64_t tot = 0, amb = 0;
  int state = 0;
  bool dir_ok = true;
  for (int g = 0; g < G; ++g) {
    const uint64_t bit = 1ull << g;
    const uint8_t c = (ign & bit) ? '~' : (mm & bit) ? '*' : (mA & bit) ? 'A' : (mB & bit) ? 'B' : '!';
    if (out) out[g] = c;
    if (cmp && sh.syn[g] != c) e.same = 0;
    if (c == 'A' || c == 'B' || c == '*') {
      tot += sh.len[g];
      if (c == '*') amb += sh.len[g];
    }
    if (c != '~') {  // "^A+B+A+$" on synteny without '~' (orgscorer.py:542)
      if (state == 0) { if (c == 'A') state = 1; else dir_ok = false; }
      else if (state == 1) { if (c == 'B') state = 2; else if (c != 'A') dir_ok = false; }
      else if (state == 2) { if (c == 'A') state = 3; else if (c != 'B') dir_ok = false; }
      else { if (c != 'A') dir_ok = false; }
    }
  }
  const int nA = __popcll(mA), nB = __popcll(mB);
  e.dir = (dir_ok && state == 3) ? 1 : 0;
  e.c1p = e.swapped ? 1 : 0;
  e.c2p = e.swapped ? 0 : 1;
  e.ok = 1;
  if ((double)amb / (double)tot > P.amb_frac) e.ok = 0;           // :693-702
  if (P.clade_genes >= 0 && min(nA, nB) < P.clade_genes) e.ok = 0; // :704-708
  const SpMember& X = e.swapped ? B : A;
  const SpMember& Y = e.swapped ? A : B;
  if (P.clade_leaves >= 0) {                                       // :710-715
    const int64_t lc = e.dir ? K.leaves[Y.cl] : min(K.leaves[X.cl], K.leaves[Y.cl]);
    if (lc < P.clade_leaves) e.ok = 0;
  }
  if (P.sister_on && e.ok) {                                       // :717-744
    const int px = K.parent[X.cl], py = K.parent[Y.cl];
    const uint64_t fb = sp_sisters(sp_par_find(par, pcap, px), px, X, Y);   // sisters of X
    const uint64_t fa = sp_sisters(sp_par_find(par, pcap, py), py, X, Y);   // sisters of Y
    if ((fb & mB) || (!e.dir && (fa & mA))) e.ok = 0;
  }
  return e;
}

// Every candidate pair (the members of each passing class pair): f(u, v, mu, mv) on the
// lane that owns it, mu's potential index below mv's.
template <class F>
__device__ __forceinline__ void sp_for_cands(const SpShared& sh, const SpMember* mem, const int* gidx, F f) {
  const int lane = threadIdx.x & 63;
  const int np = sh.n_pairs;
  const int T = sh.pref[np];
  for (int x = lane; x < T; x += 64) {
    int lo = 0, hi = np - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (sh.pref[mid] <= x) lo = mid; else hi = mid - 1;
    }
    const int a = sh.pair[lo] & 0xFFFF, b = sh.pair[lo] >> 16;
    const int y = x - sh.pref[lo];
    const int a0 = sh.coff[a], na = sh.ccnt[a];
    int u, v;
    if (a == b) {
      // y-th (p, q), p < q, in row-major order: row p starts at p*(2na-p-1)/2
      int plo = 0, phi = na - 2;
      while (plo < phi) {
        const int mid = (plo + phi + 1) >> 1;
        if ((long long)mid * (2 * na - mid - 1) / 2 <= y) plo = mid; else phi = mid - 1;
      }
      const int rs = (int)((long long)plo * (2 * na - plo - 1) / 2);
      u = a0 + plo;
      v = a0 + plo + 1 + (y - rs);
    } else {
      const int nb = sh.ccnt[b];
      u = a0 + y / nb;
      v = sh.coff[b] + y % nb;
    }
    const int qu = gidx[u], qv = gidx[v];
    const SpMember mu = mem[qu], mv = mem[qv];
    if (mu.pi < mv.pi) f(qu, qv, mu, mv);
    else f(qv, qu, mv, mu);
  }
}

// Roll-up bookkeeping of one contig raised by one wave (decide_contig's kDecRaise branch).
__device__ __forceinline__ void sp_raise(const SArgs& S, int c, int64_t pair_evals) {
  const KArgs& K = S.k;
  const int lane = threadIdx.x & 63;
  const int64_t a0 = S.catt_off[c], a1 = S.catt_off[c + 1];
  if (lane == 0) {
    const unsigned long long old = atomicAdd(&S.counters[0], (1ull << 40) | (unsigned long long)(a1 - a0));
    const int slot = (int)(old >> 40);
    S.act_next[slot] = c;
    S.act_base_next[slot] = (int64_t)(old & ((1ull << 40) - 1));
    K.pair_evals[c] = pair_evals;
  }
  for (int64_t ab = a0; ab < a1; ab += 4 * 64) {
    int cl[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t a = ab + r * 64 + lane;
      cl[r] = a < a1 ? S.att_clade[a] : 0;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) cl[r] = K.parent[cl[r]];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t a = ab + r * 64 + lane;
      if (a < a1) S.att_clade[a] = cl[r];
    }
  }
}

// Returns false when the contig must go to the dense decision (nothing written then).
// `ws`: this wave's HBM scratch (kSpSlot bytes).
__device__ __forceinline__ bool sp_level(const SArgs& S, SpShared& sh, char* ws, int c, int cr, int level,
                                         int64_t n_keys) {
  const KArgs& K = S.k;
  const DevParams& P = K.p;
  const int lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1ull;
  const int64_t h0 = K.hit_off[c];
  const int64_t l0 = K.loc_off[c];
  const int G = (int)(K.loc_off[c + 1] - l0);
  if (K.hit_off[c + 1] == h0 || G == 0) return true;   // never evaluated (orgscorer.py:959)
  if (G > kSpMaxG) return false;
  const int so = n_keys > 0 ? S.crank_first[cr] : 0;
  const int se = n_keys > 0 ? S.crank_first[cr + 1] : 0;
  const uint64_t allg = (1ull << G) - 1ull;
  const int64_t mbase = 2 * h0 + 2 * (int64_t)c;
  const int iteration = level + 1;
  int64_t pair_evals = level == 0 ? 0 : K.pair_evals[c];
  SpMember* mem = reinterpret_cast<SpMember*>(ws);
  int* gidx = reinterpret_cast<int*>(ws + kSpOffGidx);
  SpParent* par = reinterpret_cast<SpParent*>(ws + kSpOffPar);
  double* drows = reinterpret_cast<double*>(ws + kSpOffDense);
  double* urow = reinterpret_cast<double*>(ws + kSpOffUrow);   // --weak-loci assign-unknown: 1 - maxes
  unsigned* bm1 = reinterpret_cast<unsigned*>(ws + kSpOffBm);  // members melded as clade 1 / 2
  unsigned* bm2 = bm1 + kSpMemG / 32;
  BLAP_MARK(c);
  BSTAT(15, 1);
  BSTAT(12, se - so);
  BSTAT(19 + min(level, 2), 1);
  if (level > 0) BSTAT(34, 1);

  // ---- pass 1: per-locus maxes over known clades, root present (:407-411) -------------
  sh.mx[lane] = 0;
  if (lane < G) {
    const int ls = K.lstart[l0 + lane], le = K.lend[l0 + lane];
    sh.len[lane] = max(ls, le) - min(ls, le) + 1;
  }
  for (int i = lane; i < kSpCls; i += 64) {
    sh.ckey[i] = ~0ull; sh.cmany[i] = 0; sh.ccnt[i] = 0; sh.cint[i] = 0; sh.cfill[i] = 0;
  }
  if (lane == 0) { sh.n_used = 0; sh.n_pairs = 0; sh.cnt = 0; sh.over = 0; }
  __syncthreads();
  bool root = false;
  {
    int2 cg[kSpP1];
    double v[kSpP1];
    auto fetch = [&](int base) {
#pragma unroll
      for (int j = 0; j < kSpP1; ++j) {
        const int t = base + 64 * j + lane;
        cg[j] = t < se ? S.seg_cg[t] : make_int2(-2, 0);
        v[j] = t < se ? S.seg_mean[t] : 0.0;
      }
    };
    if (so < se) fetch(so);
    for (int base = so; base < se; base += 64 * kSpP1) {
      int2 c2[kSpP1];
      double v2[kSpP1];
#pragma unroll
      for (int j = 0; j < kSpP1; ++j) { c2[j] = cg[j]; v2[j] = v[j]; }
      if (base + 64 * kSpP1 < se) fetch(base + 64 * kSpP1);   // (the next step's loads in flight)
#pragma unroll
      for (int j = 0; j < kSpP1; ++j) {
        root |= c2[j].x == K.root;
        if (c2[j].x >= 0 && c2[j].x != K.unknown && v2[j] > 0.0) atomicMax(&sh.mx[c2[j].y], dbits(v2[j]));
      }
    }
  }
  const bool root_present = __ballot(root) != 0ull;
  __syncthreads();
  BLAP(0);
  // weak loci: ignore -> mask (:420-427), penalize -> none (:413-414)
  const double mxv = __longlong_as_double((long long)sh.mx[lane]);
  const uint64_t keep = __ballot(lane < G && (P.weak != 0 || mxv >= P.kmin));
  const uint64_t ign = allg & ~keep;
  const int Gu = __popcll(keep);
  // --weak-loci assign-unknown: the virtual "Unknown" row 1 - maxes (:416-418) and its bits
  const bool vu = P.weak == 2;
  const double uval = 1.0 - mxv;
  if (vu && lane < G) urow[lane] = uval;
  if (vu) __threadfence_block();                    // (read by other lanes after pass 2's barriers)
  const uint64_t u_k1 = vu ? __ballot(lane < G && uval >= P.k1) : 0ull;
  const uint64_t u_k2 = vu ? __ballot(lane < G && uval >= P.k2) : 0ull;
  const uint64_t u_hs = vu ? __ballot(lane < G && uval >= P.sister_thr) : 0ull;
  const bool u_pot = u_k2 != 0ull;                  // max over all loci >= k2 (:603-605)
  const bool no_rows = se == so && !vu;             // Pn == 0
  if (level == 0 && keep == 0) return true;        // skipped contig (orgscorer.py:959)
  if (Gu == 0) {                                    // np.min of an empty array upstream
    if (lane == 0) {
      K.iters[c] = (int16_t)min(iteration, 32767);
      K.pair_evals[c] = pair_evals;
      K.status[c] = WF_E_EMPTYMASK;
    }
    return true;
  }

  // ---- pass 2: explain_one options, potential clades, mask classes ------------------------
  double br = -__builtin_inf();
  long long bk = -1;
  int brs = -1;
  int Pp = 0, upi = 0;                              // upi: potential clades before "Unknown"
  // class table: a plain read finds an existing class; only a new one takes a CAS (the
  // loser of a race for the same new class is its second clade)
  auto ins_class = [&](uint64_t cmask) {
    int h = sp_hash(cmask, kSpCls);
    for (int probe = 0; probe < kSpCls; ++probe) {
      unsigned long long k = sh.ckey[h];
      if (k == ~0ull) {
        k = atomicCAS(&sh.ckey[h], ~0ull, (unsigned long long)cmask);
        if (k == ~0ull) { atomicAdd(&sh.n_used, 1); break; }
      }
      if (k == cmask) { sh.cmany[h] = 1; break; }
      h = (h + 1) & (kSpCls - 1);
    }
  };
  WF_STAMPS_ONLY(unsigned long long p2_row = 0, p2_ins = 0);   // (stamps: pass 2's row summaries / class inserts)
  sp_rows(S, sh, so, se, [&](bool st, int t, int w, int cl) {
    WF_STAMPS_ONLY(const unsigned long long q0 = __builtin_amdgcn_s_memtime());
    // past 3/4 of the class table the contig goes to the dense decision unless it has an
    // explain_one option: stop inserting (a full table made every new class probe all of it)
    const bool cls_full = sh.n_used * 4 > kSpCls * 3;
    bool pot = false;
    uint64_t cmask = 0;
    if (st && !(vu && cl == K.unknown)) {          // (a real "Unknown" run is replaced)
      const SpRow r = sp_row(sh, P, w, cl, allg);
      if ((r.mk1 & keep) == keep) {                 // crit >= k1 (:585-597)
        const double rank = sp_rank_w(sh, w, cl, keep, Gu);
        if (better(rank, cl, br, bk)) { br = rank; bk = cl; brs = t; }
      }
      pot = r.mk2 != 0ull;                          // max over all loci >= k2 (:603-605)
      cmask = r.mk2 & keep;
    }
    Pp += __popcll(__ballot(pot));
    upi += __popcll(__ballot(pot && cl < K.unknown));
    WF_STAMPS_ONLY(const unsigned long long q1 = __builtin_amdgcn_s_memtime());
    if (pot && !cls_full) ins_class(cmask);
    WF_STAMPS_ONLY(const unsigned long long q2 = __builtin_amdgcn_s_memtime(); p2_row += q1 - q0; p2_ins += q2 - q1);
  });
  WF_STAMPS_ONLY(BSTAT(10, p2_row); BSTAT(11, p2_ins));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double r2 = __shfl_xor(br, off, 64);
    const long long k2 = __shfl_xor(bk, off, 64);
    const int rs2 = __shfl_xor(brs, off, 64);
    if (better(r2, k2, br, bk)) { br = r2; bk = k2; brs = rs2; }
  }
  // the virtual "Unknown" row: an option, a potential clade
  double u_rank = 0.0;
  const bool u_opt = vu && (u_k1 & keep) == keep;
  if (u_opt) {
    uint64_t m = keep;
    auto next = [&]() -> double {
      const int g = __builtin_ctzll(m);
      m &= m - 1;
      return urow[g];
    };
    u_rank = (0.0 + np_sum_seq(Gu, next)) / (double)Gu;
    if (better(u_rank, K.unknown, br, bk)) { br = u_rank; bk = K.unknown; brs = -1; }
  }
  if (u_pot) {
    Pp += 1;
    if (lane == 0 && sh.n_used * 4 <= kSpCls * 3) ins_class(u_k2 & keep);
  }
  __syncthreads();
  BLAP(1);
  BSTAT(13, Pp);

  if (bk >= 0) {
    BSTAT(18, 1);
    // meld_one (:621-631): options within --range of the best
    const int best = (int)bk;
    int acc = -1;
    if (P.dis1 == 1) {
      sp_rows(S, sh, so, se, [&](bool st, int, int w, int cl) {
        if (!st || (vu && cl == K.unknown)) return;
        const SpRow r = sp_row(sh, P, w, cl, allg);
        if ((r.mk1 & keep) != keep) return;
        const double rank = sp_rank_w(sh, w, cl, keep, Gu);
        if ((br - rank) <= P.range) {
          K.meld[mbase + atomicAdd(&sh.cnt, 1)] = cl;
          acc = lca2(K, acc, cl);
        }
      });
      if (u_opt && lane == 0 && (br - u_rank) <= P.range) {
        K.meld[mbase + atomicAdd(&sh.cnt, 1)] = K.unknown;
        acc = lca2(K, acc, K.unknown);
      }
      __syncthreads();
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) acc = lca2(K, acc, __shfl_xor(acc, off, 64));
    }
    const int m = sh.cnt;
    if (P.dis1 == 1 && m == 0) {                    // negative --range: get_lca() of nothing
      if (lane == 0) K.status[c] = WF_E_BADINPUT;
      return true;
    }
    // the best clade's row: crit (min over kept loci) and set_synteny_one (:495-509)
    sh.row[lane] = brs < 0 && lane < G ? urow[lane] : 0.0;
    __syncthreads();
    if (brs >= 0) {
      const int t = brs + lane;
      if (t < se) {
        const int2 cg = S.seg_cg[t];
        if (cg.x == best) sh.row[cg.y] = S.seg_mean[t];
      }
    }
    __syncthreads();
    if (lane < G) {
      const double s = sh.row[lane];
      K.syn[l0 + lane] = ((ign >> lane) & 1ull) ? '~' : (s >= P.k1 ? 'A' : '!');
    }
    if (lane == 0) {
      double crit = 0.0;
      bool first = true;
      for (uint64_t r = keep; r; r &= r - 1) {
        const double v = sh.row[__builtin_ctzll(r)];
        crit = (first || v < crit) ? v : crit;
        first = false;
      }
      K.call[c] = WF_CALL_NO_LGT;
      K.crit[c] = crit;
      K.rank[c] = br;
      K.c1[c] = P.dis1 == 1 ? acc : best;
      K.c2[c] = -1;
      K.nm1[c] = P.dis1 == 1 ? m : 0;
      K.iters[c] = (int16_t)iteration;
      K.pair_evals[c] = pair_evals;
    }
    BLAP(2);
    return true;
  }

  // ---- explain_two (:599-619) --------------------------------------------------------
  pair_evals += (int64_t)Pp * (Pp - 1) / 2;
  if (lane == 0) note_ppot(K, c, iteration, Pp);
  if (sh.n_used * 4 > kSpCls * 3) {                // too many classes for the table
    BSTAT(16, 1);
    return false;
  }
  // passing class pairs: (ma | mb) == keep (a == b: at least 2 clades)
  int U = 0;
  for (int base = 0; base < kSpCls; base += 64) {  // the occupied slots, compacted
    const int h = base + lane;
    const bool occ = sh.ckey[h] != ~0ull;
    const uint64_t w = __ballot(occ);
    if (occ) sh.cls[U + __popcll(w & below)] = h;
    U += __popcll(w);
  }
  __syncthreads();
  for (int ia = 0; ia < U; ++ia) {
    const int a = sh.cls[ia];
    const unsigned long long ma = sh.ckey[a];
    for (int ib = ia + lane; ib < U; ib += 64) {
      const int b = sh.cls[ib];
      if ((ma | sh.ckey[b]) != keep || (a == b && !sh.cmany[a])) continue;
      const int q = atomicAdd(&sh.n_pairs, 1);
      if (q < kSpPairs) sh.pair[q] = min(a, b) | (max(a, b) << 16);
      sh.cint[a] = 1;
      sh.cint[b] = 1;
    }
  }
  __syncthreads();
  BLAP(3);
  bool have_ok = false;
  if (sh.n_pairs > 0) {
    if (sh.n_pairs > kSpPairs) {
      BSTAT(17, 1);
      return false;
    }
    // ---- pass 3: members (potential clades of passing classes), counted per class -------
    int pbase = 0;
    sp_rows(S, sh, so, se, [&](bool st, int t, int w, int cl) {
      bool pot = false;
      SpRow r{0, 0, 0};
      if (st && !(vu && cl == K.unknown)) {
        r = sp_row(sh, P, w, cl, allg);
        pot = r.mk2 != 0ull;
      }
      const uint64_t pb = __ballot(pot);
      const int pi = pbase + __popcll(pb & below) + (u_pot && cl > K.unknown ? 1 : 0);
      pbase += __popcll(pb);
      if (pot) {
        const uint64_t cmask = r.mk2 & keep;
        int h = sp_hash(cmask, kSpCls);
        while (sh.ckey[h] != cmask) h = (h + 1) & (kSpCls - 1);
        if (sh.cint[h]) {
          const int q = atomicAdd(&sh.cnt, 1);
          atomicAdd(&sh.ccnt[h], 1);
          if (q < kSpMemG) {
            SpMember m;
            m.rs = t; m.cl = cl; m.pi = pi; m.sp = K.sibp[cl];
            m.h = h; m.pad = 0; m.hm = r.mhs;
            mem[q] = m;
          }
        }
      }
    });
    if (u_pot && lane == 0) {                        // the virtual "Unknown" row
      const uint64_t cmask = u_k2 & keep;
      int h = sp_hash(cmask, kSpCls);
      while (sh.ckey[h] != cmask) h = (h + 1) & (kSpCls - 1);
      if (sh.cint[h]) {
        const int q = atomicAdd(&sh.cnt, 1);
        atomicAdd(&sh.ccnt[h], 1);
        if (q < kSpMemG) {
          SpMember m;
          m.rs = -1; m.cl = K.unknown; m.pi = upi; m.sp = K.sibp[K.unknown];
          m.h = h; m.pad = 0; m.hm = u_hs;
          mem[q] = m;
        }
      }
    }
    __threadfence_block();
    __syncthreads();
    BLAP(4);
    const int M = sh.cnt;
    BSTAT(14, M);
    if (M > kSpMemG) return false;
    // members grouped by class (gidx), candidate counts per passing class pair
    if (lane == 0) {
      int acc = 0;
      for (int ia = 0; ia < U; ++ia) {
        const int a = sh.cls[ia];
        sh.coff[a] = acc;
        if (sh.cint[a]) acc += sh.ccnt[a];
      }
      int tot = 0;
      for (int q = 0; q < sh.n_pairs; ++q) {
        sh.pref[q] = tot;
        const int a = sh.pair[q] & 0xFFFF, b = sh.pair[q] >> 16;
        const long long n = a == b ? (long long)sh.ccnt[a] * (sh.ccnt[a] - 1) / 2
                                   : (long long)sh.ccnt[a] * sh.ccnt[b];
        tot = (int)min<long long>((long long)tot + n, 0x7FFFFFFF);
      }
      sh.pref[sh.n_pairs] = tot;
    }
    __syncthreads();
    if (sh.pref[sh.n_pairs] == 0x7FFFFFFF) return false;
    for (int q = lane; q < M; q += 64) {
      const int h = mem[q].h;
      gidx[sh.coff[h] + atomicAdd(&sh.cfill[h], 1)] = q;
    }
    // the members' dense rows (the pair evaluations then load a row's loci independently)
    const bool dense = (int64_t)M * G <= kSpDense;
    if (dense)
      for (int q = lane; q < M; q += 64) {
        const SpMember m = mem[q];
        double* row = drows + (int64_t)q * G;
        if (m.rs < 0) {
          for (int g = 0; g < G; ++g) row[g] = urow[g];
        } else {
          for (int g = 0; g < G; ++g) row[g] = 0.0;
          for (int t = m.rs; t < se; ++t) {
            const int2 cg = S.seg_cg[t];
            if (cg.x != m.cl) break;
            row[cg.y] = S.seg_mean[t];
          }
        }
      }
    const double* rows = dense ? drows : nullptr;     // (after pass 4: an LDS copy when it fits)
    auto acc = [&](int q, const SpMember& m) -> SpRowAcc {
      return SpRowAcc{rows ? rows + (int64_t)q * G : nullptr, SpCursor{m.rs, m.cl, se, m.rs < 0 ? urow : nullptr}};
    };
    __threadfence_block();
    __syncthreads();
    BLAP(5);
    // ---- pass 4: per parent of a member, clades listed under it scoring >= threshold ----
    int pcap = 64;
    while (pcap < 2 * M) pcap <<= 1;
    if (pcap <= kSpLPar) par = sh.lpar;              // (the class table is done with)
    if (P.sister_on) {
      for (int h = lane; h < pcap; h += 64) par[h].key = ~0ull;
      __threadfence_block();
      __syncthreads();
      for (int q = lane; q < M; q += 64) {             // the members' parents
        const int p = K.parent[mem[q].cl];
        for (int h = sp_hash((uint64_t)p, pcap);; h = (h + 1) & (pcap - 1)) {
          const unsigned long long old = atomicCAS(&par[h].key, ~0ull, (unsigned long long)p);
          if (old == ~0ull) { par[h].c1 = 0; par[h].c2 = 0; par[h].c3 = 0; }
          if (old == ~0ull || old == (unsigned long long)p) break;
        }
      }
      __threadfence_block();
      __syncthreads();
      auto count = [&](int sp, uint64_t hm) {
        const SpParent* e = sp >= 0 && hm ? sp_par_find(par, pcap, sp) : nullptr;
        if (!e) return;
        SpParent* x = const_cast<SpParent*>(e);
        const uint64_t o1 = atomicOr(&x->c1, (unsigned long long)hm);   // saturating count
        const uint64_t t2 = o1 & hm;
        if (t2) {
          const uint64_t o2 = atomicOr(&x->c2, (unsigned long long)t2);
          if (o2 & t2) atomicOr(&x->c3, (unsigned long long)(o2 & t2));
        }
      };
      // (each window's listed parents loaded at once: one round trip per window, not per chunk)
      sp_rows_pf(S, sh, so, se,
                 [&](bool st, int cl) { return st && !(vu && cl == K.unknown) ? K.sibp[cl] : -1; },
                 [&](bool, int, int w, int cl, int sp) {
                   if (sp < 0) return;
                   count(sp, sp_row(sh, P, w, cl, allg).mhs);
                 });
      if (vu && lane == 0) count(K.sibp[K.unknown], u_hs);
      __threadfence_block();
    }
    __syncthreads();
    // the segment window is done with: the members' dense rows move into it when they fit, so
    // the pair evaluations below read LDS instead of each taking dependent HBM round trips
    if (dense && M * G <= kSpLdsRows) {
      double* lrows = reinterpret_cast<double*>(sh.wcg);
      for (int i = lane; i < M * G; i += 64) lrows[i] = drows[i];
      __syncthreads();
      rows = lrows;
    }
    BLAP(6);

    // ---- pass 1 over the candidates: best by (rank, pair index) ------------------------
    double pr = -__builtin_inf();
    long long pk = -1;
    int pu = -1, pv = -1;
    sp_for_cands(sh, mem, gidx, [&](int u, int v, const SpMember& mu, const SpMember& mv) {
      const double r = sp_pair_rank(S, acc(u, mu), acc(v, mv), keep, Gu);
      const long long key = (long long)mu.pi * Pp + mv.pi;
      if (better(r, key, pr, pk)) { pr = r; pk = key; pu = u; pv = v; }
    });
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double r2 = __shfl_xor(pr, off, 64);
      const long long k2 = __shfl_xor(pk, off, 64);
      const int u2 = __shfl_xor(pu, off, 64), v2 = __shfl_xor(pv, off, 64);
      if (better(r2, k2, pr, pk)) { pr = r2; pk = k2; pu = u2; pv = v2; }
    }
    // a passing class pair has at least one candidate, so pk >= 0 here
    int best_ok = 0, best_dir = 0;
    int best_c1 = -1, best_c2 = -1;
    double best_crit = 0.0;
    if (lane == 0) {
      const SpMember A = mem[pu], B = mem[pv];
      const OptEval e = sp_eval_two(S, sh, A, B, acc(pu, A), acc(pv, B), par, pcap, G, ign, false, sh.syn);
      best_ok = e.ok; best_dir = e.dir;
      best_c1 = e.c1p ? pv : pu;
      best_c2 = e.c2p ? pv : pu;
      best_crit = sp_pair_crit(S, acc(pu, A), acc(pv, B), keep);
      sh.n_in = 0; sh.all_ok = 1; sh.all_same = 1;
    }
    for (int i = lane; i < kSpMemG / 32; i += 64) { bm1[i] = 0; bm2[i] = 0; }
    __threadfence_block();
    __syncthreads();
    BLAP(7);
    // ---- pass 2 over the candidates: options within --range get the LGT filters --------
    sp_for_cands(sh, mem, gidx, [&](int u, int v, const SpMember& mu, const SpMember& mv) {
      const SpRowAcc a = acc(u, mu), b = acc(v, mv);
      const double r = sp_pair_rank(S, a, b, keep, Gu);
      if (!((pr - r) <= P.range)) return;                       // (:636-639)
      const OptEval e = sp_eval_two(S, sh, mu, mv, a, b, par, pcap, G, ign, true, nullptr);
      atomicAdd(&sh.n_in, 1);
      if (!e.ok) atomicAnd(&sh.all_ok, 0);
      if (!e.same) atomicAnd(&sh.all_same, 0);
      const int q1 = e.c1p ? v : u, q2 = e.c2p ? v : u;
      atomicOr(&bm1[q1 >> 5], 1u << (q1 & 31));
      atomicOr(&bm2[q2 >> 5], 1u << (q2 & 31));
    });
    __threadfence_block();
    __syncthreads();
    BLAP(8);
    // ---- meld_two (:640-669) ----------------------------------------------------------------
    int kind;   // 0 none, 1 best as is, 2 meld, 3 unchecked best, 4 upstream crash
    const int n_in = sh.n_in;
    if (n_in == 0) kind = (P.dis2 == 0) ? 3 : (P.dis2 == 1 ? 0 : 4);   // --range < 0
    else if (n_in == 1 || P.dis2 == 0) kind = 1;
    else if (P.dis2 == 1) kind = 0;
    else kind = (sh.all_ok && sh.all_same) ? 2 : 0;
    if (kind == 4) {
      if (lane == 0) K.status[c] = WF_E_BADINPUT;
      return true;
    }
    int lca1 = -1, lca2v = -1, m1 = 0, m2 = 0;
    auto in_bm = [&](const unsigned* bm, int q) { return q < M && ((bm[q >> 5] >> (q & 31)) & 1u); };
    if (kind == 2) {
      // the melded clades' LCAs (utils.py:401-411)
      int a1 = -1, a2 = -1;
      for (int q = lane; q < M; q += 64) {
        if (in_bm(bm1, q)) { a1 = lca2(K, a1, mem[q].cl); ++m1; }
        if (in_bm(bm2, q)) { a2 = lca2(K, a2, mem[q].cl); ++m2; }
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        a1 = lca2(K, a1, __shfl_xor(a1, off, 64));
        a2 = lca2(K, a2, __shfl_xor(a2, off, 64));
        m1 += __shfl_xor(m1, off, 64);
        m2 += __shfl_xor(m2, off, 64);
      }
      lca1 = a1;
      lca2v = a2;
      bool keepit = true;
      if (!P.allow_lca) {
        const int nl = lca2(K, lca1, lca2v);
        keepit = !(nl == lca1 || nl == lca2v);
      }
      have_ok = keepit;   // melded options are all OK
    } else if (kind == 1) {
      have_ok = __shfl(best_ok, 0, 64) != 0;
    } else if (kind == 3) {
      have_ok = true;
    }
    if (have_ok) {
      if (lane < G) K.syn[l0 + lane] = sh.syn[lane];
      if (kind == 2) {                               // melded clades, in member order
        int o1 = 0, o2 = 0;
        for (int base = 0; base < M; base += 64) {
          const int q = base + lane;
          const bool in1 = in_bm(bm1, q), in2 = in_bm(bm2, q);
          const uint64_t w1 = __ballot(in1), w2 = __ballot(in2);
          if (in1) K.meld[mbase + o1 + __popcll(w1 & below)] = mem[q].cl;
          if (in2) K.meld[mbase + m1 + o2 + __popcll(w2 & below)] = mem[q].cl;
          o1 += __popcll(w1);
          o2 += __popcll(w2);
        }
      }
      if (lane == 0) {
        K.call[c] = WF_CALL_LGT;
        K.crit[c] = best_crit;
        K.rank[c] = pr;
        K.dir[c] = (int8_t)best_dir;
        K.c1[c] = (kind == 2) ? lca1 : mem[best_c1].cl;
        K.c2[c] = (kind == 2) ? lca2v : mem[best_c2].cl;
        K.nm1[c] = (kind == 2) ? m1 : 0;
        K.nm2[c] = (kind == 2) ? m2 : 0;
        K.iters[c] = (int16_t)iteration;
        K.pair_evals[c] = pair_evals;
      }
      BLAP(9);
      return true;
    }
  }
  const int dec = (no_rows || root_present) ? kDecStop : kDecRaise;
  if (dec == kDecRaise && iteration + 1 <= kMaxIter) {
    if (S.seed_pend) {                               // level 0 of the wave kernels: a staged
      if (lane == 0) {                               // level-1 seed (k_rekey_seeds rolls it up)
        S.seed_pend[c] = 2;
        K.pair_evals[c] = pair_evals;
      }
      return true;
    }
    sp_raise(S, c, pair_evals);                      // roll up (orgscorer.py:431-445)
    BLAP(9);
    return true;
  }
  if (lane == 0) {                                   // unclassified after evaluation
    const int it = dec == kDecRaise ? iteration + 1 : iteration;
    K.iters[c] = (int16_t)min(it, 32767);
    K.pair_evals[c] = pair_evals;
    K.status[c] = dec == kDecRaise ? WF_E_RUNAWAY : 0;
  }
  return true;
}

// ---- explain_two from the wave form's compact hand-over ---------------------------------
// sp_level's explain_two, LGT checks and meld_two (orgscorer.py:599-744) on the compact table
// the first wave form writes when passes 4 and 5 ran (<= 64 potential clades, <= 63 loci,
// wf_fast.hip): the potential clades' rows whole, plus every other segment at or above the
// sister threshold; the unmasked loci (the first form's weak-locus mask, :420-427) and
// whether r__Root is present come with it.  A segment left out either belongs to no
// potential clade and scores below the threshold (it enters no test), or was never
// evaluated because its mean cannot reach one (the prune2d comment in k_wave).
//
// The table is staged in LDS once; potential clade i (clade order) gets a row of summaries
// (loci present, ">= k2 on unmasked loci", ">= the sister threshold"), and its gene scores
// are read from its run (locus g is segment t + popcount(present loci below g), 0.0 without
// a segment).  The sister checks (:717-744) use, per potential clade X, the loci where at
// least one / two clades listed under parent(X), X excluded, score at or above the
// threshold: the pair's other clade is removed with one bit operation (sp_sisters'
// saturating counts, restated for one parent per clade).
struct E2Shared {
  union {                                    // (9,920 bytes in all: 16 waves per CU)
    struct {                                 // the scans of the table ...
      int2 cg[kE2Seg];                       // (clade, locus), clade then locus order
      unsigned long long pm[64];             // potential clade i: ">= k2" on unmasked loci
    };
    unsigned short cand[64 * 63 / 2];        // ... then the candidate pairs i | j << 8 (i < j)
  };
  double v[kE2Seg];                          // gene score
  int t[64], cl[64], par[64], sibp[64];      // potential clade i: run start, clade, parent,
                                             // listed parent
  unsigned long long pres[64], hm[64], s1[64], s2[64];
  int len[64];                               // locus lengths (ambiguous fraction)
};

// S[row][g] (0.0 without a segment)
__device__ __forceinline__ double e2_at(const E2Shared& sh, int t, uint64_t pres, int g) {
  return ((pres >> g) & 1ull) ? sh.v[t + __popcll(pres & ((1ull << g) - 1ull))] : 0.0;
}

// Contig.score(c1, c2) rank (orgscorer.py:447-461): numpy-order mean over the unmasked loci
// of the per-locus max (sp_pair_rank's arithmetic)
__device__ __forceinline__ double e2_rank(const E2Shared& sh, int a, int b, uint64_t um, int Gu) {
  const int ta = sh.t[a], tb = sh.t[b];
  const uint64_t pa = sh.pres[a], pb = sh.pres[b];
  uint64_t m = um;
  auto next = [&]() -> double {
    const int g = __builtin_ctzll(m);
    m &= m - 1;
    const double x = e2_at(sh, ta, pa, g), y = e2_at(sh, tb, pb, g);
    return x < y ? y : x;
  };
  return (0.0 + np_sum_seq(Gu, next)) / (double)Gu;
}

struct E2Eval {
  int ok, swapped, dir;
  uint64_t mm, mA, mB;                       // synteny '*', 'A', 'B' after the swap
};

// set_synteny_two + apply_lgt_checks (orgscorer.py:511-545, 678-744) for potential clades
// a < b: sp_eval_two's arithmetic
__device__ __forceinline__ E2Eval e2_eval(const KArgs& K, const E2Shared& sh, int a, int b, uint64_t um) {
  const DevParams& P = K.p;
  const bool unk = sh.cl[a] == K.unknown || sh.cl[b] == K.unknown;
  uint64_t mm = 0, ma = 0, mb = 0;
  {
    const int ta = sh.t[a], tb = sh.t[b];
    const uint64_t pa = sh.pres[a], pb = sh.pres[b];
    for (uint64_t r = um; r; r &= r - 1) {
      const int g = __builtin_ctzll(r);
      const uint64_t bit = 1ull << g;
      const double s1 = e2_at(sh, ta, pa, g), s2 = e2_at(sh, tb, pb, g);
      const double mn = s2 < s1 ? s2 : s1;
      if (mn >= P.k_amb && !unk) mm |= bit;
      else if (s1 >= P.k2) ma |= bit;
      else if (s2 >= P.k2) mb |= bit;
    }
  }
  E2Eval e;
  const uint64_t ab = ma | mb;                       // "^[^A]*B" -> swap (:537-540)
  e.swapped = (ab && ((mb >> __builtin_ctzll(ab)) & 1ull)) ? 1 : 0;
  e.mm = mm;
  e.mA = e.swapped ? mb : ma;
  e.mB = e.swapped ? ma : mb;
  int64_t tot = 0, amb = 0;
  int state = 0;
  bool dir_ok = true;
  for (uint64_t r = um; r; r &= r - 1) {             // "^A+B+A+$" without '~' (:542)
    const int g = __builtin_ctzll(r);
    const uint64_t bit = 1ull << g;
    const char c = (mm & bit) ? '*' : (e.mA & bit) ? 'A' : (e.mB & bit) ? 'B' : '!';
    if (c != '!') {
      tot += sh.len[g];
      if (c == '*') amb += sh.len[g];
    }
    if (state == 0) { if (c == 'A') state = 1; else dir_ok = false; }
    else if (state == 1) { if (c == 'B') state = 2; else if (c != 'A') dir_ok = false; }
    else if (state == 2) { if (c == 'A') state = 3; else if (c != 'B') dir_ok = false; }
    else { if (c != 'A') dir_ok = false; }
  }
  e.dir = (dir_ok && state == 3) ? 1 : 0;
  e.ok = 1;
  if ((double)amb / (double)tot > P.amb_frac) e.ok = 0;                       // :693-702
  if (P.clade_genes >= 0 && min(__popcll(e.mA), __popcll(e.mB)) < P.clade_genes) e.ok = 0;   // :704-708
  const int x = e.swapped ? b : a, y = e.swapped ? a : b;   // clade1 / clade2 after the swap
  if (P.clade_leaves >= 0) {                         // :710-715 (recip = clade2 when B>A)
    const int64_t ly = K.leaves[sh.cl[y]];
    const int64_t lc = e.dir ? ly : min(K.leaves[sh.cl[x]], ly);
    if (lc < P.clade_leaves) e.ok = 0;
  }
  if (P.sister_on && e.ok) {                         // :717-744
    // sisters["B"] = get_sisters(clade1) - {clade2}; sisters["A"] = get_sisters(clade2) - {clade1}
    const int px = sh.par[x], py = sh.par[y];
    const uint64_t fb = sh.sibp[y] == px ? (sh.s2[x] | (sh.s1[x] & ~sh.hm[y])) : sh.s1[x];
    uint64_t fa = 0;
    if (!e.dir) fa = sh.sibp[x] == py ? (sh.s2[y] | (sh.s1[y] & ~sh.hm[x])) : sh.s1[y];
    if ((fb & e.mB) || (fa & e.mA)) e.ok = 0;
  }
  return e;
}

__device__ __forceinline__ int e2_wave_lca(const KArgs& K, int acc) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc = lca2(K, acc, __shfl_xor(acc, off, 64));
  return acc;
}

// One compact slot (table [so, se), contig c, the roll-up level): writes the contig's
// result or its roll-up bookkeeping (as sp_level).  False: the table breaks the compact
// form's limits (the dense decision takes the contig; never expected).
// (h0, l0, G: the contig's hit and locus offsets and locus count, loaded with the slot)
__device__ __forceinline__ bool sp_two(const SArgs& S, E2Shared& sh, int c, int so, int se, uint64_t hdr,
                                       int64_t h0, int64_t l0, int G, int level) {
  const KArgs& K = S.k;
  const DevParams& P = K.p;
  const int lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1ull;
  const int ns = se - so;
  if (G > kE2MaxG || ns > kE2Seg) return false;
  SLAP_MARK(c);
  SSTAT(8, 1);
  SSTAT(9, ns);
  const uint64_t um = hdr & ~(1ull << 63);
  const bool root = (hdr >> 63) != 0ull;
  const int Gu = __popcll(um);
  const uint64_t allG = (1ull << G) - 1ull;
  const int iteration = level + 1;
  int64_t pair_evals = level == 0 ? 0 : K.pair_evals[c];
  // Global loads in two rounds for the whole table (not one round trip per 64 segments):
  // the table and the loci, then the parents / listed parents of the clades it names.
  constexpr int kCh = kE2Seg / 64;
  {
    int2 cgr[kCh];
    double vr[kCh];
#pragma unroll
    for (int k = 0; k < kCh; ++k) {
      const int q = 64 * k + lane;
      cgr[k] = make_int2(-1, 0);
      vr[k] = 0.0;
      if (q < ns) {
        cgr[k] = S.dump_cg[so + q];
        vr[k] = S.dump_mean[so + q];
      }
    }
    int ln = 0;
    if (lane < G) {
      const int ls = K.lstart[l0 + lane], le = K.lend[l0 + lane];
      ln = max(ls, le) - min(ls, le) + 1;
    }
#pragma unroll
    for (int k = 0; k < kCh; ++k) {
      const int q = 64 * k + lane;
      if (q < ns) {
        sh.cg[q] = cgr[k];
        sh.v[q] = vr[k];
      }
    }
    if (lane < G) sh.len[lane] = ln;
  }
  __syncthreads();
  SLAP(0);
  // clade runs (one per run head): potential clades (a locus >= k2, missing loci scoring
  // 0.0; :603-605) and, for the sister checks, the loci at or above the threshold
  int Pp = 0;
  int hcl[kCh];
  uint64_t hh[kCh];
#pragma unroll
  for (int k = 0; k < kCh; ++k) {
    const int t = 64 * k + lane;
    bool pot = false;
    uint64_t pres = 0, mk2 = 0, hm = 0;
    int cl = -1;
    if (t < ns) {
      cl = sh.cg[t].x;
      if (t == 0 || sh.cg[t - 1].x != cl) {
        for (int q = t; q < ns && sh.cg[q].x == cl; ++q) {
          const uint64_t bit = 1ull << sh.cg[q].y;
          const double x = sh.v[q];
          pres |= bit;
          if (x >= P.k2) mk2 |= bit;
          if (x >= P.sister_thr) hm |= bit;
        }
        const uint64_t miss = allG & ~pres;
        if (0.0 >= P.k2) mk2 |= miss;
        if (0.0 >= P.sister_thr) hm |= miss;
        pot = mk2 != 0ull;
      } else {
        cl = -1;                                       // (not a run head)
      }
    }
    hcl[k] = cl;
    hh[k] = hm;
    const uint64_t pb = __ballot(pot);
    const int i = Pp + __popcll(pb & below);
    if (pot && i < 64) {
      sh.t[i] = t; sh.cl[i] = cl;
      sh.pres[i] = pres; sh.pm[i] = mk2 & um; sh.hm[i] = hm; sh.s1[i] = 0; sh.s2[i] = 0;
    }
    Pp += __popcll(pb);
  }
  if (Pp > 64) return false;
  __syncthreads();
  SLAP(1);
  SSTAT(10, Pp);
  const uint64_t my_pm = lane < Pp ? sh.pm[lane] : 0ull;   // (cand overwrites pm and cg)
  pair_evals += (int64_t)Pp * (Pp - 1) / 2;
  if (lane == 0) note_ppot(K, c, iteration, Pp);
  // the candidate pairs, crit >= k2 <=> (m_i | m_j) == um, listed so that their ranks are
  // taken 64 at a time (one pair per lane): the Pp (Pp - 1) / 2 pairs are tested 64 at a
  // time too, pair p = j (j - 1) / 2 + i (i < j) on lane p mod 64, the two masks fetched
  // from lanes i and j (the list order does not matter: pass 1 selects by (rank, pair
  // index), pass 2 only aggregates)
  __syncthreads();                                   // (every read of cg and pm done)
  int nc = 0;
  const int n_pairs = Pp * (Pp - 1) / 2;
  for (int p0 = 0; p0 < n_pairs; p0 += 64) {
    const int p = min(p0 + lane, n_pairs - 1);
    int j = (int)((1.0f + __fsqrt_rn(1.0f + 8.0f * (float)p)) * 0.5f);
    j -= j * (j - 1) / 2 > p ? 1 : 0;                 // (float rounding at the row ends)
    j += (j + 1) * j / 2 <= p ? 1 : 0;
    const int i = p - j * (j - 1) / 2;
    const uint64_t mi = (uint64_t)__shfl((long long)my_pm, i, 64), mj = (uint64_t)__shfl((long long)my_pm, j, 64);
    const bool cand = p0 + lane < n_pairs && (mi | mj) == um;
    const uint64_t cb = __ballot(cand);
    if (cand) sh.cand[nc + __popcll(cb & below)] = (unsigned short)(i | (j << 8));
    nc += __popcll(cb);
  }
  __syncthreads();
  // the potential clades in some candidate pair: the only ones whose parent, listed parent
  // and sister masks the LGT checks read (e2_eval)
  uint64_t memb = 0;
  for (int q = lane; q < nc; q += 64) memb |= (1ull << (sh.cand[q] & 0xFF)) | (1ull << (sh.cand[q] >> 8));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) memb |= (uint64_t)__shfl_xor((long long)memb, off, 64);
  SLAP(2);
  SSTAT(11, nc);
  if (P.sister_on && memb) {
    const bool me = (memb >> lane) & 1ull;
    const int my_cl = me ? sh.cl[lane] : -1;
    const int my_par = me ? K.parent[my_cl] : -2;
    if (me) {
      sh.par[lane] = my_par;
      sh.sibp[lane] = K.sibp[my_cl];
    }
    int hsp[kCh];                                      // listed parents of the runs' clades
#pragma unroll
    for (int k = 0; k < kCh; ++k) hsp[k] = (hcl[k] >= 0 && hh[k] != 0ull) ? K.sibp[hcl[k]] : -1;
    // per member, the present clades listed under its parent (itself excluded) at or above
    // the threshold (a segment left out of the table scores below it)
    uint64_t s1 = 0, s2 = 0;
#pragma unroll
    for (int k = 0; k < kCh; ++k) {
      if (64 * k >= ns) break;
      const int sp = hsp[k], cl = hcl[k];
      const uint64_t h = hh[k];
      bool match = false;
      for (uint64_t r = memb; r; r &= r - 1) match = match || (sp >= 0 && sp == lane_bcast(my_par, __builtin_ctzll(r)));
      for (uint64_t mb = __ballot(match); mb; mb &= mb - 1) {
        const int src = __builtin_ctzll(mb);
        const int sp_r = lane_bcast(sp, src), cl_r = lane_bcast(cl, src);
        const uint64_t h_r = lane_bcast(h, src);
        if (my_par == sp_r && my_cl != cl_r) {
          s2 |= s1 & h_r;
          s1 |= h_r;
        }
      }
    }
    if (me) { sh.s1[lane] = s1; sh.s2[lane] = s2; }
    __syncthreads();
  }
  SLAP(3);
  // pass 1: the best candidate pair by (rank, pair index)
  double pr = -__builtin_inf();
  long long pk = -1;
  if (nc > 0) {
    for (int q = lane; q < nc; q += 64) {
      const int i = sh.cand[q] & 0xFF, j = sh.cand[q] >> 8;
      const double r = e2_rank(sh, i, j, um, Gu);
      const long long key = (long long)i * Pp + j;
      if (better(r, key, pr, pk)) { pr = r; pk = key; }
    }
    each_stride([&](auto J) {
      constexpr int js = decltype(J)::value;
      const double r2 = xor_lanes<js>(pr);
      const long long k2 = xor_lanes<js>(pk);
      if (better(r2, k2, pr, pk)) { pr = r2; pk = k2; }
    });
  }
  SLAP(4);
  if (pk >= 0) {
    const int bi = (int)(pk / Pp), bj = (int)(pk % Pp);
    const E2Eval be = e2_eval(K, sh, bi, bj, um);
    // pass 2: options within --range of the best get the LGT checks (:636-639)
    int n_in = 0;
    bool all_ok = true, all_same = true;
    uint64_t b1 = 0, b2 = 0;
    for (int q = lane; q < nc; q += 64) {
      const int i = sh.cand[q] & 0xFF, j = sh.cand[q] >> 8;
      if ((pr - e2_rank(sh, i, j, um, Gu)) <= P.range) {
        const E2Eval e = e2_eval(K, sh, i, j, um);
        ++n_in;
        all_ok = all_ok && e.ok;
        all_same = all_same && e.mm == be.mm && e.mA == be.mA && e.mB == be.mB;
        b1 |= 1ull << (e.swapped ? j : i);
        b2 |= 1ull << (e.swapped ? i : j);
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      n_in += __shfl_xor(n_in, off, 64);
      b1 |= (uint64_t)__shfl_xor((long long)b1, off, 64);
      b2 |= (uint64_t)__shfl_xor((long long)b2, off, 64);
    }
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
      return true;
    }
    bool have_ok = false;
    int lca1 = -1, lca2v = -1;
    const bool in1 = (b1 >> lane) & 1ull, in2 = (b2 >> lane) & 1ull;
    const int my_cl = lane < Pp ? sh.cl[lane] : -1;
    if (kind == 2) {
      lca1 = e2_wave_lca(K, in1 ? my_cl : -1);
      lca2v = e2_wave_lca(K, in2 ? my_cl : -1);
      bool keep = true;
      if (!P.allow_lca) {
        const int nl = lca2(K, lca1, lca2v);
        keep = !(nl == lca1 || nl == lca2v);
      }
      have_ok = keep;                                // melded options are all OK
    } else if (kind == 1) {
      have_ok = be.ok != 0;
    } else if (kind == 3) {
      have_ok = true;
    }
    if (have_ok) {
      const int64_t mbase = 2 * h0 + 2 * (int64_t)c;
      const int m1 = __popcll(b1), m2 = __popcll(b2);
      if (kind == 2) {                               // melded clades, in potential order
        if (in1) K.meld[mbase + __popcll(b1 & below)] = my_cl;
        if (in2) K.meld[mbase + m1 + __popcll(b2 & below)] = my_cl;
      }
      if (lane < G) {
        const uint64_t bit = 1ull << lane;
        K.syn[l0 + lane] = !(um & bit) ? '~' : (be.mm & bit) ? '*' : (be.mA & bit) ? 'A' : (be.mB & bit) ? 'B' : '!';
      }
      if (lane == 0) {
        double bcrit = 0.0;                          // sp_pair_crit: min over the unmasked loci
        bool first = true;
        const int ta = sh.t[bi], tb = sh.t[bj];
        const uint64_t pa = sh.pres[bi], pb = sh.pres[bj];
        for (uint64_t r = um; r; r &= r - 1) {
          const int g = __builtin_ctzll(r);
          const double x = e2_at(sh, ta, pa, g), y = e2_at(sh, tb, pb, g);
          const double m = x < y ? y : x;
          bcrit = (first || m < bcrit) ? m : bcrit;
          first = false;
        }
        K.call[c] = WF_CALL_LGT;
        K.crit[c] = bcrit;
        K.rank[c] = pr;
        K.dir[c] = (int8_t)be.dir;
        K.c1[c] = kind == 2 ? lca1 : sh.cl[be.swapped ? bj : bi];
        K.c2[c] = kind == 2 ? lca2v : sh.cl[be.swapped ? bi : bj];
        K.nm1[c] = kind == 2 ? m1 : 0;
        K.nm2[c] = kind == 2 ? m2 : 0;
        K.iters[c] = (int16_t)iteration;
        K.pair_evals[c] = pair_evals;
      }
      SLAP(5);
      return true;
    }
  }
  SLAP(5);
  // no explanation at this level (:570-583): raise, or stop at r__Root (the table is never
  // empty: explain_one ran on this contig's segments)
  if (!root && iteration + 1 <= kMaxIter) {
    if (lane == 0) {
      S.seed_pend[c] = 2;
      K.pair_evals[c] = pair_evals;
    }
    return true;
  }
  if (lane == 0) {                                   // unclassified after evaluation
    K.iters[c] = (int16_t)min(root ? iteration : iteration + 1, 32767);
    K.pair_evals[c] = pair_evals;
    K.status[c] = root ? 0 : WF_E_RUNAWAY;
  }
  return true;
}

// The contigs whose dense decision state outgrew the LDS arena (big_list, counters[2]):
// one wave each with kSpSlot bytes of HBM scratch (S.sp_ws); the ones sp_level declines go
// to big2_list (counters[1]) for k_decide_big.
// S_arg stays the first parameter: the loop body re-reads the argument block through
// kernarg_fresh (wf_device.h) per contig -- held across the loop, its fields overflowed the
// SGPR file (309 SGPRs spilled to VGPR lanes: a v_readlane per use, the kernel's SALU excess).
__global__ __launch_bounds__(64, 4) void k_big_sparse(const SArgs S_arg, int level, int64_t n_keys) {
  __shared__ SpShared sh;
  char* ws = S_arg.sp_ws + (int64_t)blockIdx.x * kSpSlot;
  const int count = (int)S_arg.counters[2];
  for (int i = blockIdx.x; i < count; i += gridDim.x) {
    const SArgs& S = kernarg_fresh<SArgs>(S_arg);
    const int cr = S.big_list[2 * i], c = S.big_list[2 * i + 1];
    const bool ok = sp_level(S, sh, ws, c, cr, level, n_keys);
    if (!ok && threadIdx.x == 0) {
      const int slot = (int)atomicAdd(&S.counters[1], 1ull);
      S.big2_list[2 * slot] = cr;
      S.big2_list[2 * slot + 1] = c;
    }
    __syncthreads();
  }
}

// Level 0 of the contigs the first wave form handed over with their segment tables
// (S.dump_*: slot i holds entries [dump_first[i], dump_first[i + 1]) of contig
// dump_list[2 i + 1], dump_list[2 i] its form: 1 compact (explain_two only, sp_two), 0 the
// whole table (sp_level)).  S.seed_pend / ccnt / cleaves: decided -> pend 0 and no staged
// attachments; raised -> pend 2 (level-1 seed); declined (> 63 loci, class or pair tables
// outgrown) -> pend 1, the staged kernels take level 0.
//
// Wave levels (S.roll_next set): level `level` of the contigs the first form handed over at
// that level; a raised contig is appended to the next level's list.  The compact kernel
// (launched first) also sets up the next level: its table counter (S.dump_ctr_next) and the
// ancestors one level up (S.anc: parent^(jump + level + 1) of every name; k_wave of this
// level is done with them, and neither decision body reads them).
//
// KIND 1 takes the compact slots, KIND 0 the whole tables: two kernels, so that sp_two's
// smaller register file gives it twice the resident waves of sp_level.  A wave reads the
// headers of 64 of its slots (stride gridDim.x, as one slot per step would) at once.
// (S_arg first: the per-contig loop re-reads the argument block through kernarg_fresh, as
// k_big_sparse)
template <int KIND>
__global__ __launch_bounds__(64, KIND ? 4 : 2) void k_dump_sparse(const SArgs S_arg, int64_t* ccnt, int64_t* cleaves,
                                                                  int level) {
  using Sh = typename std::conditional<KIND == 1, E2Shared, SpShared>::type;
  __shared__ Sh sh;
  const int lane = threadIdx.x & 63;
  const SArgs& S0 = S_arg;
  if (KIND == 1) {
    if (S0.dump_ctr_next && blockIdx.x == 0 && lane == 0) *S0.dump_ctr_next = 0ull;
    if (S0.anc) {
      const int up = level == 0 ? S0.k.p.jump + 1 : 1;
      for (int t = blockIdx.x * 64 + lane; t < S0.n_tax; t += gridDim.x * 64) {
        int x = level == 0 ? t : S0.anc[t];
        for (int j = 0; j < up; ++j) x = S0.k.parent[x];
        S0.anc[t] = x;
      }
    }
  }
  char* ws = KIND ? nullptr : S0.sp_ws + (int64_t)blockIdx.x * kSpSlot;
  const int count = (int)(*S0.dump_ctr >> 40);
  const int stride = (int)gridDim.x;
  // a decided contig's pend / counts, a raised one onto the next level's list, a declined one
  // back to the staged kernels
  auto finish = [&](const SArgs& S, int c, bool ok) {
    if (lane == 0) {
      const int pd = S.seed_pend[c];
      if (!ok) {
        S.seed_pend[c] = 1;
        if (S.fail_ctr) atomicAdd(S.fail_ctr, 1ull);
      } else if (pd == 3) {
        S.seed_pend[c] = 0;
        ccnt[c] = 0;
        cleaves[c] = 0;
      } else if (pd == 2 && S.roll_next) {
        S.roll_next[atomicAdd(S.roll_next_n, 1ull)] = c;
      }
    }
    __syncthreads();
  };
  for (int base = blockIdx.x; base < count; base += 64 * stride) {
    const int my = base + lane * stride;
    int mc = -1, so = 0, se = 0, G = 0;
    uint64_t hdr = 0;
    int64_t h0 = 0, l0 = 0;
    if (my < count) {
      const int2 dl = reinterpret_cast<const int2*>(S0.dump_list)[my];
      if (dl.x == KIND && dl.y >= 0) {               // (c < 0: its table did not fit, pend 1 stands)
        mc = dl.y;
        if (KIND == 1) {
          so = S0.dump_first[my];
          se = S0.dump_first[my + 1];
          hdr = S0.dump_um[my];
          h0 = S0.k.hit_off[mc];
          l0 = S0.k.loc_off[mc];
          G = (int)(S0.k.loc_off[mc + 1] - l0);
        }
      }
    }
    for (uint64_t m = __ballot(mc >= 0); m; m &= m - 1) {
      const SArgs& S = kernarg_fresh<SArgs>(S_arg);
      const int src = __builtin_ctzll(m);
      const int c = lane_bcast(mc, src);
      bool ok;
      if constexpr (KIND == 1) {
        ok = sp_two(S, sh, c, lane_bcast(so, src), lane_bcast(se, src), lane_bcast(hdr, src),
                    (int64_t)lane_bcast((uint64_t)h0, src), (int64_t)lane_bcast((uint64_t)l0, src),
                    lane_bcast(G, src), level);
      } else {
        ok = sp_level(S, sh, ws, c, base + src * stride, level, 1);
      }
      finish(S, c, ok);
    }
  }
}
