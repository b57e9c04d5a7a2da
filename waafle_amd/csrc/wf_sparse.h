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
//           classes that pass with some class hold the only clades that can form an option
//   pass 3  row-parallel: those clades ("members": potential index, run start, mask,
//           sister mask) into LDS
//   pass 4  row-parallel, --sister-penalty on: for every parent of a member, the OR of the
//           sister masks (score >= threshold, :717-744) of the present clades listed under
//           it that are not members; member sisters are added per pair (the pair itself is
//           excluded, as get_sisters(clade1) - {clade2} does)
//   pairs   member pairs whose masks pass: rank (numpy order), best by (rank, pair index),
//           eval_two and meld_two exactly as decide_two, rows read from the runs
//
// A contig whose classes, members or member parents outgrow the LDS tables, with > 63 loci
// or with --weak-loci assign-unknown goes on to the dense decision (k_decide_big) instead.
constexpr int kSpCls = 256;      // mask-class hash slots
constexpr int kSpMem = 256;      // member clades
constexpr int kSpPar = 128;      // parents of member clades
constexpr int kSpMaxG = 63;      // loci per contig (mask bits; ~0 marks an empty class slot)

struct SpShared {
  unsigned long long mx[64];                 // per-locus max score bits (known clades)
  unsigned long long ckey[kSpCls];           // class mask (~0: empty)
  int ccnt[kSpCls];                          // potential clades in the class
  int cint[kSpCls];                          // class passes with some class
  int cls[kSpCls];                           // occupied slots, compacted
  unsigned long long mmask[kSpMem], mhm[kSpMem];
  int mrs[kSpMem], mcl[kSpMem], mpi[kSpMem], msp[kSpMem];
  int pkey[kSpPar];
  unsigned long long por[kSpPar];
  double row[64];                            // one dense row (explain_one's best)
  int len[64];                               // locus lengths (ambiguous fraction)
  uint8_t syn[64];                           // best option's synteny
  unsigned bm1[kSpMem / 32], bm2[kSpMem / 32];
  int n_used, n_mem, n_par, n_in, all_ok, all_same, cnt;
};

// Value of clade run `cl` at locus g (0 without a segment); calls in ascending g.
struct SpCursor {
  int t, cl, se;
  __device__ __forceinline__ double at(const SArgs& S, int g) {
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

// Bit summary of one clade run: loci at or above k1 / k2 / the sister threshold (a locus
// without a segment scores 0.0 and is compared as such).
struct SpRow {
  uint64_t mk1, mk2, mhs;
};

__device__ __forceinline__ SpRow sp_row(const SArgs& S, const DevParams& P, int rs, int se, int cl,
                                        uint64_t allg) {
  uint64_t cov = 0, k1 = 0, k2 = 0, hs = 0;
  for (int t = rs; t < se; ++t) {
    const int2 cg = S.seg_cg[t];
    if (cg.x != cl) break;
    const double v = S.seg_mean[t];
    const uint64_t bit = 1ull << cg.y;
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

// Runs of the contig's segments [so, se) in clade order, one per lane: f(is_start, t, clade)
// is called by every lane of the wave for each 64-segment chunk (is_start false on lanes
// that hold no run start), so f may use wave operations.
template <class F>
__device__ __forceinline__ void sp_rows(const SArgs& S, int so, int se, F f) {
  const int lane = threadIdx.x & 63;
  int carry = -1;
  for (int base = so; base < se; base += 64) {
    const int t = base + lane;
    const int cl = t < se ? S.seg_cg[t].x : -2;
    int prev = __shfl_up(cl, 1, 64);
    if (lane == 0) prev = carry;
    carry = __shfl(cl, 63, 64);
    f(t < se && cl != prev, t, cl);
  }
}

// (rank, crit) of a clade pair over the kept loci: numpy-order mean and min of the
// per-locus max (orgscorer.py:447-461).
__device__ __forceinline__ double sp_pair_rank(const SArgs& S, int ra, int ca, int rb, int cb, int se,
                                               uint64_t keep, int Gu) {
  SpCursor a{ra, ca, se}, b{rb, cb, se};
  uint64_t m = keep;
  auto next = [&]() -> double {
    const int g = __builtin_ctzll(m);
    m &= m - 1;
    const double x = a.at(S, g), y = b.at(S, g);
    return x < y ? y : x;
  };
  return (0.0 + np_sum_seq(Gu, next)) / (double)Gu;
}

__device__ __forceinline__ double sp_pair_crit(const SArgs& S, int ra, int ca, int rb, int cb, int se,
                                               uint64_t keep) {
  SpCursor a{ra, ca, se}, b{rb, cb, se};
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

__device__ __forceinline__ int sp_par_slot(const SpShared& sh, int p) {
  for (int i = 0; i < sh.n_par; ++i)
    if (sh.pkey[i] == p) return i;
  return -1;
}

// eval_two (wf_device.h, G <= 64 form) for members u, v (u's potential index < v's): the
// synteny masks from the two runs, swap rule, direction, LGT filters, sister penalty.
__device__ __forceinline__ OptEval sp_eval_two(const SArgs& S, const SpShared& sh, int u, int v, int se,
                                               int G, uint64_t ign, bool cmp, uint8_t* out, int& same) {
  const KArgs& K = S.k;
  const DevParams& P = K.p;
  const int ca = sh.mcl[u], cb = sh.mcl[v];
  const bool unk = ca == K.unknown || cb == K.unknown;
  SpCursor a{sh.mrs[u], ca, se}, b{sh.mrs[v], cb, se};
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
  same = 1;
  int64_t tot = 0, amb = 0;
  int state = 0;
  bool dir_ok = true;
  for (int g = 0; g < G; ++g) {
    const uint64_t bit = 1ull << g;
    const uint8_t c = (ign & bit) ? '~' : (mm & bit) ? '*' : (mA & bit) ? 'A' : (mB & bit) ? 'B' : '!';
    if (out) out[g] = c;
    if (cmp && sh.syn[g] != c) same = 0;
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
  e.c1p = e.swapped ? v : u;                       // member slots
  e.c2p = e.swapped ? u : v;
  e.same = same;
  e.ok = 1;
  if ((double)amb / (double)tot > P.amb_frac) e.ok = 0;           // :693-702
  if (P.clade_genes >= 0 && min(nA, nB) < P.clade_genes) e.ok = 0; // :704-708
  const int X = sh.mcl[e.c1p], Y = sh.mcl[e.c2p];
  if (P.clade_leaves >= 0) {                                       // :710-715
    const int64_t lc = e.dir ? K.leaves[Y] : min(K.leaves[X], K.leaves[Y]);
    if (lc < P.clade_leaves) e.ok = 0;
  }
  if (P.sister_on && e.ok) {                                       // :717-744
    const int px = K.parent[X], py = K.parent[Y];
    const int sx = sp_par_slot(sh, px), sy = sp_par_slot(sh, py);
    uint64_t fb = sx >= 0 ? sh.por[sx] : 0ull, fa = sy >= 0 ? sh.por[sy] : 0ull;
    for (int q = 0; q < sh.n_mem; ++q) {
      const int sp = sh.msp[q];
      if (sp != px && sp != py) continue;
      const int s = sh.mcl[q];
      if (s == X || s == Y) continue;
      if (sp == px) fb |= sh.mhm[q];
      if (sp == py) fa |= sh.mhm[q];
    }
    if ((fb & mB) || (!e.dir && (fa & mA))) e.ok = 0;
  }
  return e;
}

// Member pairs (u, v), u < v in potential order, whose masks pass: f(u, v, i, j) on the lane
// that owns the pair (i, j: potential indices, i < j).
template <class F>
__device__ __forceinline__ void sp_for_pairs(const SpShared& sh, uint64_t keep, F f) {
  const int lane = threadIdx.x & 63;
  const int M = sh.n_mem;
  for (int a = 0; a < M - 1; ++a) {
    const uint64_t ma = sh.mmask[a];
    const int pa = sh.mpi[a];
    for (int b = a + 1 + lane; b < M; b += 64) {
      if ((ma | sh.mmask[b]) != keep) continue;
      const int pb = sh.mpi[b];
      if (pa < pb) f(a, b, pa, pb);
      else f(b, a, pb, pa);
    }
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
__device__ __forceinline__ bool sp_level(const SArgs& S, SpShared& sh, int c, int cr, int level, int64_t n_keys) {
  const KArgs& K = S.k;
  const DevParams& P = K.p;
  const int lane = threadIdx.x & 63;
  const int64_t h0 = K.hit_off[c];
  const int64_t l0 = K.loc_off[c];
  const int G = (int)(K.loc_off[c + 1] - l0);
  if (K.hit_off[c + 1] == h0 || G == 0) return true;   // never evaluated (orgscorer.py:959)
  if (G > kSpMaxG || P.weak == 2) return false;
  const int so = n_keys > 0 ? S.crank_first[cr] : 0;
  const int se = n_keys > 0 ? S.crank_first[cr + 1] : 0;
  const uint64_t allg = (1ull << G) - 1ull;
  const int64_t mbase = 2 * h0 + 2 * (int64_t)c;
  const int iteration = level + 1;
  int64_t pair_evals = level == 0 ? 0 : K.pair_evals[c];

  // ---- pass 1: per-locus maxes over known clades, root present (:407-411) -------------
  sh.mx[lane] = 0;
  if (lane < G) {
    const int ls = K.lstart[l0 + lane], le = K.lend[l0 + lane];
    sh.len[lane] = max(ls, le) - min(ls, le) + 1;
  }
  for (int i = lane; i < kSpCls; i += 64) { sh.ckey[i] = ~0ull; sh.ccnt[i] = 0; sh.cint[i] = 0; }
  if (lane == 0) { sh.n_used = 0; sh.n_mem = 0; sh.n_par = 0; sh.cnt = 0; }
  __syncthreads();
  bool root = false;
  for (int t = so + lane; t < se; t += 64) {
    const int2 cg = S.seg_cg[t];
    const double v = S.seg_mean[t];
    root |= cg.x == K.root;
    if (cg.x != K.unknown && v > 0.0) atomicMax(&sh.mx[cg.y], dbits(v));
  }
  const bool root_present = __ballot(root) != 0ull;
  __syncthreads();
  // weak loci: ignore -> mask (:420-427), penalize -> none (:413-414)
  const double mxv = __longlong_as_double((long long)sh.mx[lane]);
  const uint64_t keep = __ballot(lane < G && (P.weak != 0 || mxv >= P.kmin));
  const uint64_t ign = allg & ~keep;
  const int Gu = __popcll(keep);
  const bool no_rows = se == so;                    // Pn == 0
  if (level == 0 && keep == 0) return true;        // skipped contig (orgscorer.py:959)
  if (Gu == 0) {                                  // np.min of an empty array upstream
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
  int Pp = 0;
  sp_rows(S, so, se, [&](bool st, int t, int cl) {
    bool pot = false;
    uint64_t cmask = 0;
    if (st) {
      const SpRow r = sp_row(S, P, t, se, cl, allg);
      if ((r.mk1 & keep) == keep) {                 // crit >= k1 (:585-597)
        SpCursor cur{t, cl, se};
        uint64_t m = keep;
        auto next = [&]() -> double {
          const int g = __builtin_ctzll(m);
          m &= m - 1;
          return cur.at(S, g);
        };
        const double rank = (0.0 + np_sum_seq(Gu, next)) / (double)Gu;
        if (better(rank, cl, br, bk)) { br = rank; bk = cl; brs = t; }
      }
      pot = r.mk2 != 0ull;                          // max over all loci >= k2 (:603-605)
      cmask = r.mk2 & keep;
    }
    Pp += __popcll(__ballot(pot));
    if (pot) {
      int h = (int)(((cmask * 0x9E3779B97F4A7C15ull) >> 56) & (kSpCls - 1));
      for (int probe = 0; probe < kSpCls; ++probe) {
        const unsigned long long old = atomicCAS(&sh.ckey[h], ~0ull, (unsigned long long)cmask);
        if (old == ~0ull) atomicAdd(&sh.n_used, 1);
        if (old == ~0ull || old == cmask) { atomicAdd(&sh.ccnt[h], 1); break; }
        h = (h + 1) & (kSpCls - 1);
      }
    }
  });
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double r2 = __shfl_xor(br, off, 64);
    const long long k2 = __shfl_xor(bk, off, 64);
    const int rs2 = __shfl_xor(brs, off, 64);
    if (better(r2, k2, br, bk)) { br = r2; bk = k2; brs = rs2; }
  }
  __syncthreads();

  if (bk >= 0) {
    // meld_one (:621-631): options within --range of the best
    const int best = (int)bk;
    int acc = -1;
    if (P.dis1 == 1) {
      sp_rows(S, so, se, [&](bool st, int t, int cl) {
        if (!st) return;
        const SpRow r = sp_row(S, P, t, se, cl, allg);
        if ((r.mk1 & keep) != keep) return;
        SpCursor cur{t, cl, se};
        uint64_t m = keep;
        auto next = [&]() -> double {
          const int g = __builtin_ctzll(m);
          m &= m - 1;
          return cur.at(S, g);
        };
        const double rank = (0.0 + np_sum_seq(Gu, next)) / (double)Gu;
        if ((br - rank) <= P.range) {
          K.meld[mbase + atomicAdd(&sh.cnt, 1)] = cl;
          acc = lca2(K, acc, cl);
        }
      });
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) acc = lca2(K, acc, __shfl_xor(acc, off, 64));
    }
    __syncthreads();
    const int m = sh.cnt;
    if (P.dis1 == 1 && m == 0) {                    // negative --range: get_lca() of nothing
      if (lane == 0) K.status[c] = WF_E_BADINPUT;
      return true;
    }
    // the best clade's row: crit (min over kept loci) and set_synteny_one (:495-509)
    sh.row[lane] = 0.0;
    __syncthreads();
    {
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
    return true;
  }

  // ---- explain_two (:599-619) --------------------------------------------------------
  pair_evals += (int64_t)Pp * (Pp - 1) / 2;
  if (sh.n_used * 4 > kSpCls * 3) return false;    // too many classes for the table
  // class pairs: a class passes when (ma | mb) == keep for some class b (itself: >= 2 clades)
  int U = 0;
  for (int base = 0; base < kSpCls; base += 64) {  // the occupied slots, compacted
    const int h = base + lane;
    const bool occ = sh.ckey[h] != ~0ull;
    const uint64_t w = __ballot(occ);
    if (occ) sh.cls[U + __popcll(w & ((1ull << lane) - 1ull))] = h;
    U += __popcll(w);
  }
  __syncthreads();
  bool any = false;
  for (int ia = 0; ia < U; ++ia) {
    const int a = sh.cls[ia];
    const unsigned long long ma = sh.ckey[a];
    bool pass = false;
    for (int ib = lane; ib < U; ib += 64) {
      const int b = sh.cls[ib];
      if ((ma | sh.ckey[b]) != keep) continue;
      if (a == b && sh.ccnt[a] < 2) continue;
      pass = true;
    }
    if (__ballot(pass)) {
      any = true;
      if (lane == 0) sh.cint[a] = 1;
    }
  }
  __syncthreads();
  bool have_ok = false;
  int M = 0;
  if (any) {
    int Mtot = 0;
    for (int a = lane; a < kSpCls; a += 64) Mtot += sh.cint[a] ? sh.ccnt[a] : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) Mtot += __shfl_xor(Mtot, off, 64);
    if (Mtot > kSpMem) return false;
    // ---- pass 3: members (potential clades of passing classes), in potential order -----
    int pbase = 0;
    sp_rows(S, so, se, [&](bool st, int t, int cl) {
      bool pot = false, mem = false;
      SpRow r{0, 0, 0};
      if (st) {
        r = sp_row(S, P, t, se, cl, allg);
        pot = r.mk2 != 0ull;
        if (pot) {
          const uint64_t cmask = r.mk2 & keep;
          int h = (int)(((cmask * 0x9E3779B97F4A7C15ull) >> 56) & (kSpCls - 1));
          while (sh.ckey[h] != cmask) h = (h + 1) & (kSpCls - 1);
          mem = sh.cint[h] != 0;
        }
      }
      const uint64_t pb = __ballot(pot);
      const int pi = pbase + __popcll(pb & ((1ull << lane) - 1ull));
      pbase += __popcll(pb);
      if (mem) {
        const int q = atomicAdd(&sh.n_mem, 1);
        sh.mmask[q] = r.mk2 & keep;
        sh.mhm[q] = r.mhs;
        sh.mrs[q] = t;
        sh.mcl[q] = cl;
        sh.mpi[q] = pi;
        sh.msp[q] = K.sibp[cl];
      }
    });
    __syncthreads();
    M = sh.n_mem;
    if (P.sister_on) {
      // parents of the members (the parents whose listed children are their sisters)
      if (lane == 0) {
        int np = 0;
        bool over = false;
        for (int q = 0; q < M && !over; ++q) {
          const int p = K.parent[sh.mcl[q]];
          bool seen = false;
          for (int i = 0; i < np; ++i) seen |= sh.pkey[i] == p;
          if (seen) continue;
          if (np == kSpPar) { over = true; break; }
          sh.pkey[np] = p;
          sh.por[np] = 0;
          ++np;
        }
        sh.n_par = over ? -1 : np;
      }
      __syncthreads();
      if (sh.n_par < 0) return false;
      // ---- pass 4: sister masks of the non-member clades under those parents ----------
      sp_rows(S, so, se, [&](bool st, int t, int cl) {
        if (!st) return;
        const int sp = K.sibp[cl];
        const int slot = sp >= 0 ? sp_par_slot(sh, sp) : -1;
        if (slot < 0) return;
        const SpRow r = sp_row(S, P, t, se, cl, allg);
        if (r.mhs == 0ull) return;
        if (r.mk2 != 0ull) {                        // a member itself? (added per pair)
          const uint64_t cmask = r.mk2 & keep;
          int h = (int)(((cmask * 0x9E3779B97F4A7C15ull) >> 56) & (kSpCls - 1));
          while (sh.ckey[h] != cmask) h = (h + 1) & (kSpCls - 1);
          if (sh.cint[h]) return;
        }
        atomicOr(&sh.por[slot], (unsigned long long)r.mhs);
      });
      __syncthreads();
    }

    // ---- pass 1 over the pairs: best by (rank, pair index) ----------------------------------
    double pr = -__builtin_inf();
    long long pk = -1;
    int pu = -1, pv = -1;
    sp_for_pairs(sh, keep, [&](int u, int v, int i, int j) {
      const double r = sp_pair_rank(S, sh.mrs[u], sh.mcl[u], sh.mrs[v], sh.mcl[v], se, keep, Gu);
      const long long key = (long long)i * Pp + j;
      if (better(r, key, pr, pk)) { pr = r; pk = key; pu = u; pv = v; }
    });
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double r2 = __shfl_xor(pr, off, 64);
      const long long k2 = __shfl_xor(pk, off, 64);
      const int u2 = __shfl_xor(pu, off, 64), v2 = __shfl_xor(pv, off, 64);
      if (better(r2, k2, pr, pk)) { pr = r2; pk = k2; pu = u2; pv = v2; }
    }
    // every member is in some passing pair, so pk >= 0 here
    int best_ok = 0, best_dir = 0, best_c1 = -1, best_c2 = -1;
    double best_crit = 0.0;
    if (lane == 0) {
      int same;
      const OptEval e = sp_eval_two(S, sh, pu, pv, se, G, ign, false, sh.syn, same);
      best_ok = e.ok; best_dir = e.dir; best_c1 = e.c1p; best_c2 = e.c2p;
      best_crit = sp_pair_crit(S, sh.mrs[pu], sh.mcl[pu], sh.mrs[pv], sh.mcl[pv], se, keep);
      sh.n_in = 0; sh.all_ok = 1; sh.all_same = 1;
    }
    for (int i = lane; i < kSpMem / 32; i += 64) { sh.bm1[i] = 0; sh.bm2[i] = 0; }
    __syncthreads();
    // ---- pass 2 over the pairs: options within --range get the LGT filters (:636-639) --
    sp_for_pairs(sh, keep, [&](int u, int v, int, int) {
      const double r = sp_pair_rank(S, sh.mrs[u], sh.mcl[u], sh.mrs[v], sh.mcl[v], se, keep, Gu);
      if (!((pr - r) <= P.range)) return;
      int same;
      const OptEval e = sp_eval_two(S, sh, u, v, se, G, ign, true, nullptr, same);
      atomicAdd(&sh.n_in, 1);
      if (!e.ok) atomicAnd(&sh.all_ok, 0);
      if (!e.same) atomicAnd(&sh.all_same, 0);
      atomicOr(&sh.bm1[e.c1p >> 5], 1u << (e.c1p & 31));
      atomicOr(&sh.bm2[e.c2p >> 5], 1u << (e.c2p & 31));
    });
    __syncthreads();
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
        if (in_bm(sh.bm1, q)) a1 = lca2(K, a1, sh.mcl[q]);
        if (in_bm(sh.bm2, q)) a2 = lca2(K, a2, sh.mcl[q]);
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        a1 = lca2(K, a1, __shfl_xor(a1, off, 64));
        a2 = lca2(K, a2, __shfl_xor(a2, off, 64));
      }
      for (int w = 0; w < kSpMem / 32; ++w) { m1 += __popc(sh.bm1[w]); m2 += __popc(sh.bm2[w]); }
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
        const uint64_t below = (1ull << lane) - 1ull;
        int o1 = 0, o2 = 0;
        for (int base = 0; base < M; base += 64) {
          const int q = base + lane;
          const bool in1 = in_bm(sh.bm1, q), in2 = in_bm(sh.bm2, q);
          const uint64_t w1 = __ballot(in1), w2 = __ballot(in2);
          if (in1) K.meld[mbase + o1 + __popcll(w1 & below)] = sh.mcl[q];
          if (in2) K.meld[mbase + m1 + o2 + __popcll(w2 & below)] = sh.mcl[q];
          o1 += __popcll(w1);
          o2 += __popcll(w2);
        }
      }
      if (lane == 0) {
        K.call[c] = WF_CALL_LGT;
        K.crit[c] = best_crit;
        K.rank[c] = pr;
        K.dir[c] = (int8_t)best_dir;
        K.c1[c] = (kind == 2) ? lca1 : sh.mcl[best_c1];
        K.c2[c] = (kind == 2) ? lca2v : sh.mcl[best_c2];
        K.nm1[c] = (kind == 2) ? m1 : 0;
        K.nm2[c] = (kind == 2) ? m2 : 0;
        K.iters[c] = (int16_t)iteration;
        K.pair_evals[c] = pair_evals;
      }
      return true;
    }
  }
  const int dec = (no_rows || root_present) ? kDecStop : kDecRaise;
  if (dec == kDecRaise && iteration + 1 <= kMaxIter) {
    sp_raise(S, c, pair_evals);                      // roll up (orgscorer.py:431-445)
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

// The contigs whose dense decision state outgrew the LDS arena (big_list, counters[2]):
// one wave each; the ones sp_level declines go to big2_list (counters[1]) for k_decide_big.
__global__ __launch_bounds__(64) void k_big_sparse(const SArgs S, int level, int64_t n_keys) {
  __shared__ SpShared sh;
  const int count = (int)S.counters[2];
  for (int i = blockIdx.x; i < count; i += gridDim.x) {
    const int cr = S.big_list[2 * i], c = S.big_list[2 * i + 1];
    const bool ok = sp_level(S, sh, c, cr, level, n_keys);
    if (!ok && threadIdx.x == 0) {
      const int slot = (int)atomicAdd(&S.counters[1], 1ull);
      S.big2_list[2 * slot] = cr;
      S.big2_list[2 * slot + 1] = c;
    }
    __syncthreads();
  }
}
