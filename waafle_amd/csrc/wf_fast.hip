// Fused level 0 of the contig-scoring path (gfx950 / MI355X).
//
// One 256-thread workgroup carries one contig from its hits to its explain_one decision
// with every intermediate in LDS: attachments (orgscorer.py:359-392), the (clade, locus)
// sort and segments (:394-406), the exact numpy segment means (:399-406), per-locus maxes
// and the weak-locus mask (:407-429), Contig.score of every clade (:447-461), explain_one
// and meld_one (:585-597, :621-631).  A contig it cannot finish -- no one-clade option
// (explain_two), more attachments than the LDS holds, more than 64 loci, a segment no
// LDS-resident mean covers -- is handed to the staged path (wf_staged.hip) through a
// per-contig flag with its attachment and leaf counts; the staged level 0 then runs on
// those contigs only.  Contigs finished here never write attachments, keys or segment
// records to HBM: their traffic is the hits and loci read once plus the result record.
#include "wf_device.h"

namespace wf {

namespace {

constexpr int kFastNT = 256;
constexpr int kFastW = kFastNT / 64;
constexpr int kFastCap = 512;        // attachments held in LDS (the sort width)
constexpr int kSlotBits = 9;         // key = clade << 15 | locus << 9 | attachment slot
constexpr int kCladeShift = 15;
constexpr int kFastLoc = 64;         // loci per contig (locus bitmasks are 64-bit)
constexpr int kFastRuns = 64;        // envelope runs of a multi-attachment segment
constexpr int kFastMultiAtt = 32;    // ... so at most 32 attachments (2 * 32 - 1 runs)

struct FastSmem {
  uint64_t key[kFastCap];            // sort keys (slot order until the sort)
  int2 lohi[kFastCap];               // by slot: site range [lo, hi); after the means: (clade, locus) by segment
  double sc[kFastCap];               // by slot: score; after the means: option rank by segment
  int hit[kFastCap];                 // by slot: hit index; then the multi-run list, then meld members
  int seg[kFastCap + 1];             // segment starts (sorted positions)
  double v[kFastCap];                // segment means
  int lo[kFastLoc], len[kFastLoc], nl[kFastLoc];
  int8_t st[kFastLoc];
  unsigned long long mx[kFastLoc];   // per-locus max score bits over known clades
  unsigned long long abest[kAnnSlots];
  int ahit[kAnnSlots];
  WaveRunsT<kFastRuns> runs[kFastW];
  int red_i[kFastW];
  long long red_l[kFastW];
  double red_r[kFastW], red_c[kFastW];
  long long red_k[kFastW];
  int n_multi, n_mem, flag, lca;
  unsigned long long um;
};

// Exclusive block prefix sum (two barriers); *total = block sum.
__device__ __forceinline__ int fast_scan(int v, int* total, FastSmem& F) {
  const int lane = lane_id(), w = wave_id();
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) F.red_i[w] = x;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kFastW; ++i) {
    const int t = F.red_i[i];
    base += i < w ? t : 0;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

__device__ __forceinline__ long long fast_sum(long long v, FastSmem& F) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if (lane_id() == 0) F.red_l[wave_id()] = v;
  __syncthreads();
  long long t = 0;
#pragma unroll
  for (int i = 0; i < kFastW; ++i) t += F.red_l[i];
  __syncthreads();
  return t;
}

__device__ __forceinline__ int leaves_for(const SArgs& S, int len) {
  return (len / kNpyBuf) * (S.lut_off[kNpyBuf + 1] - S.lut_off[kNpyBuf]) +
         (S.lut_off[len % kNpyBuf + 1] - S.lut_off[len % kNpyBuf]);
}

__global__ __launch_bounds__(kFastNT) void k_fast(const SArgs S, int64_t* ccnt, int64_t* cleaves,
                                                  int32_t* pend) {
  const KArgs& K = S.k;
  const DevParams& P = K.p;
  __shared__ FastSmem F;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nsys = K.n_sys;
  for (int c = blockIdx.x; c < K.n_contigs; c += gridDim.x) {
    const int64_t h0 = K.hit_off[c], h1 = K.hit_off[c + 1];
    const int64_t l0 = K.loc_off[c];
    const int G = (int)(K.loc_off[c + 1] - l0);
    const int Gs = min(G, kFastLoc);
    for (int g = tid; g < kFastLoc; g += kFastNT) {
      F.mx[g] = 0ull;
      if (g < Gs) {
        const int a = K.lstart[l0 + g], b = K.lend[l0 + g];
        const int len = max(a, b) - min(a, b) + 1;
        F.lo[g] = min(a, b);
        F.len[g] = len;
        F.st[g] = K.lstrand[l0 + g];
        F.nl[g] = leaves_for(S, len);
      }
    }
    const int nann = Gs * nsys;                    // <= kAnnSlots (checked on the host)
    for (int i = tid; i < nann; i += kFastNT) { F.abest[i] = 0ull; F.ahit[i] = -1; }
    if (tid == 0) { F.n_multi = 0; F.n_mem = 0; F.flag = 0; }
    __syncthreads();

    // ---- hits -> attachments, in (hit, locus) order (orgscorer.py:359-382) ----
    int n_att = 0;
    long long nl_sum = 0;
    for (int64_t hb = h0; hb < h1; hb += kFastNT) {
      const int64_t h = hb + tid;
      int n = 0;
      uint64_t am = 0;
      int qlo = 0, qhi = 0;
      const bool live = h < h1 && K.scov[h] >= P.min_scov;
      if (live) {
        qlo = K.qlo[h];
        qhi = K.qhi[h];
        const int hs = K.hstrand[h];
        for (int g = 0; g < G; ++g) {
          int lo, len, st, nlg;
          if (g < kFastLoc) {
            lo = F.lo[g]; len = F.len[g]; st = F.st[g]; nlg = F.nl[g];
          } else {                                   // counted only (the contig goes staged)
            const int a = K.lstart[l0 + g], b = K.lend[l0 + g];
            lo = min(a, b); len = max(a, b) - lo + 1; st = K.lstrand[l0 + g]; nlg = leaves_for(S, len);
          }
          if (attaches(P, qlo, qhi, hs, lo, len, st)) {
            ++n;
            nl_sum += nlg;
            if (g < kFastLoc) am |= 1ull << g;
          }
        }
      }
      int total;
      const int o = fast_scan(n, &total, F);
      if (n > 0 && G <= kFastLoc && n_att + o + n <= kFastCap) {
        int clade = K.taxon[h];
        for (int j = 0; j < P.jump; ++j) clade = K.parent[clade];   // orgscorer.py:955-957
        const double sc = K.score[h];
        const uint32_t m = nsys > 0 ? K.sysmask[h] : 0u;
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
          F.key[slot] = ((uint64_t)(uint32_t)clade << kCladeShift) | ((uint64_t)g << kSlotBits) | (uint64_t)slot;
          F.lohi[slot] = make_int2(start, stop);
          F.sc[slot] = sc;
          F.hit[slot] = (int)h;
          if (ann)                                   // annotation pass 1: best score bits (:383-392)
            for (int b = 0; b < nsys; ++b)
              if ((m >> b) & 1u) atomicMax(&F.abest[g * nsys + b], dbits(sc));
        }
      }
      n_att += total;
    }
    const long long leaves = fast_sum(nl_sum, F);
    bool staged = G > kFastLoc || n_att > kFastCap;
    if (!staged && G > 0) {
      // annotation pass 2: the last hit (largest index) at the best score per (locus, system)
      if (nsys > 0) {
        for (int t = tid; t < n_att; t += kFastNT) {
          const int h = F.hit[t];
          const uint32_t m = K.sysmask[h];
          const double sc = F.sc[t];
          if (m == 0 || !(sc >= P.annot_ref)) continue;
          const int g = (int)((F.key[t] >> kSlotBits) & (kFastLoc - 1));
          for (int b = 0; b < nsys; ++b)
            if (((m >> b) & 1u) && F.abest[g * nsys + b] == dbits(sc)) atomicMax(&F.ahit[g * nsys + b], h);
        }
        __syncthreads();
        for (int i = tid; i < nann; i += kFastNT) K.annot[l0 * nsys + i] = F.ahit[i];
      }
    }
    const bool evaluated = !staged && G > 0 && h1 > h0;   // else: never evaluated (:959)
    if (evaluated) {
      // ---- per-contig sort of (clade, locus, slot) keys ----
      int n2 = 2;
      while (n2 < n_att) n2 <<= 1;
      for (int t = n_att + tid; t < n2; t += kFastNT) F.key[t] = ~0ull;
      __syncthreads();
      for (int k = 2; k <= n2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = tid; i < (n2 >> 1); i += kFastNT) {
            const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1));
            const int hi = lo | j;
            const bool up = (lo & k) == 0;
            const uint64_t ka = F.key[lo], kb = F.key[hi];
            if ((ka > kb) == up) { F.key[lo] = kb; F.key[hi] = ka; }
          }
          __syncthreads();
        }
      }
      // ---- segments = runs of equal (clade, locus) ----
      const int per = (n_att + kFastNT - 1) / kFastNT;
      const int b0 = min(n_att, tid * per), e0 = min(n_att, b0 + per);
      int heads = 0;
      for (int t = b0; t < e0; ++t)
        heads += (t == 0 || (F.key[t] >> kSlotBits) != (F.key[t - 1] >> kSlotBits)) ? 1 : 0;
      int ns;
      int so = fast_scan(heads, &ns, F);
      for (int t = b0; t < e0; ++t)
        if (t == 0 || (F.key[t] >> kSlotBits) != (F.key[t - 1] >> kSlotBits)) F.seg[so++] = t;
      if (tid == 0) F.seg[ns] = n_att;
      __syncthreads();
      // ---- segment means (numpy pairwise order, exact) ----
      for (int s = tid; s < ns; s += kFastNT) {
        const int kb = F.seg[s], ke = F.seg[s + 1], na = ke - kb;
        const int g = (int)((F.key[kb] >> kSlotBits) & (kFastLoc - 1));
        const int len = F.len[g];
        const int nl = len < kNpyBuf ? S.lut_off[len + 1] - S.lut_off[len] : 1 << 30;
        const bool thread_ok = len < kNpyBuf && nl <= kThreadLeaves;
        bool one_run = false;
        int lo = 0, hi = 0;
        double v = 0.0;
        if (na == 1) {
          if (thread_ok) {
            const int slot = (int)(F.key[kb] & ((1u << kSlotBits) - 1));
            lo = F.lohi[slot].x; hi = F.lohi[slot].y; v = F.sc[slot];
            one_run = true;
          }
        } else if (na <= kPruneMax) {
          double Fw = 0.0;                             // best whole-locus attachment
          for (int t = kb; t < ke; ++t) {
            const int slot = (int)(F.key[t] & ((1u << kSlotBits) - 1));
            const int2 x = F.lohi[slot];
            const double sc = F.sc[slot];
            if (x.x <= 0 && x.y >= len && sc > Fw) Fw = sc;
          }
          int kept = 0;                                // attachments the envelope still needs
          for (int t = kb; t < ke; ++t) {
            const int slot = (int)(F.key[t] & ((1u << kSlotBits) - 1));
            const int2 x = F.lohi[slot];
            kept += (x.x < x.y && F.sc[slot] > Fw) ? 1 : 0;
          }
          if (kept == 0 && thread_ok) { lo = 0; hi = len; v = Fw; one_run = true; }
        }
        if (one_run)
          F.v[s] = one_run_mean(S.lut + S.lut_off[len], nl, len, lo, hi, v);
        else if (na <= kFastMultiAtt && nl <= 64 && len < kNpyBuf)
          F.hit[atomicAdd(&F.n_multi, 1)] = s;
        else
          F.flag = 1;                                  // the staged leaf kernels take it
      }
      __syncthreads();
      const int n_multi = F.n_multi;
      for (int i = w; i < n_multi; i += kFastW) {      // one wave per multi-run segment
        const int s = F.hit[i];
        const int kb = F.seg[s], na = F.seg[s + 1] - kb;
        const int g = (int)((F.key[kb] >> kSlotBits) & (kFastLoc - 1));
        const int len = F.len[g];
        int lo = 0, hi = 0;
        double sc = 0.0;
        if (lane < na) {
          const int slot = (int)(F.key[kb + lane] & ((1u << kSlotBits) - 1));
          const int2 x = F.lohi[slot];
          if (x.x < x.y) { lo = x.x; hi = x.y; sc = F.sc[slot]; }
        }
        const double m = wave_seg_mean(S.lut + S.lut_off[len], S.lut_off[len + 1] - S.lut_off[len], len,
                                       lo, hi, sc, F.runs[w]);
        if (lane == 0) F.v[s] = m;
      }
      __syncthreads();
      staged = F.flag != 0;
      if (!staged) {
        // ---- explain_one (k_one's arithmetic, orgscorer.py:407-429, 447-461, 585-597) ----
        for (int s = tid; s < ns; s += kFastNT) {      // (clade, locus) by segment, into lohi
          const uint64_t k0 = F.key[F.seg[s]];
          F.lohi[s] = make_int2((int)(k0 >> kCladeShift), (int)((k0 >> kSlotBits) & (kFastLoc - 1)));
        }
        __syncthreads();
        for (int s = tid; s < ns; s += kFastNT) {      // per-locus max over known clades
          const int2 cg = F.lohi[s];
          const double v = F.v[s];
          if (cg.x != K.unknown && v > 0.0) atomicMax(&F.mx[cg.y], dbits(v));
        }
        __syncthreads();
        if (w == 0) {                                  // weak loci: ignore -> mask, penalize -> none
          const double mx = __longlong_as_double((long long)F.mx[lane]);
          const unsigned long long um = __ballot(lane < G && (P.weak != 0 || mx >= P.kmin));
          if (lane == 0) F.um = um;
        }
        __syncthreads();
        const uint64_t um = F.um;
        const int Gu = __popcll(um);
        if (Gu > 0) {                                  // else: skipped contig at level 0 (:959)
          double br = -__builtin_inf(), bcrit = 0.0;
          long long bk = -1;
          for (int t = tid; t < ns; t += kFastNT) {
            double rk = -1.0;
            const int clade = F.lohi[t].x;
            if (t == 0 || F.lohi[t - 1].x != clade) {
              uint64_t m = um;
              int q = t;
              double crit = 0.0;
              bool firstv = true;
              auto next = [&]() -> double {
                const int g = __builtin_ctzll(m);
                m &= m - 1;
                while (q < ns && F.lohi[q].x == clade && F.lohi[q].y < g) ++q;
                const double v = (q < ns && F.lohi[q].x == clade && F.lohi[q].y == g) ? F.v[q] : 0.0;
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
            F.sc[t] = rk;                              // option rank by segment (-1: none)
          }
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) {
            const double r2 = __shfl_xor(br, off, 64), c2 = __shfl_xor(bcrit, off, 64);
            const long long k2 = __shfl_xor(bk, off, 64);
            if (better(r2, k2, br, bk)) { br = r2; bk = k2; bcrit = c2; }
          }
          if (lane == 0) { F.red_r[w] = br; F.red_k[w] = bk; F.red_c[w] = bcrit; }
          __syncthreads();
          br = F.red_r[0]; bk = F.red_k[0]; bcrit = F.red_c[0];
#pragma unroll
          for (int i = 1; i < kFastW; ++i)
            if (better(F.red_r[i], F.red_k[i], br, bk)) { br = F.red_r[i]; bk = F.red_k[i]; bcrit = F.red_c[i]; }
          if (bk < 0) {
            staged = true;                             // explain_two (:570): the staged level 0
          } else {
            if (P.dis1 == 1)                           // meld_one (:621-631): options within --range
              for (int t = tid; t < ns; t += kFastNT) {
                const double rk = F.sc[t];
                if (rk >= 0.0 && (br - rk) <= P.range) F.hit[atomicAdd(&F.n_mem, 1)] = F.lohi[t].x;
              }
            __syncthreads();
            const int nm = F.n_mem;
            if (P.dis1 == 1 && nm == 0) {              // negative --range upstream crash
              if (tid == 0) K.status[c] = WF_E_BADINPUT;
            } else {
              int lca = (int)bk;
              if (P.dis1 == 1) {
                if (w == 0) {
                  int acc = -1;
                  for (int i = lane; i < nm; i += 64) acc = lca2(K, acc, F.hit[i]);
#pragma unroll
                  for (int off = 32; off > 0; off >>= 1) acc = lca2(K, acc, __shfl_xor(acc, off, 64));
                  if (lane == 0) F.lca = acc;
                }
                __syncthreads();
                lca = F.lca;
              }
              const int64_t mbase = 2 * h0 + 2 * (int64_t)c;
              for (int i = tid; i < nm; i += kFastNT) K.meld[mbase + i] = F.hit[i];
              for (int g = tid; g < G; g += kFastNT)   // set_synteny_one (:495-509)
                K.syn[l0 + g] = ((um >> g) & 1ull) ? 'A' : '~';
              if (tid == 0) {
                K.call[c] = WF_CALL_NO_LGT;
                K.crit[c] = bcrit;
                K.rank[c] = br;
                K.c1[c] = lca;
                K.c2[c] = -1;
                K.nm1[c] = nm;
                K.iters[c] = 1;
                K.pair_evals[c] = 0;
              }
            }
          }
        }
      }
    }
    if (tid == 0) {
      ccnt[c] = staged ? n_att : 0;
      cleaves[c] = staged ? leaves : 0;
      pend[c] = staged ? 1 : 0;
    }
    __syncthreads();                                   // LDS reuse by the next contig
  }
}

}  // namespace

int fast_blocks_per_cu() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&k_fast), kFastNT, 0) !=
          hipSuccess || n < 1)
    n = 1;
  return n;
}

hipError_t launch_fast(const SArgs& sa, int64_t* ccnt, int64_t* cleaves, int32_t* pend, unsigned grid,
                       hipStream_t s) {
  hipLaunchKernelGGL(k_fast, dim3(grid), dim3(kFastNT), 0, s, sa, ccnt, cleaves, pend);
  return hipGetLastError();
}

}  // namespace wf
