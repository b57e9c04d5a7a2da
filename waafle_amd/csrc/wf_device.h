// Device code shared by the fused per-contig kernels (wf_kernels.hip) and the staged
// pipeline (wf_staged.hip): block primitives, numpy's pairwise-sum leaf tables, the exact
// segment-mean arithmetic, and the per-level decision logic (explain_one / explain_two /
// melding / LGT filters).  Included by exactly those two translation units.
//
// Exactness rules: device code is compiled with -ffp-contract=off (no fma fusion), fp64
// division is IEEE-correct, and every float64 sum follows numpy's add.reduce order
// (8192-element buffers added sequentially from 0.0; each buffer summed pairwise with
// 128-element leaves of eight strided accumulators).
#pragma once
#include "wf_internal.h"

#include "waafle_hip.h"
#include "wf_lanes.h"

namespace wf {

namespace {


constexpr uint64_t kKeyPad = ~0ull;

#include "wf_stamps.h"
constexpr int kLocVirtual = 0xFFFF;     // locus field of the virtual "Unknown" key

// wf_result.ppot_sum: P_pot of an explain_two call that evaluates pairs (P_pot >= 2, the
// calls behind pair_evals), once per (contig, iteration).  Every form takes a contig's levels
// in increasing order, and a contig a form hands on is taken again from level 0 or from the
// level it stopped at (same data, same P_pot): so an iteration at or below the last one
// counted is a repeat.  One thread calls it.
__device__ __forceinline__ void note_ppot(const KArgs& K, int c, int iteration, int Pp) {
  if (!K.ppot || Pp < 2) return;
  const uint64_t old = (uint64_t)K.ppot[c];
  if (iteration > (int)(old >> 40))
    K.ppot[c] = (int64_t)(((uint64_t)iteration << 40) | ((old & ((1ull << 40) - 1ull)) + (uint64_t)Pp));
}

struct Ctl {
  int A, A1, npow, S_n, P, Gu, Pp;
  int overflow, status, cnt, cnt2, p_unk, root_present, all_ignored;
  int n_in, all_ok, all_same, best_ok, best_dir, best_c1p, best_c2p;
  int lca1, lca2, res_kind, lca_out;
  int cls_cnt[5], cls_off[5];
  double best_r, best_crit;
  long long best_k;
  int64_t need;
  double red_r[kWaves];
  long long red_k[kWaves];
  int red_i[kWaves];
  int red_j[kWaves];
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

struct Arena {
  char* base;
  int64_t cap;
  int64_t used;
  template <class T>
  __device__ __forceinline__ T* take(int64_t count) {
    int64_t off = (used + 15) & ~int64_t(15);
    used = off + count * (int64_t)sizeof(T);
    return reinterpret_cast<T*>(base + off);
  }
  __device__ __forceinline__ bool fits() const { return used <= cap; }
};

__device__ __forceinline__ uint64_t dbits(double x) { return (uint64_t)__double_as_longlong(x); }

// The kernel's first argument (at kernarg offset 0), through a pointer the compiler cannot
// see through: loads of its fields are not hoisted out of the loop that calls this.
template <class T>
__device__ __forceinline__ const T& kernarg_fresh(const T& arg) {
#ifdef __HIP_DEVICE_COMPILE__
  uint64_t a = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr());
  asm volatile("" : "+s"(a));
  return *reinterpret_cast<const __attribute__((address_space(4))) T*>(a);
#else
  return arg;                                        // (host pass: never executed)
#endif
}

// --------------------------------------------------------------------------
// block-wide primitives
// --------------------------------------------------------------------------

// Exclusive prefix sum of one int per thread; *total receives the block sum.
template <int NT>
__device__ __forceinline__ int block_scan(int v, int* total, Ctl& ctl) {
  const int lane = lane_id(), w = wave_id();
  int x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) ctl.red_i[w] = x;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    int t = ctl.red_i[i];
    base += (i < w) ? t : 0;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

// Two exclusive prefix sums at once.
template <int NT>
__device__ __forceinline__ void block_scan2(int v1, int v2, int* p1, int* p2, int* t1, int* t2, Ctl& ctl) {
  const int lane = lane_id(), w = wave_id();
  int x = v1, y = v2;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int a = __shfl_up(x, d, 64), b = __shfl_up(y, d, 64);
    if (lane >= d) { x += a; y += b; }
  }
  if (lane == 63) { ctl.red_i[w] = x; ctl.red_j[w] = y; }
  __syncthreads();
  int b1 = 0, b2 = 0, s1 = 0, s2 = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    int a = ctl.red_i[i], b = ctl.red_j[i];
    if (i < w) { b1 += a; b2 += b; }
    s1 += a;
    s2 += b;
  }
  __syncthreads();
  *p1 = b1 + x - v1;
  *p2 = b2 + y - v2;
  *t1 = s1;
  *t2 = s2;
}

// (rank, key) maximum; ties on rank go to the larger key (= later in enumeration order,
// which is what `sorted(options, key=rank)[-1]` picks, orgscorer.py:623-624, 634-635).
__device__ __forceinline__ bool better(double r2, long long k2, double r, long long k) {
  return k2 >= 0 && (k < 0 || r2 > r || (r2 == r && k2 > k));
}

template <int NT>
__device__ __forceinline__ void block_argmax(double& r, long long& k, Ctl& ctl) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    double r2 = __shfl_xor(r, off, 64);
    long long k2 = __shfl_xor(k, off, 64);
    if (better(r2, k2, r, k)) { r = r2; k = k2; }
  }
  if (lane_id() == 0) { ctl.red_r[wave_id()] = r; ctl.red_k[wave_id()] = k; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double br = ctl.red_r[0];
    long long bk = ctl.red_k[0];
    for (int i = 1; i < NT / 64; ++i)
      if (better(ctl.red_r[i], ctl.red_k[i], br, bk)) { br = ctl.red_r[i]; bk = ctl.red_k[i]; }
    ctl.best_r = br;
    ctl.best_k = bk;
  }
  __syncthreads();
  r = ctl.best_r;
  k = ctl.best_k;
}

template <int NT, class T>
__device__ __forceinline__ void bitonic_sort(T* keys, int n) {
  for (int k = 2; k <= n; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < n; i += NT) {
        int ixj = i ^ j;
        if (ixj > i) {
          T a = keys[i], b = keys[ixj];
          bool up = (i & k) == 0;
          if ((a > b) == up) { keys[i] = b; keys[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }
}

// --------------------------------------------------------------------------
// taxonomy helpers (utils.py:401-411)
// --------------------------------------------------------------------------

__device__ __forceinline__ int lca2(const KArgs& K, int a, int b) {
  if (a < 0) return b;
  if (b < 0) return a;
  if (a == b) return a;
  if (K.lin) {
    // lineage rows agree on a prefix (root first); the LCA is the deepest common entry.
    // Two independent 64-B row loads instead of a walk of dependent parent loads.
    const int4* ra = reinterpret_cast<const int4*>(K.lin + (int64_t)a * kLin);
    const int4* rb = reinterpret_cast<const int4*>(K.lin + (int64_t)b * kLin);
    int4 x[kLin / 4], y[kLin / 4];
#pragma unroll
    for (int i = 0; i < kLin / 4; ++i) { x[i] = ra[i]; y[i] = rb[i]; }
    int r = x[0].x;                                    // the root (depth 0)
#pragma unroll
    for (int i = 0; i < kLin / 4; ++i) {
      if (x[i].x >= 0 && x[i].x == y[i].x) r = x[i].x;
      if (x[i].y >= 0 && x[i].y == y[i].y) r = x[i].y;
      if (x[i].z >= 0 && x[i].z == y[i].z) r = x[i].z;
      if (x[i].w >= 0 && x[i].w == y[i].w) r = x[i].w;
    }
    return r;
  }
  int da = K.depth[a], db = K.depth[b];
  while (da > db) { a = K.parent[a]; --da; }
  while (db > da) { b = K.parent[b]; --db; }
  while (a != b) { a = K.parent[a]; b = K.parent[b]; }
  return a;
}

// LCA of list[0..m) (clade ids); wave 0 folds, result broadcast through ctl.
__device__ __forceinline__ int block_lca(const KArgs& K, const int* list, int m, Ctl& ctl) {
  if (m <= 0) return -1;
  if (m == 1) return list[0];
  if (wave_id() == 0) {
    int acc = -1;
    for (int i = lane_id(); i < m; i += 64) acc = lca2(K, acc, list[i]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      int o = __shfl_xor(acc, off, 64);
      acc = lca2(K, acc, o);
    }
    if (lane_id() == 0) ctl.lca_out = acc;
  }
  __syncthreads();
  int r = ctl.lca_out;
  __syncthreads();
  return r;
}

// --------------------------------------------------------------------------
// numpy pairwise summation order
// --------------------------------------------------------------------------

constexpr int kMaxDepth = 7;   // internal-node depths of one <=8192-element buffer: 0..6
constexpr int kGroupMax = 64;  // leaves combined by lane shuffles (one 8192 buffer = 64)

// Leaves of numpy's pairwise sum over one buffer [off0, off0+cl): emitted left to right
// as (start, length, number of parent additions completed right after this leaf).  The
// frame stack is a shift register (static indices) so it stays in VGPRs; depth <= 8.
// If `sched` is given (8 bytes for each of the first `stride` leaves, pre-set to -1) it
// also records the combine schedule: byte d of leaf i = j when leaf i is the leftmost leaf
// of an internal node at depth d whose right child starts at leaf j.
__device__ int gen_leaves(int off0, int cl, int4* out, int8_t* sched = nullptr, int stride = 0) {
  int so[8], sl[8], ss[8], sf[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { so[i] = 0; sl[i] = 0; ss[i] = 0; sf[i] = 0; }
  int cnt = 0;
  auto push = [&](int o, int l) {
#pragma unroll
    for (int i = 7; i > 0; --i) { so[i] = so[i - 1]; sl[i] = sl[i - 1]; ss[i] = ss[i - 1]; sf[i] = sf[i - 1]; }
    so[0] = o; sl[0] = l; ss[0] = 0; sf[0] = cnt;
  };
  auto pop = [&]() {
#pragma unroll
    for (int i = 0; i < 7; ++i) { so[i] = so[i + 1]; sl[i] = sl[i + 1]; ss[i] = ss[i + 1]; sf[i] = sf[i + 1]; }
  };
  int sp = 1;
  so[0] = off0; sl[0] = cl; ss[0] = 0; sf[0] = 0;
  while (sp > 0) {
    if (sl[0] > kLeafMax && ss[0] == 0) {
      int h = sl[0] / 2;
      h -= h % 8;
      ss[0] = 1;
      push(so[0], h);
      ++sp;
      continue;
    }
    const int lo = so[0], ll = sl[0];
    int adds = 0;
    pop();
    --sp;
    ++cnt;
    while (sp > 0) {
      if (ss[0] == 1) {
        int h = sl[0] / 2;
        h -= h % 8;
        ss[0] = 2;
        if (sched && sp - 1 < kMaxDepth && sf[0] < stride)
          sched[sf[0] * 8 + (sp - 1)] = (int8_t)cnt;
        push(so[0] + h, sl[0] - h);
        ++sp;
        break;
      }
      ++adds;
      pop();
      --sp;
    }
    if (out) out[cnt - 1] = make_int4(lo, ll, adds, 0);
  }
  return cnt;
}

__device__ int leaves_of_length(int n) {
  int cnt = 0;
  for (int o = 0; o < n; o += kNpyBuf) cnt += gen_leaves(o, min(kNpyBuf, n - o), nullptr);
  return cnt;
}

// One leaf (<= 128 elements) exactly as numpy's pairwise_sum inner block.
template <class F>
__device__ double serial_block(int o, int l, F f) {
  if (l < 8) {
    double r = 0.0;
    for (int i = 0; i < l; ++i) r += f(o + i);
    return r;
  }
  double r0 = f(o), r1 = f(o + 1), r2 = f(o + 2), r3 = f(o + 3);
  double r4 = f(o + 4), r5 = f(o + 5), r6 = f(o + 6), r7 = f(o + 7);
  int i = 8;
  const int m = l - (l & 7);
  for (; i < m; i += 8) {
    r0 += f(o + i); r1 += f(o + i + 1); r2 += f(o + i + 2); r3 += f(o + i + 3);
    r4 += f(o + i + 4); r5 += f(o + i + 5); r6 += f(o + i + 6); r7 += f(o + i + 7);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < l; ++i) res += f(o + i);
  return res;
}

// numpy's pairwise sum of one buffer (<= 8192 elements) by one thread: the leaves in
// order (the walk of gen_leaves, frame stack in shift registers so nothing spills to
// scratch), each folded onto a SumStack with its completed parent additions.
template <class F>
__device__ double serial_pairwise(int off0, int cl, F f) {
  if (cl <= kLeafMax) return serial_block(off0, cl, f);
  int so[8], sl[8], ss[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { so[i] = 0; sl[i] = 0; ss[i] = 0; }
  auto push = [&](int o, int l) {
#pragma unroll
    for (int i = 7; i > 0; --i) { so[i] = so[i - 1]; sl[i] = sl[i - 1]; ss[i] = ss[i - 1]; }
    so[0] = o; sl[0] = l; ss[0] = 0;
  };
  auto pop = [&]() {
#pragma unroll
    for (int i = 0; i < 7; ++i) { so[i] = so[i + 1]; sl[i] = sl[i + 1]; ss[i] = ss[i + 1]; }
  };
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0, a4 = 0.0, a5 = 0.0, a6 = 0.0, a7 = 0.0;
  int sp = 1;
  so[0] = off0; sl[0] = cl;
  while (sp > 0) {
    if (sl[0] > kLeafMax && ss[0] == 0) {
      int h = sl[0] / 2;
      h -= h % 8;
      ss[0] = 1;
      push(so[0], h);
      ++sp;
      continue;
    }
    const double v = serial_block(so[0], sl[0], f);
    a7 = a6; a6 = a5; a5 = a4; a4 = a3; a3 = a2; a2 = a1; a1 = a0; a0 = v;
    pop();
    --sp;
    while (sp > 0) {
      if (ss[0] == 1) {
        int h = sl[0] / 2;
        h -= h % 8;
        ss[0] = 2;
        push(so[0] + h, sl[0] - h);
        ++sp;
        break;
      }
      a0 = a1 + a0;                          // (left) + (right)
      a1 = a2; a2 = a3; a3 = a4; a4 = a5; a5 = a6; a6 = a7;
      pop();
      --sp;
    }
  }
  return a0;
}

// np.add.reduce over f(0..n) (one thread): 8192-element buffers added from 0.0.
template <class F>
__device__ __forceinline__ double np_sum(int n, F f) {
  if (n <= kLeafMax) return 0.0 + serial_block(0, n, f);   // one leaf (n = 0: 0.0)
  double total = 0.0;
  for (int o = 0; o < n; o += kNpyBuf) total += serial_pairwise(o, min(kNpyBuf, n - o), f);
  return total;
}

// --------------------------------------------------------------------------
// per-contig state
// --------------------------------------------------------------------------

struct Contig {
  int64_t h0, l0, mbase;
  int H, G;
  // persistent
  int *loc_lo, *loc_len, *loc_st, *leaf_off;
  int *loc_grp, *loc_steps, *sched_off;   // lane-group size, combine steps, schedule offset
  uint64_t* sched;                        // per leaf of a lane-group locus: 8 schedule bytes
  int4* leaves;
  int *alo, *ahi, *ahit, *aloc, *acl;
  double* asc;
  uint64_t* maxes;
  int *ign, *um;
  // per level
  uint64_t* keys;
  int *seg_start, *seg_cl, *cl_id, *pot, *mem1, *mem2, *sorder;
  double* S;
  uint64_t* mask;
  unsigned *bm1, *bm2;
  uint8_t* best_syn;
  char* xws = nullptr;                    // optional scratch for mask classes (explain_two)
  int64_t xcap = 0;
  int* sib_of = nullptr;                  // [Pn] listed parent of each clade (sister checks)
  uint64_t* hm = nullptr;                 // [Pn] loci where the clade scores >= the sister
                                          // threshold (G <= 64; null: per-locus scan)
};

// Shift-register stack of partial sums for numpy's pairwise tree.  Static indexing keeps
// it in VGPRs; 8 entries cover the deepest tree of one 8192-element buffer (depth 7).
struct SumStack {
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0, s4 = 0.0, s5 = 0.0, s6 = 0.0, s7 = 0.0;
  __device__ __forceinline__ void push(double v) {
    s7 = s6; s6 = s5; s5 = s4; s4 = s3; s3 = s2; s2 = s1; s1 = s0; s0 = v;
  }
  __device__ __forceinline__ void add_top() {   // (left) + (right), left pushed first
    s0 = s1 + s0;
    s1 = s2; s2 = s3; s3 = s4; s4 = s5; s5 = s6; s6 = s7;
  }
};

// Sequential float64 sum of `cnt` copies of v, starting from 0.0 (the value a strided
// accumulator reaches over `cnt` covered sites of a constant run; zeros add nothing).
__device__ __forceinline__ double seqsum(double v, int cnt) {
  double r = 0.0;
  for (int i = 0; i < cnt; ++i) r += v;
  return r;
}

__device__ __forceinline__ double leaf_tree(double r0, double r1, double r2, double r3, double r4,
                                            double r5, double r6, double r7) {
  return ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
}

// Number of t in [0, m) with base + 8t < bound.
__device__ __forceinline__ int below(int base, int bound, int m) {
  const int d = bound - base;
  return d <= 0 ? 0 : min(m, (d + 7) >> 3);
}

// --------------------------------------------------------------------------
// segment means shared by the staged kernels and the fused level-0 kernel (wf_fast.hip)
// --------------------------------------------------------------------------
constexpr int kThreadLeaves = 32;
// explain_two from the wave form's compact hand-over (wf_fast.hip, sp_two in wf_sparse.h)
constexpr int kE2Seg = 320;        // segments of one compact table (LDS of k_dump_sparse)
constexpr int kE2MaxG = 63;        // loci (locus masks keep bit 63 for the root flag)
constexpr int kPruneMax = 64;      // attachments scanned for whole-locus domination

__device__ __forceinline__ bool attaches(const DevParams& P, int qlo, int qhi, int hs, int l1,
                                         int len, int lst) {
  if (P.stranded && hs != lst) return false;
  const int l2 = l1 + len - 1;
  if (l1 > qhi || qlo > l2) return 0.0 >= P.min_overlap;   // calc_overlap -> int 0
  const int ov = min(qhi, l2) - max(qlo, l1) + 1;
  const int den = min(qhi - qlo + 1, l2 - l1 + 1);
  if (ov == den) return 1.0 >= P.min_overlap;       // one interval inside the other: exactly 1.0
  // RN(ov / den) >= m decided without the division when ov is clearly above or below den * m
  // (rounding is monotone; the margins cover den * m's own rounding)
  const double t = (double)den * P.min_overlap;
  if ((double)ov > t + fabs(t) * 1e-9) return true;
  if ((double)ov < t - fabs(t) * 1e-9) return false;
  return (double)ov / (double)den >= P.min_overlap;
}

// numpy's leaf [st, st+ln) over sites holding v on [lo, hi) and 0 elsewhere: accumulator c
// adds v k_c times from 0.0 (k_c in {kmin, kmin+1, kmin+2}: seqsum closed form, see
// SegAttT::closed_body), tree of the 8, then the tail sites in order.
__device__ __forceinline__ double run_leaf(int lo, int hi, double v, int st, int ln) {
  const int m = ln >> 3, be = st + (m << 3);
  hi = max(hi, lo);                                  // empty slice (--min-overlap 0 wrap)
  double res = 0.0;
  if (m > 0) {
    int k[8], kmin = m;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      k[c] = below(st + c, hi, m) - below(st + c, lo, m);
      kmin = min(kmin, k[c]);
    }
    double s0 = 0.0;
    for (int i = 0; i < kmin; ++i) s0 += v;
    const double s1 = s0 + v, s2 = s1 + v;
    double r[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) r[c] = k[c] == kmin ? s0 : (k[c] == kmin + 1 ? s1 : s2);
    res = leaf_tree(r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
  }
  for (int x = be; x < st + ln; ++x) res += (x >= lo && x < hi) ? v : 0.0;
  return res;
}

// numpy add.reduce of n <= 128 values produced in order by next() (pairwise_sum's leaf:
// n < 8 sequential, else eight strided accumulators combined as a tree, then the tail)
template <class F>
__device__ __forceinline__ double np_sum_seq(int n, F next) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += next();
    return r;
  }
  double r0 = next(), r1 = next(), r2 = next(), r3 = next();
  double r4 = next(), r5 = next(), r6 = next(), r7 = next();
  int i = 8;
  const int m = n - (n & 7);
  for (; i < m; i += 8) {
    r0 += next(); r1 += next(); r2 += next(); r3 += next();
    r4 += next(); r5 += next(); r6 += next(); r7 += next();
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += next();
  return res;
}

// Mean of a segment whose site array is ONE run of value v on [lo, hi) over a zero
// background (len < kNpyBuf: one numpy buffer; lt/nl: its leaf table).  Three uniform
// phases instead of one leaf formula per loop trip (the lanes of a wave would otherwise run
// every leaf kind on every trip):
//  A. classify the leaves against the run: at most two straddle a run boundary, the ones
//     inside have at most 4 distinct lengths (numpy's split of one buffer);
//  B. the <= 2 boundary leaves by run_leaf, each inside length once (8 equal accumulators:
//     8 * seqsum, exact doubling, then the tail in order);
//  C. the tree, picking each leaf's value (outside leaves are 0).
// Leaf tables are read through a getter: q -> (start, length, parent adds) of leaf q.
struct PtrLut {                       // the device table (int4 per leaf)
  const int4* p;
  __device__ __forceinline__ int4 operator()(int q) const { return p[q]; }
};
// Packed leaf entry (LDS copies): start | length << 13 | parent adds << 21.
__device__ __forceinline__ uint32_t pack_leaf(int4 e) { return (uint32_t)e.x | ((uint32_t)e.y << 13) | ((uint32_t)e.z << 21); }
struct PackedLut {
  const uint32_t* p;
  __device__ __forceinline__ int4 operator()(int q) const {
    const uint32_t u = p[q];
    return make_int4((int)(u & 8191u), (int)((u >> 13) & 255u), (int)(u >> 21), 0);
  }
};

// numpy's pairwise sum of n copies of v (n < kNpyBuf: one buffer) from registers alone,
// without the leaf table.  A node of size n > 128 splits into 8*floor(n/16) (left) and the
// rest, so the right-most nodes (the spine) have sizes = n mod 8 and every other node is a
// multiple of 8.  Those are 8*B_d or 8*(B_d + 1) at depth d, B_d = a0 >> d with a0 the top
// split's left size / 8, and the spine's left sibling at depth d is one of the two.  So
// with Q(x) = the sum over 8x sites (8 * seqsum(v, x) for x <= 16, else Q(floor(x/2)) +
// Q(ceil(x/2))) one pair (Q(B_d), Q(B_d + 1)) per depth carries the whole tree: bottom pair
// from seqsum captures (seqsum(v, x + 1) = seqsum(v, x) + v exactly), each pair above from
// the one below, and the spine sum adds its left sibling's Q level by level.  Equal to the
// leaf-table walk bit for bit for every n < 8192 (tests/test_pw_const.py checks the model).
__device__ __forceinline__ double pw_const_sum(int n, double v) {
  const int a0 = n >> 4;
  int K = 0, m = n;
  unsigned sel = 0;                                  // bit d: the spine's sibling is 8*(B_d + 1)
  while (m > 128) {
    const int a = m >> 4;
    sel |= (a != (a0 >> K) ? 1u : 0u) << K;
    m -= 8 * a;
    ++K;
  }
  int Db = 0, Dmax = -1, xB = 0, xC = 0;
  bool need16 = false;
  if (K > 0) {
    Db = max(0, 28 - __clz(a0));                     // first depth with B_d <= 15
    Dmax = max(K - 1, Db);
    xB = a0 >> Db;
    xC = Dmax == Db + 1 ? a0 >> (Db + 1) : 0;
    need16 = Db >= 1 && (a0 >> (Db - 1)) == 16;      // Q(16) is a leaf, not Q(8) + Q(8)
  }
  const int mL = m < 8 ? m : m >> 3;                 // the spine leaf's accumulator length
  const int imax = max(max(xB, mL), need16 ? 16 : 0);
  double t = 0.0, sB = 0.0, sC = 0.0, sL = 0.0;
  for (int i = 1; i <= imax; ++i) {                  // seqsum(v, i), captured where needed
    t += v;
    sB = i == xB ? t : sB;
    sC = i == xC ? t : sC;
    sL = i == mL ? t : sL;
  }
  double R;
  if (m < 8) {
    R = sL;
  } else {
    R = 8.0 * sL;
    for (int x = 0; x < (m & 7); ++x) R += v;
  }
  double q0 = 0.0, q1 = 0.0;
  for (int d = Dmax; d >= 0; --d) {
    const int B = a0 >> d;
    if (d >= Db) {
      const double sd = d == Db ? sB : sC;
      q0 = 8.0 * sd;
      q1 = 8.0 * (sd + v);
    } else {
      const double c0 = q0, c1 = q1;
      q0 = (B & 1) ? c0 + c1 : c0 + c0;
      q1 = (B & 1) ? c1 + c1 : c0 + c1;
      if (B == 16) q0 = 8.0 * t;                     // t = seqsum(v, 16) (imax = 16)
    }
    if (d < K) R = (((sel >> d) & 1u) ? q1 : q0) + R;
  }
  return R;
}

// run_leaf in two steps, for callers that share one seqsum chain: the leaf's shape from
// integers alone -- kmin, then per accumulator 2 bits (k_c - kmin, 2 meaning "or more" as
// run_leaf's select), the in-run tail sites (bits 16-19; a 0.0 tail site adds nothing to
// a non-negative sum) and m > 0 (bit 20) -- then its value from s0 = seqsum(v, kmin).
// Same operations as run_leaf, with two registers of state between the steps.
struct LeafCode { int kmin, code; };
__device__ __forceinline__ LeafCode run_leaf_code(int lo, int hi, int st, int ln) {
  const int m = ln >> 3, be = st + (m << 3);
  hi = max(hi, lo);
  int k[8], kmin = m;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    k[c] = below(st + c, hi, m) - below(st + c, lo, m);
    kmin = min(kmin, k[c]);
  }
  int code = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) code |= min(k[c] - kmin, 2) << (2 * c);
  const int tail = max(0, min(st + ln, hi) - max(be, lo));
  return LeafCode{kmin, code | (tail << 16) | (m > 0 ? 1 << 20 : 0)};
}
__device__ __forceinline__ double run_leaf_value(double v, LeafCode lc, double s0) {
  double res = 0.0;
  if ((lc.code >> 20) & 1) {
    const double s1 = s0 + v, s2 = s1 + v;
    double r[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int d = (lc.code >> (2 * c)) & 3;
      r[c] = d == 0 ? s0 : (d == 1 ? s1 : s2);
    }
    res = leaf_tree(r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
  }
  for (int x = (lc.code >> 16) & 15; x > 0; --x) res += v;
  return res;
}

// numpy's pairwise sum of n sites (n < kNpyBuf) holding v on [lo, hi) and 0.0 elsewhere,
// from registers alone.  A node disjoint from the run sums to 0.0 and x + 0.0 = x, so above
// the split node (the deepest one holding the whole run) every node passes its child's sum
// up; below it the run is a suffix of the left child and a prefix of the right one.  A
// suffix (prefix) node whose boundary falls in its left (right) child adds the whole other
// child, else it passes the child holding the boundary up; each path ends at a node inside
// the run or at a leaf.  Whole nodes are the spine or pair nodes of pw_const_sum, so one
// ascent of its pair chain supplies every whole node's sum at its depth, and the two paths'
// additions (recorded as bits per depth on the way down) are applied in the same ascent.
// The walks are integer bookkeeping only: the (at most two) boundary leaves take their
// seqsum values from the chain that also feeds the pair chain, so every lane runs the same
// straight sequence -- one chain, two closed-form leaves, one ascent -- whatever its run's
// shape (the leaf evaluations used to sit in three divergent branches, each with its own
// chain).  tests/test_pw_const.py restates this line by line and checks it against numpy's
// tree on explicit arrays.
__device__ __forceinline__ double pw_run_sum(int n, int lo, int hi, double v) {
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
  int mode = 0;                                      // 0 two paths, 1 a whole node, 2 one leaf
  for (;;) {                                         // down to the split node
    if (lo <= nd.s && hi >= nd.s + nd.z) { mode = 1; break; }
    if (nd.z <= 128) { mode = 2; break; }
    const int nl = nd.kind == 0 ? 8 * (nd.z >> 4) : 8 * ((nd.z >> 3) >> 1);
    if (hi <= nd.s + nl) nd = child(nd, false);
    else if (lo >= nd.s + nl) nd = child(nd, true);
    else break;
  }
  // the two paths: terminal depth / type (0 whole spine, 1 whole pair, 2 leaf) / class, per
  // depth a whole sibling to add (is it the spine, its class), and a leaf end's run and span.
  // One leaf holding the whole run (mode 2) is path 0's leaf at the split depth.
  struct Path { int tu, ty, tc; unsigned ev, evk, evc; LeafCode lc; };
  auto walk = [&](bool suffix) -> Path {
    Path q{0, 0, 0, 0u, 0u, 0u, LeafCode{0, 0}};
    Nd x = child(nd, !suffix);
    for (;;) {
      if (suffix ? lo <= x.s : hi >= x.s + x.z) { q.tu = x.t; q.ty = x.kind; q.tc = x.cls; return q; }
      if (x.z <= 128) {
        q.tu = x.t; q.ty = 2;
        q.lc = suffix ? run_leaf_code(lo, x.s + x.z, x.s, x.z) : run_leaf_code(x.s, hi, x.s, x.z);
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
  Path p0{0, 0, 0, 0u, 0u, 0u, LeafCode{0, 0}}, p1{0, 0, 0, 0u, 0u, 0u, LeafCode{0, 0}};
  if (mode == 0) {
    p0 = walk(true);
    p1 = walk(false);
  } else if (mode == 2) {
    p0.ty = 2;
    p0.lc = run_leaf_code(lo, hi, nd.s, nd.z);
  }
  const int k0 = p0.lc.kmin, k1 = p1.lc.kmin;         // (0 without a leaf end)
  const int mL = m < 8 ? m : m >> 3;
  const int imax = mode == 2 ? k0 : max(max(max(xB, mL), need16 ? 16 : 0), max(k0, k1));   // (<= 16)
  double t = 0.0, sB = 0.0, sC = 0.0, sL = 0.0, s0a = 0.0, s0b = 0.0;
  for (int i = 1; i <= imax; ++i) {                  // seqsum(v, i), captured where needed
    t += v;
    sB = i == xB ? t : sB;
    sC = i == xC ? t : sC;
    sL = i == mL ? t : sL;
    s0a = i == k0 ? t : s0a;
    s0b = i == k1 ? t : s0b;
  }
  const double lv0 = p0.ty == 2 ? run_leaf_value(v, p0.lc, s0a) : 0.0;
  if (mode == 2) return lv0;
  const double lv1 = p1.ty == 2 ? run_leaf_value(v, p1.lc, s0b) : 0.0;
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
        if (B == 16) q0 = 8.0 * t;                   // t = seqsum(v, 16) (imax = 16)
      }
    }
    if (mode == 1) {
      if (u == nd.t) return nd.kind == 0 ? R : (nd.cls ? q1 : q0);
    } else {
      if (u == p0.tu) acc0 = p0.ty == 2 ? lv0 : (p0.ty == 0 ? R : (p0.tc ? q1 : q0));
      if (u <= p0.tu && ((p0.ev >> u) & 1u))
        acc0 = acc0 + (((p0.evk >> u) & 1u) ? R : (((p0.evc >> u) & 1u) ? q1 : q0));
      if (u == p1.tu) acc1 = p1.ty == 2 ? lv1 : (p1.ty == 0 ? R : (p1.tc ? q1 : q0));
      if (u <= p1.tu && ((p1.ev >> u) & 1u))
        acc1 = (((p1.evc >> u) & 1u) ? q1 : q0) + acc1;
      if (u == nd.t + 1) return acc0 + acc1;
    }
    if (d >= 0 && d < K) R = (((sel >> d) & 1u) ? q1 : q0) + R;
  }
  return 0.0;                                        // (not reached)
}

template <class LT>
__device__ __forceinline__ double one_run_mean(LT lt, int nl, int len, int lo, int hi, double v) {
  hi = max(hi, lo);
  if (lo <= 0 && hi >= len && len < kNpyBuf)         // one run over the whole locus
    return (0.0 + pw_const_sum(len, v)) / (double)len;
  if (len < kNpyBuf)                                 // any other run: no leaf table either
    return (0.0 + pw_run_sum(len, lo, hi, v)) / (double)len;
  int pst0 = -1, pln0 = 0, pst1 = -1, pln1 = 0;
  int L0 = -1, L1 = -1, L2 = -1, L3 = -1;
#pragma unroll 4
  for (int q = 0; q < nl; ++q) {
    const int4 e = lt(q);
    const int le = e.x + e.y;
    const bool in = lo <= e.x && le <= hi && lo < hi;
    const bool out = le <= lo || e.x >= hi || lo >= hi;
    if (!in && !out) {
      if (pst0 < 0) { pst0 = e.x; pln0 = e.y; } else { pst1 = e.x; pln1 = e.y; }
    } else if (in && e.y != L0 && e.y != L1 && e.y != L2 && e.y != L3) {
      if (L0 < 0) L0 = e.y; else if (L1 < 0) L1 = e.y; else if (L2 < 0) L2 = e.y; else L3 = e.y;
    }
  }
  const double vp0 = pst0 >= 0 ? run_leaf(lo, hi, v, pst0, pln0) : 0.0;
  const double vp1 = pst1 >= 0 ? run_leaf(lo, hi, v, pst1, pln1) : 0.0;
  auto inside = [&](int ln) -> double {
    if (ln < 0) return 0.0;
    double b = 0.0;
    for (int i = 0; i < (ln >> 3); ++i) b += v;
    double res = 8.0 * b;
    for (int x = ln & ~7; x < ln; ++x) res += v;
    return res;
  };
  const double V0 = inside(L0), V1 = inside(L1), V2 = inside(L2), V3 = inside(L3);
  SumStack stk;
#pragma unroll 4
  for (int q = 0; q < nl; ++q) {
    const int4 e = lt(q);
    const int le = e.x + e.y;
    const bool in = lo <= e.x && le <= hi && lo < hi;
    const bool out = le <= lo || e.x >= hi || lo >= hi;
    double x = 0.0;
    if (in) x = e.y == L0 ? V0 : e.y == L1 ? V1 : e.y == L2 ? V2 : V3;
    else if (!out) x = e.x == pst0 ? vp0 : vp1;
    stk.push(x);
    for (int a = 0; a < e.z; ++a) stk.add_top();
  }
  return (0.0 + stk.s0) / (double)len;
}

// Orders this wave's LDS accesses (one wave of a multi-wave workgroup working alone).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Segments with up to 64 attachments, one wave each: the max-envelope is swept once into
// runs (lane i holds attachment i; run value = wave max over the covering ones, run end =
// wave min over the next boundaries), then lane q evaluates leaf q (nl <= 64) from the runs
// -- each of the eight stride accumulators adds its sites in site order, a run of value v
// contributing v k_c times (zero runs add nothing: x + 0.0 = x for x >= 0) -- and lane 0
// folds the leaves in tree order.  Same sums as k_leaf's per-leaf stride walks.  A lane
// without an attachment passes lo = hi = 0.  Returns the mean on every lane.
// R bounds the positive runs: 2 * attachments - 1.
constexpr int kWaveRuns = 2 * 64 + 2;
template <int R>
struct WaveRunsT {
  int r_lo[R], r_hi[R];
  double r_v[R];
  double lv[64];
  int z[64];
};
using WaveRuns = WaveRunsT<kWaveRuns>;

template <int R, class LT>
__device__ __forceinline__ double wave_seg_mean(LT lt, int nl, int len, int lo, int hi, double sc,
                                                WaveRunsT<R>& W) {
  const int lane = lane_id();
  int nr = 0;
  for (int x = 0; x < len;) {                       // wave-uniform sweep
    double v = (lo <= x && x < hi) ? sc : 0.0;
    int nb = len;
    if (lo < hi) {
      if (lo > x) nb = lo;
      else if (hi > x) nb = hi;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double v2 = __shfl_xor(v, off, 64);
      const int n2 = __shfl_xor(nb, off, 64);
      v = v2 > v ? v2 : v;
      nb = n2 < nb ? n2 : nb;
    }
    if (v > 0.0) {
      if (lane == 0) { W.r_lo[nr] = x; W.r_hi[nr] = nb; W.r_v[nr] = v; }
      ++nr;
    }
    x = nb;
  }
  wave_sync();
  if (lane < nl) {
    const int4 e = lt(lane);
    const int st = e.x, ln = e.y, m = ln >> 3, be = st + (m << 3);
    int j = 0;
    while (j < nr && W.r_hi[j] <= st) ++j;
    double r[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) r[c] = 0.0;
    for (int jj = j; jj < nr && W.r_lo[jj] < be; ++jj) {
      const int a = max(W.r_lo[jj], st), b = min(W.r_hi[jj], be);
      const double v = W.r_v[jj];
      int k[8], kmin = m;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        k[c] = below(st + c, b, m) - below(st + c, a, m);
        kmin = min(kmin, k[c]);
      }
      for (int q = 0; q < kmin; ++q) {
#pragma unroll
        for (int c = 0; c < 8; ++c) r[c] += v;
      }
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if (k[c] > kmin) r[c] += v;
    }
    double res = m > 0 ? leaf_tree(r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]) : 0.0;
    for (int x = be; x < st + ln; ++x) {            // tail sites, in order
      while (j < nr && W.r_hi[j] <= x) ++j;
      res += (j < nr && W.r_lo[j] <= x) ? W.r_v[j] : 0.0;
    }
    W.lv[lane] = res;
    W.z[lane] = e.z;
  }
  wave_sync();
  double mean = 0.0;
  if (lane == 0) {
    SumStack stk;
    for (int q = 0; q < nl; ++q) {
      stk.push(W.lv[q]);
      for (int a = 0; a < W.z[q]; ++a) stk.add_top();
    }
    mean = (0.0 + stk.s0) / (double)len;
  }
  wave_sync();                                      // W is reused by the next segment
  return __shfl(mean, 0, 64);
}

constexpr int kRegAtt = 4;   // attachments of a segment held in registers

// The attachments of one (clade, locus) segment -- sorted keys [kb, ke) -- and the exact
// numpy value of one pairwise-sum leaf of its site array.  Site x holds
// max(0, max{score_a : lo_a <= x < hi_a}).
// Where a segment's attachments come from: the fused kernel's sorted LDS keys (attachment
// index in the low 24 bits) or the staged path's sorted (key, attachment index) pairs.
// Attachment sources for SegAttT: sorted position t -> attachment index -> (range, score).
struct KeySrc {
  const uint64_t* keys;
  const int *alo, *ahi;
  const double* asc;
  __device__ __forceinline__ int idx(int t) const { return (int)(keys[t] & 0xFFFFFFull); }
  __device__ __forceinline__ void att(int a, int& l, int& h, double& v) const {
    l = alo[a]; h = ahi[a]; v = asc[a];
  }
};
struct SortedSrc {                       // attachments gathered into sorted order
  const int2* lohi;
  const double* sc;
  __device__ __forceinline__ int idx(int t) const { return t; }
  __device__ __forceinline__ void att(int a, int& l, int& h, double& v) const {
    const int2 x = lohi[a];
    l = x.x; h = x.y; v = sc[a];
  }
};
struct ValSrc {
  const int* vals;
  const int *alo, *ahi;
  const double* asc;
  __device__ __forceinline__ int idx(int t) const { return vals[t]; }
  __device__ __forceinline__ void att(int a, int& l, int& h, double& v) const {
    l = alo[a]; h = ahi[a]; v = asc[a];
  }
};

// NREG: attachments held in registers (segments of at most NREG attachments; the rest are
// read from the source each time)
template <class Src, int NREG = kRegAtt>
struct SegAttT {
  int kb, ke;
  bool reg;
  int lo[NREG], hi[NREG];
  double sc[NREG];

  __device__ __forceinline__ void load(const Src& C, int kb_, int ke_) {
    kb = kb_; ke = ke_;
    reg = ke - kb <= NREG;
#pragma unroll
    for (int i = 0; i < NREG; ++i) {
      const bool use = reg && kb + i < ke;
      int l = 0, h = 0;
      double v = 0.0;
      if (use) C.att(C.idx(kb + i), l, h, v);
      lo[i] = l;
      hi[i] = h;                           // lo == hi: never covers
      sc[i] = v;
    }
  }
  __device__ __forceinline__ void get(const Src& C, int t, int& l, int& h, double& v) const {
    C.att(C.idx(t), l, h, v);
  }
  __device__ __forceinline__ double value_at(const Src& C, int x) const {
    double v = 0.0;
    if (reg) {
#pragma unroll
      for (int i = 0; i < NREG; ++i)
        if (x >= lo[i] && x < hi[i]) v = sc[i] > v ? sc[i] : v;
    } else {
      for (int t = kb; t < ke; ++t) {
        int l, h; double s;
        get(C, t, l, h, s);
        if (x >= l && x < h) v = s > v ? s : v;
      }
    }
    return v;
  }
  // numpy's leaf: 8 strided accumulators over the body of 8m sites, combined as
  // ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the tail added in order.  Accumulator c
  // adds the sites st+c+8t, t = 0..m-1, sequentially from 0.0.  The closed forms are
  // bit-identical to that sequence (adding +0.0 to a non-negative partial sum is exact and
  // a constant v added k times from 0.0 is seqsum(v, k)):
  //  - kConst, envelope F over the whole body: every r_c = seqsum(F, m), and the tree of 8
  //    equal values is 8*seqsum(F, m) (each level doubles exactly);
  //  - kSingle, one nonzero run s over a zero background (a hit boundary inside the leaf,
  //    ~97% of the non-constant leaves): r_c = seqsum(s, k_c), k_c spans <= 3 values;
  //  - kRuns, anything else: stride_sum() walks the envelope's runs in site order and adds
  //    each run's value k_c times (used by 8 cooperating lanes, one accumulator each).
  static constexpr int kConst = 0, kSingle = 1, kRuns = 2;
  template <bool REG>
  __device__ __forceinline__ void att(const Src& C, int i, int& l, int& h, double& v) const {
    if (REG) { l = lo[i]; h = hi[i]; v = sc[i]; } else get(C, kb + i, l, h, v);
  }
  template <bool REG>
  __device__ __forceinline__ int classify(const Src& C, int st, int m, double& F, int& plo,
                                          int& phi, double& ps) const {
    const int be = st + (m << 3);
    const int na = REG ? NREG : ke - kb;
    F = 0.0;
#pragma unroll
    for (int i = 0; i < na; ++i) {
      int l, h; double v;
      att<REG>(C, i, l, h, v);
      if (l < h && l <= st && be <= h) F = v > F ? v : F;
    }
    int npos = 0;
    plo = phi = 0; ps = 0.0;
#pragma unroll
    for (int i = 0; i < na; ++i) {
      int l, h; double v;
      att<REG>(C, i, l, h, v);
      if (l < h && l < be && h > st && !(l <= st && be <= h) && v > F) {
        ++npos; plo = l; phi = h; ps = v;
      }
    }
    return npos == 0 ? kConst : (npos == 1 && !(F > 0.0)) ? kSingle : kRuns;
  }
  __device__ __forceinline__ static double closed_body(int kind, int st, int m, double F,
                                                       int plo, int phi, double ps) {
    if (kind == kConst) return F > 0.0 ? 8.0 * seqsum(F, m) : 0.0;
    int k[8], kmin = m;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      k[c] = below(st + c, phi, m) - below(st + c, plo, m);
      kmin = min(kmin, k[c]);
    }
    const double s0 = seqsum(ps, kmin), s1 = s0 + ps, s2 = s1 + ps;
    double r[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) r[c] = k[c] == kmin ? s0 : (k[c] == kmin + 1 ? s1 : s2);
    return leaf_tree(r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
  }
  // Stride accumulator c of the body [st, st+8m): sequential sum of its m sites.
  template <bool REG>
  __device__ __forceinline__ double stride_sum_t(const Src& C, int st, int m, int c) const {
    const int be = st + (m << 3), na = REG ? NREG : ke - kb;
    double r = 0.0;
    for (int x = st; x < be;) {
      double v = 0.0;
      int nx = be;
#pragma unroll
      for (int i = 0; i < na; ++i) {
        int l, h; double s;
        att<REG>(C, i, l, h, s);
        if (l < h) {
          if (l <= x && x < h) { v = s > v ? s : v; nx = min(nx, h); }
          else if (l > x) nx = min(nx, l);
        }
      }
      if (v > 0.0) {
        const int k = below(st + c, nx, m) - below(st + c, x, m);
        for (int q = 0; q < k; ++q) r += v;
      }
      x = nx;
    }
    return r;
  }
  __device__ __forceinline__ double stride_sum(const Src& C, int st, int m, int c) const {
    return reg ? stride_sum_t<true>(C, st, m, c) : stride_sum_t<false>(C, st, m, c);
  }
  // Sites past the body (only the rightmost leaf of a locus has them), in order.
  __device__ __forceinline__ double add_tail(const Src& C, int st, int ln, double res) const {
    for (int x = st + ((ln >> 3) << 3); x < st + ln; ++x) res += value_at(C, x);
    return res;
  }
  // Leaf value if it has a closed form (returns false for kRuns leaves).
  __device__ __forceinline__ bool leaf_fast(const Src& C, int st, int ln, double& out) const {
    const int m = ln >> 3;
    double body = 0.0;
    if (m > 0) {
      double F, ps; int plo, phi;
      const int kind = reg ? classify<true>(C, st, m, F, plo, phi, ps)
                           : classify<false>(C, st, m, F, plo, phi, ps);
      if (kind == kRuns) return false;
      body = closed_body(kind, st, m, F, plo, phi, ps);
    }
    out = add_tail(C, st, ln, body);
    return true;
  }
  // All eight stride accumulators of the body [st, st+8m) in one pass over the envelope's
  // runs: a run [x, nx) of value v adds v k_c times to accumulator c, where k_c (its sites
  // of residue c) is kmin or kmin + 1.  Each accumulator still adds its own sites in site
  // order, so the sums are those of stride_sum(); the runs are found once, not per c, and
  // the eight independent chains interleave.
  template <bool REG>
  __device__ __forceinline__ double runs_body(const Src& C, int st, int m) const {
    const int be = st + (m << 3), na = REG ? NREG : ke - kb;
    double r[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) r[c] = 0.0;
    for (int x = st; x < be;) {
      double v = 0.0;
      int nx = be;
#pragma unroll
      for (int i = 0; i < na; ++i) {
        int l, h; double s;
        att<REG>(C, i, l, h, s);
        if (l < h) {
          if (l <= x && x < h) { v = s > v ? s : v; nx = min(nx, h); }
          else if (l > x) nx = min(nx, l);
        }
      }
      if (v > 0.0) {
        int k[8], kmin = m;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          k[c] = below(st + c, nx, m) - below(st + c, x, m);
          kmin = min(kmin, k[c]);
        }
        for (int q = 0; q < kmin; ++q) {
#pragma unroll
          for (int c = 0; c < 8; ++c) r[c] += v;
        }
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (k[c] > kmin) r[c] += v;
      }
      x = nx;
    }
    return leaf_tree(r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
  }
  // Leaf value by one thread (serial path).
  __device__ __forceinline__ double leaf(const Src& C, int st, int ln) const {
    double v;
    if (leaf_fast(C, st, ln, v)) return v;
    const int m = ln >> 3;
    const double body = reg ? runs_body<true>(C, st, m) : runs_body<false>(C, st, m);
    return add_tail(C, st, ln, body);
  }
};
using SegAtt = SegAttT<KeySrc>;

// Exact np.mean of one (clade, locus) site array (orgscorer.py:399-406) by one thread:
// leaves in order, combined on a shift-register stack; 8192-element buffers added from
// 0.0 (numpy NPY_BUFSIZE).  Used for loci too long for the lane-parallel path.
__device__ __forceinline__ double segment_mean(const Contig& C, int g, int kb, int ke) {
  const KeySrc asrc{C.keys, C.alo, C.ahi, C.asc};
  const int n = C.loc_len[g];
  const int4* lv = C.leaves + C.leaf_off[g];
  const int nl = C.leaf_off[g + 1] - C.leaf_off[g];
  const int full_bufs = n / kNpyBuf;
  SegAtt at;
  at.load(asrc, kb, ke);
  SumStack stk;
  double total = 0.0;
  for (int j = 0; j < nl; ++j) {
    const int4 e = lv[j];
    stk.push(at.leaf(asrc, e.x, e.y));
    for (int a = 0; a < e.z; ++a) stk.add_top();
    if (j == nl - 1 || (((j + 1) & 63) == 0 && ((j + 1) >> 6) <= full_bufs)) {
      total += stk.s0;
      stk.s0 = 0.0;
    }
  }
  return total / (double)n;
}

// Lane-parallel site means: a group of gs lanes (8/16/32/64) takes one segment whose locus
// has <= gs leaves in a single numpy buffer; lane i computes leaf i, then the pairwise
// tree is combined bottom-up with lane shuffles following the locus' schedule (lane i
// adds lane j's partial sum when i starts an internal node whose right child starts at
// j), so every addition is numpy's (left + right).  `list` holds the class's segments.
template <int NW>
__device__ __forceinline__ void site_means_grouped(const Contig& C, const int* list, int count, int gs) {
  const KeySrc asrc{C.keys, C.alo, C.ahi, C.asc};
  const int lane = lane_id(), w = wave_id();
  const int per_round = 64 / gs, gi = lane / gs, li = lane % gs;
  for (int base = w * per_round; base < count; base += NW * per_round) {
    const int idx = base + gi;
    const bool has = idx < count;
    const int s = has ? list[idx] : 0;
    const int kb = has ? C.seg_start[s] : 0, ke = has ? C.seg_start[s + 1] : 0;
    const int g = has ? (int)((C.keys[kb] >> 24) & 0xFFFF) : 0;
    const int nl = has ? C.leaf_off[g + 1] - C.leaf_off[g] : 0;
    // this lane's combine schedule: byte d = partner leaf at tree depth d, or -1
    const uint64_t sv = (has && li < nl) ? C.sched[C.sched_off[g] + li] : ~0ull;
    double v = 0.0;
    int st = 0, ln = 0;
    bool runs = false;
    SegAtt at;
    LAP_MARK();
    if (has && li < nl) {
      at.load(asrc, kb, ke);
      const int4 e = C.leaves[C.leaf_off[g] + li];
      st = e.x; ln = e.y;
      LAP_WAIT_LDS();
      LAP(13);
      runs = !at.leaf_fast(asrc, st, ln, v);
      LAP_WAIT_V(v);
    }
    // kRuns leaves, up to 8 at a time: lane octet j takes the j-th such leaf, lane c of
    // the octet its stride accumulator c; the 8 sums are combined with xor shuffles as
    // ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) -- float addition is commutative, so exact.
    uint64_t pend = __ballot(runs);
    while (pend) {
      const int oct = lane >> 3, c = lane & 7;
      uint64_t m = pend;
      for (int k = 0; k < oct && m; ++k) m &= m - 1;
      const int src = m ? __builtin_ctzll(m) : lane;
      const int okb = __shfl(kb, src, 64), oke = __shfl(ke, src, 64);
      const int ost = __shfl(st, src, 64), oln = __shfl(ln, src, 64);
      double r = 0.0;
      if (m) {
        SegAtt a2;
        a2.load(asrc, okb, oke);
        r = a2.stride_sum(asrc, ost, oln >> 3, c);
      }
      r = r + __shfl_xor(r, 1, 64);
      r = r + __shfl_xor(r, 2, 64);
      r = r + __shfl_xor(r, 4, 64);
      const int j = __popcll(pend & ((1ull << lane) - 1ull));
      const double body = __shfl(r, (j & 7) * 8, 64);
      if (runs && j < 8) { v = at.add_tail(asrc, st, ln, body); runs = false; }
      for (int k = 0; k < 8 && pend; ++k) pend &= pend - 1;
    }
    LAP(14);
    const int steps = has ? C.loc_steps[g] : 0;
    int maxsteps = steps;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) maxsteps = max(maxsteps, __shfl_xor(maxsteps, off, 64));
    for (int d = maxsteps - 1; d >= 0; --d) {
      const int src = (d < steps) ? (int)(int8_t)(sv >> (8 * d)) : -1;
      const double o = __shfl(v, src >= 0 ? gi * gs + src : lane, 64);
      if (src >= 0) v = v + o;
    }
    if (has && li == 0) C.S[(int64_t)C.seg_cl[s] * C.G + g] = v / (double)C.loc_len[g];
    LAP(15);
  }
}

// Every pair i < j of potential clades whose "score >= k2" locus masks cover all unmasked
// loci, i.e. crit(i, j) >= k2 (orgscorer.py:606-608, 457-461: min over loci of max(S_i, S_j)
// >= k2 iff each locus has S_i >= k2 or S_j >= k2).  Register-tiled: a wave owns a tile of
// 64*R consecutive j, each lane keeps its R masks in registers; the i masks are loaded 64 at
// a time (one per lane) and broadcast with readlane, so a test costs 3 VALU per 64 pairs
// and mask memory (LDS or the HBM workspace) is read once per tile.  f(i, j) runs on the
// lane that owns j.
// Without masks (MASK = false: more than 64 unmasked loci) `slow(i, j)` decides instead.
template <int NW, bool MASK, class Slow, class F>
__device__ __forceinline__ void for_each_candidate_t(const uint64_t* mask, int Pp, uint64_t full,
                                                     Slow slow, F f) {
  constexpr bool use_mask = MASK;
  constexpr int R = 4;
  const int lane = lane_id(), w = wave_id();
  for (int jb = w * 64 * R; jb < Pp; jb += NW * 64 * R) {
    uint64_t mj[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int j = jb + lane + 64 * r;
      mj[r] = (use_mask && j < Pp) ? mask[j] : 0ull;
    }
    const int iend = min(Pp - 1, jb + 64 * R - 1);   // i < j <= jb + 64R - 1
    for (int ib = 0; ib < iend; ib += 64) {
      const uint64_t mine = (use_mask && ib + lane < iend) ? mask[ib + lane] : 0ull;
      const unsigned lo = (unsigned)mine, hi = (unsigned)(mine >> 32);
      const int kend = min(64, iend - ib);
      for (int k = 0; k < kend; ++k) {
        const uint64_t mi = ((uint64_t)(unsigned)__builtin_amdgcn_readlane((int)hi, k) << 32) |
                            (unsigned)__builtin_amdgcn_readlane((int)lo, k);
        const int i = ib + k;
        unsigned hits = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int j = jb + lane + 64 * r;
          if (j > i && j < Pp && (use_mask ? (mi | mj[r]) == full : slow(i, j))) hits |= 1u << r;
        }
#pragma unroll 1
        while (hits) {                 // one inlined copy of f (candidates are rare)
          const int r = __builtin_ctz(hits);
          hits &= hits - 1;
          f(i, jb + lane + 64 * r);
        }
      }
    }
  }
}

// Mask classes for large potential sets: potential clades with the same "score >= k2" mask
// are interchangeable for the crit >= k2 test, so the test runs once per pair of classes
// (U^2 / 2 instead of Pp^2 / 2), and only members of passing class pairs are enumerated --
// exactly the same candidate pairs, in a different order (pass 1 picks by (rank, pair
// index), pass 2 only aggregates, so the order does not matter).
constexpr int kClsMin = 512;            // use classes from this many potential clades on
constexpr int kClsMaxU = 2048;          // ... unless the masks are this diverse
constexpr int kClsMaxPairs = 4096;      // ... or this many class pairs pass

__device__ __forceinline__ int64_t cls_bytes(int pmax) {
  int n2 = 1;
  while (n2 < pmax) n2 <<= 1;
  return (int64_t)n2 * 8 + (int64_t)(pmax + 1) * 4 + kClsMaxPairs * 8 + (kClsMaxPairs + 1) * 8 + 64;
}

struct MaskClasses {
  int U, npairs, ib;
  uint64_t* keys;      // (mask << ib | potential index), sorted: classes are runs
  int* cstart;         // [U + 1]
  int2* pairs;         // passing class pairs (a <= b)
  long long* pref;     // [npairs + 1] candidate-count prefix
};

// Builds the classes (block-wide).  Returns false when they would not pay off or fit.
template <int NT>
__device__ __forceinline__ bool build_mask_classes(const Contig& C, Ctl& ctl, int Pp, int Gu, uint64_t full,
                                   MaskClasses& M) {
  const int tid = threadIdx.x;
  int ib = 1;
  while ((1 << ib) < Pp) ++ib;
  if (!C.xws || Pp < kClsMin || Gu + ib > 64 || cls_bytes(Pp) > C.xcap) return false;
  int n2 = 1;
  while (n2 < Pp) n2 <<= 1;
  Arena ar{C.xws, C.xcap, 0};
  M.ib = ib;
  M.keys = ar.take<uint64_t>(n2);
  M.cstart = ar.take<int>(Pp + 1);
  M.pairs = ar.take<int2>(kClsMaxPairs);
  M.pref = ar.take<long long>(kClsMaxPairs + 1);
  for (int t = tid; t < n2; t += NT)
    M.keys[t] = t < Pp ? ((C.mask[t] << ib) | (uint64_t)t) : ~0ull;
  __syncthreads();
  bitonic_sort<NT>(M.keys, n2);
  const int per = (Pp + NT - 1) / NT;
  const int b = min(Pp, tid * per), e = min(Pp, b + per);
  int nc = 0;
  for (int t = b; t < e; ++t)
    if (t == 0 || (M.keys[t] >> ib) != (M.keys[t - 1] >> ib)) ++nc;
  int U;
  int ci = block_scan<NT>(nc, &U, ctl);
  for (int t = b; t < e; ++t)
    if (t == 0 || (M.keys[t] >> ib) != (M.keys[t - 1] >> ib)) M.cstart[ci++] = t;
  if (tid == 0) { M.cstart[U] = Pp; ctl.cnt = 0; }
  __syncthreads();
  M.U = U;
  if (U > kClsMaxU) return false;
  for (int t = tid; t < U * U; t += NT) {
    const int a = t / U, bb = t % U;
    if (a > bb) continue;
    const uint64_t ma = M.keys[M.cstart[a]] >> ib, mb = M.keys[M.cstart[bb]] >> ib;
    if ((ma | mb) != full) continue;
    if (a == bb && M.cstart[a + 1] - M.cstart[a] < 2) continue;
    const int slot = atomicAdd(&ctl.cnt, 1);
    if (slot < kClsMaxPairs) M.pairs[slot] = make_int2(a, bb);
  }
  __syncthreads();
  const int np = ctl.cnt;
  __syncthreads();
  if (np > kClsMaxPairs) return false;
  if (tid == 0) {
    long long acc = 0;
    for (int q = 0; q < np; ++q) {
      M.pref[q] = acc;
      const int2 ab = M.pairs[q];
      const long long na = M.cstart[ab.x + 1] - M.cstart[ab.x];
      const long long nb = M.cstart[ab.y + 1] - M.cstart[ab.y];
      acc += ab.x == ab.y ? na * (na - 1) / 2 : na * nb;
    }
    M.pref[np] = acc;
  }
  __syncthreads();
  M.npairs = np;
  return true;
}

// f(i, j) for every candidate pair i < j of the classes (threads stride the candidates).
template <int NT, class F>
__device__ __forceinline__ void for_each_candidate_cls(const MaskClasses& M, F f) {
  const long long T = M.npairs > 0 ? M.pref[M.npairs] : 0;
  const uint64_t imask = (1ull << M.ib) - 1;
  for (long long x = threadIdx.x; x < T; x += NT) {
    int lo = 0, hi = M.npairs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (M.pref[mid] <= x) lo = mid; else hi = mid - 1;
    }
    const int2 ab = M.pairs[lo];
    const long long y = x - M.pref[lo];
    const int a0 = M.cstart[ab.x], na = M.cstart[ab.x + 1] - a0;
    int u, v;
    if (ab.x == ab.y) {
      // y-th (p, q), p < q, in row-major order: row p starts at p*(2na-p-1)/2
      int plo = 0, phi = na - 2;
      while (plo < phi) {
        const int mid = (plo + phi + 1) >> 1;
        if ((long long)mid * (2 * na - mid - 1) / 2 <= y) plo = mid; else phi = mid - 1;
      }
      const long long rs = (long long)plo * (2 * na - plo - 1) / 2;
      u = a0 + plo;
      v = a0 + plo + 1 + (int)(y - rs);
    } else {
      const int b0 = M.cstart[ab.y], nb = M.cstart[ab.y + 1] - b0;
      u = a0 + (int)(y / nb);
      v = b0 + (int)(y % nb);
    }
    const int i = (int)(M.keys[u] & imask), j = (int)(M.keys[v] & imask);
    f(min(i, j), max(i, j));
  }
}

template <int NW, class Slow, class F>
__device__ __forceinline__ void for_each_candidate(const uint64_t* mask, bool use_mask, int Pp,
                                                   uint64_t full, Slow slow, F f) {
  if (use_mask) for_each_candidate_t<NW, true>(mask, Pp, full, slow, f);
  else for_each_candidate_t<NW, false>(mask, Pp, full, slow, f);
}

// --- two-clade option evaluation (orgscorer.py:511-545, 678-744), one thread ---------
struct OptEval {
  int ok, swapped, dir, same, c1p, c2p;
};

__device__ __forceinline__ uint8_t two_char(const KArgs& K, const Contig& C, int pa, int pb,
                                            bool unk, int g) {
  const DevParams& P = K.p;
  if (C.ign[g]) return '~';
  double s1 = C.S[(int64_t)pa * C.G + g], s2 = C.S[(int64_t)pb * C.G + g];
  double mn = s2 < s1 ? s2 : s1;
  if (mn >= P.k_amb && !unk) return '*';
  if (s1 >= P.k2) return 'A';
  if (s2 >= P.k2) return 'B';
  return '!';
}

__device__ __forceinline__ OptEval eval_two(const KArgs& K, const Contig& C, int Pcount, int pa, int pb,
                            const uint8_t* best, uint8_t* out) {
  const DevParams& P = K.p;
  const int G = C.G;
  const bool unk = C.cl_id[pa] == K.unknown || C.cl_id[pb] == K.unknown;
  OptEval e;
  e.swapped = 0;
  if (G <= 64) {
    // the synteny as four locus masks, built in one pass over the two score rows; the
    // swap rule, the counts, the direction pattern and the sister test are bit operations
    uint64_t mi = 0, mm = 0, ma = 0, mb = 0;         // '~', '*', 'A', 'B' ('!': the rest)
#pragma unroll 8
    for (int g = 0; g < G; ++g) {
      const uint64_t bit = 1ull << g;
      const double s1 = C.S[(int64_t)pa * G + g], s2 = C.S[(int64_t)pb * G + g];
      const double mn = s2 < s1 ? s2 : s1;
      if (C.ign[g]) mi |= bit;
      else if (mn >= P.k_amb && !unk) mm |= bit;
      else if (s1 >= P.k2) ma |= bit;
      else if (s2 >= P.k2) mb |= bit;
    }
    const uint64_t ab = ma | mb;                     // "^[^A]*B" -> swap (:537-540)
    e.swapped = (ab && ((mb >> __builtin_ctzll(ab)) & 1ull)) ? 1 : 0;
    const uint64_t mA = e.swapped ? mb : ma, mB = e.swapped ? ma : mb;
    auto ch = [&](int g) -> uint8_t {
      const uint64_t bit = 1ull << g;
      return (mi & bit) ? '~' : (mm & bit) ? '*' : (mA & bit) ? 'A' : (mB & bit) ? 'B' : '!';
    };
    e.same = 1;
    int64_t tot = 0, amb = 0;
    int state = 0;
    bool dir_ok = true;
    for (int g = 0; g < G; ++g) {
      const uint8_t c = ch(g);
      if (out) out[g] = c;
      if (best && best[g] != c) e.same = 0;
      if (c == 'A' || c == 'B' || c == '*') {
        const int len = C.loc_len[g];
        tot += len;
        if (c == '*') amb += len;
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
    e.c1p = e.swapped ? pb : pa;
    e.c2p = e.swapped ? pa : pb;
    e.ok = 1;
    if ((double)amb / (double)tot > P.amb_frac) e.ok = 0;           // :693-702
    if (P.clade_genes >= 0 && min(nA, nB) < P.clade_genes) e.ok = 0; // :704-708
    const int X = C.cl_id[e.c1p], Y = C.cl_id[e.c2p];
    if (P.clade_leaves >= 0) {                                       // :710-715
      const int64_t lc = e.dir ? K.leaves[Y] : min(K.leaves[X], K.leaves[Y]);
      if (lc < P.clade_leaves) e.ok = 0;
    }
    if (P.sister_on && e.ok) {                                       // :717-744
      const int px = K.parent[X], py = K.parent[Y];
      uint64_t fa = 0, fb = 0;
#pragma unroll 8
      for (int q = 0; q < Pcount; ++q) {
        const int sp = C.sib_of[q];
        if (sp != px && sp != py) continue;
        const int s = C.cl_id[q];
        if (s == X || s == Y) continue;
        uint64_t h;
        if (C.hm) {
          h = C.hm[q];
        } else {
          h = 0;
          for (int g = 0; g < G; ++g)
            if (C.S[(int64_t)q * G + g] >= P.sister_thr) h |= 1ull << g;
        }
        if (sp == px) fb |= h;
        if (sp == py) fa |= h;
      }
      if ((fb & mB) || (!e.dir && (fa & mA))) e.ok = 0;
    }
    return e;
  }
#pragma unroll 8
  for (int g = 0; g < G; ++g) {  // "^[^A]*B" -> swap (orgscorer.py:537-540)
    uint8_t c = two_char(K, C, pa, pb, unk, g);
    if (c == 'A') break;
    if (c == 'B') { e.swapped = 1; break; }
  }
  auto fin = [&](int g) -> uint8_t {
    uint8_t c = two_char(K, C, pa, pb, unk, g);
    if (e.swapped) c = (c == 'A') ? 'B' : (c == 'B' ? 'A' : c);
    return c;
  };
  int state = 0, nA = 0, nB = 0;
  uint64_t mA = 0, mB = 0;       // loci with synteny A / B (sister masks, G <= 64)
  bool dir_ok = true;
  int64_t tot = 0, amb = 0;
  e.same = 1;
#pragma unroll 8
  for (int g = 0; g < G; ++g) {
    uint8_t c = fin(g);
    if (out) out[g] = c;
    if (best && best[g] != c) e.same = 0;
    const int len = C.loc_len[g];
    if (c == 'A') { ++nA; tot += len; mA |= 1ull << (g & 63); }
    else if (c == 'B') { ++nB; tot += len; mB |= 1ull << (g & 63); }
    else if (c == '*') { tot += len; amb += len; }
    if (c != '~') {  // "^A+B+A+$" on synteny without '~' (orgscorer.py:542)
      if (state == 0) { if (c == 'A') state = 1; else dir_ok = false; }
      else if (state == 1) { if (c == 'B') state = 2; else if (c != 'A') dir_ok = false; }
      else if (state == 2) { if (c == 'A') state = 3; else if (c != 'B') dir_ok = false; }
      else { if (c != 'A') dir_ok = false; }
    }
  }
  e.dir = (dir_ok && state == 3) ? 1 : 0;
  e.c1p = e.swapped ? pb : pa;
  e.c2p = e.swapped ? pa : pb;
  e.ok = 1;
  // check_ambiguous_fraction (:693-702): total > 0 whenever crit >= k2 on >= 1 locus
  if ((double)amb / (double)tot > P.amb_frac) e.ok = 0;
  // check_clade_genes (:704-708)
  if (P.clade_genes >= 0 && min(nA, nB) < P.clade_genes) e.ok = 0;
  const int X = C.cl_id[e.c1p], Y = C.cl_id[e.c2p];
  // check_clade_leaves (:710-715); recip = clade2 when the direction is known
  if (P.clade_leaves >= 0) {
    int64_t lc = e.dir ? K.leaves[Y] : min(K.leaves[X], K.leaves[Y]);
    if (lc < P.clade_leaves) e.ok = 0;
  }
  // check_sister_penalty (:717-744): fail iff a checked locus has a present sister clade
  // (other than the pair) scoring >= threshold there
  if (P.sister_on && e.ok && C.hm) {
    // per-clade threshold masks: one pass over the clades instead of one per locus
    const int px = K.parent[X], py = K.parent[Y];
    uint64_t fa = 0, fb = 0;
    for (int q = 0; q < Pcount; ++q) {
      const int sp = C.sib_of[q];
      if (sp != px && sp != py) continue;
      const int s = C.cl_id[q];
      if (s == X || s == Y) continue;
      const uint64_t h = C.hm[q];
      if (sp == px) fb |= h;
      if (sp == py) fa |= h;
    }
    if ((fb & mB) || (!e.dir && (fa & mA))) e.ok = 0;
  } else if (P.sister_on && e.ok) {
    const int px = K.parent[X], py = K.parent[Y];
    for (int g = 0; g < G && e.ok; ++g) {
      uint8_t c = fin(g);
      int need;
      if (c == 'B') need = px;
      else if (c == 'A' && !e.dir) need = py;
      else continue;
      for (int q = 0; q < Pcount; ++q) {
        if (C.sib_of[q] != need) continue;
        const int s = C.cl_id[q];
        if (s == X || s == Y) continue;
        if (C.S[(int64_t)q * G + g] >= P.sister_thr) { e.ok = 0; break; }
      }
    }
  }
  return e;
}

__device__ __forceinline__ double pair_rank(const Contig& C, int pa, int pb, int Gu) {
  const double* ra = C.S + (int64_t)pa * C.G;
  const double* rb = C.S + (int64_t)pb * C.G;
  return np_sum(Gu, [&](int u) {
           double a = ra[C.um[u]], b = rb[C.um[u]];
           return a < b ? b : a;
         }) / (double)Gu;
}

__device__ __forceinline__ double pair_crit(const Contig& C, int pa, int pb, int Gu) {
  const double* ra = C.S + (int64_t)pa * C.G;
  const double* rb = C.S + (int64_t)pb * C.G;
  double m = 0.0;
#pragma unroll 8
  for (int u = 0; u < Gu; ++u) {
    double a = ra[C.um[u]], b = rb[C.um[u]];
    double x = a < b ? b : a;
    m = (u == 0 || x < m) ? x : m;
  }
  return m;
}

// One roll-up level after the gene-score matrix exists (orgscorer.py:407-429, 566-583):
// maxes and weak loci, explain_one (+ meld_one), explain_two (+ LGT filters, meld_two).
// C.S holds Pn x G scores with rows in clade-id order (C.cl_id), ctl.p_unk the row of
// "Unknown" when it is present.  Writes the contig's result when an explanation is found.
// Returns kDecDone (contig finished), kDecStop (no explanation possible: unclassified, with
// ctl.status possibly set) or kDecRaise (roll up one taxonomy level and try again).
constexpr int kDecDone = 0, kDecStop = 1, kDecRaise = 2, kDecNext = 3;

// Maxes over known clades and weak loci (orgscorer.py:407-429); sets ctl.Gu / C.um /
// C.ign / ctl.root_present.  kDecNext: go on to explain_one.
template <int NT>
__device__ __forceinline__ int decide_prologue(const KArgs& K, const Contig& C, Ctl& ctl, int Pn,
                                               bool& first) {
  const int tid = threadIdx.x;
  const DevParams& P = K.p;
  const int G = C.G;
  if (NT == 64 && G <= 64) {
    // one wave, lane g owns locus g: a column max over the clade rows (no atomics, no
    // index division), the unmasked-locus list by ballot
    bool root = false;
    for (int p = tid; p < Pn; p += NT) root |= C.cl_id[p] == K.root;
    double m = 0.0;
    if (tid < G)
#pragma unroll 8
      for (int p = 0; p < Pn; ++p) {
        const double v = C.S[(int64_t)p * G + tid];
        if (C.cl_id[p] != K.unknown && v > m) m = v;
      }
    int ig = 0;
    if (tid < G) {
      if (P.weak == 0) ig = !(m >= P.kmin);
      else if (P.weak == 2) C.S[(int64_t)ctl.p_unk * G + tid] = 1.0 - m;
      C.ign[tid] = ig;
      C.maxes[tid] = dbits(m);
    }
    const uint64_t keep = __ballot(tid < G && !ig);
    if (tid < G && !ig) C.um[__popcll(keep & ((1ull << tid) - 1ull))] = tid;
    const bool any_root = __ballot(root) != 0ull;
    if (tid == 0) {
      ctl.root_present = any_root ? 1 : 0;
      ctl.Gu = __popcll(keep);
      ctl.all_ignored = keep == 0ull;
    }
    __syncthreads();
  } else {
  for (int g = tid; g < G; g += NT) C.maxes[g] = 0;
  if (tid == 0) ctl.root_present = 0;
  __syncthreads();
  for (int p = tid; p < Pn; p += NT)
    if (C.cl_id[p] == K.root) ctl.root_present = 1;
  // ---- per-locus max over known clades, weak loci (:407-427) ----------------------
  for (int i = tid; i < Pn * G; i += NT) {
    if (C.cl_id[i / G] == K.unknown) continue;
    const double v = C.S[i];
    if (v > 0.0) atomicMax((unsigned long long*)&C.maxes[i % G], dbits(v));
  }
  __syncthreads();
  if (tid == 0) {
    int Gu = 0;
    for (int g = 0; g < G; ++g) {
      const double m = __longlong_as_double((long long)C.maxes[g]);
      int ig = 0;
      if (P.weak == 0) ig = !(m >= P.kmin);
      else if (P.weak == 2) C.S[(int64_t)ctl.p_unk * G + g] = 1.0 - m;
      C.ign[g] = ig;
      if (!ig) C.um[Gu++] = g;
    }
    ctl.Gu = Gu;
    ctl.all_ignored = (Gu == 0);
  }
  __syncthreads();
  }
  STAMP(9);
  const int Gu = ctl.Gu;
  if (first) {
    first = false;
    if (ctl.all_ignored) return kDecDone;   // skipped contig (orgscorer.py:959) -> unclassified
  }
  if (Gu == 0) {                   // np.min of an empty array upstream
    if (tid == 0) ctl.status = WF_E_EMPTYMASK;
    __syncthreads();
    return kDecStop;
  }

  return kDecNext;
}

// explain_one + meld_one (orgscorer.py:585-597, 621-631).  kDecDone when a one-clade
// explanation was written, kDecNext otherwise.
template <int NT>
__device__ __forceinline__ int decide_one(const KArgs& K, const Contig& C, Ctl& ctl, int c, int Pn,
                                          int iteration, int64_t pair_evals) {
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, w = wave_id();
  const DevParams& P = K.p;
  const int G = C.G;
  const int Gu = ctl.Gu;
  (void)w; (void)NW;
  // ================= explain_one (orgscorer.py:585-597) ============================
  {
    // Contig.score (:447-461) for one clade: (min, np.mean) of its masked row
    auto score_one = [&](int p, double& crit, double& rank) {
      const double* row = C.S + (int64_t)p * G;
      crit = row[C.um[0]];
      for (int u = 1; u < Gu; ++u) { const double v = row[C.um[u]]; crit = v < crit ? v : crit; }
      rank = np_sum(Gu, [&](int u) { return row[C.um[u]]; }) / (double)Gu;
    };
    double br = -__builtin_inf();
    long long bk = -1;
    for (int p = tid; p < Pn; p += NT) {
      double crit, rank;
      score_one(p, crit, rank);
      if (crit >= P.k1 && better(rank, p, br, bk)) { br = rank; bk = p; }
    }
    block_argmax<NT>(br, bk, ctl);
    STAMP(10);
    if (bk >= 0) {
      // meld_one (:621-631): options within --range of the best
      const int bp = (int)bk;
      if (tid == 0) ctl.cnt = 0;
      __syncthreads();
      if (P.dis1 == 1) {
        for (int p = tid; p < Pn; p += NT) {
          double crit, rank;
          score_one(p, crit, rank);
          if (crit >= P.k1 && (br - rank) <= P.range) {
            const int slot = atomicAdd(&ctl.cnt, 1);
            C.mem1[slot] = C.cl_id[p];
          }
        }
      }
      __syncthreads();
      const int m = ctl.cnt;
      if (P.dis1 == 1 && m == 0) {   // negative --range: get_lca() of nothing raises upstream
        if (tid == 0) K.status[c] = WF_E_BADINPUT;
        return kDecDone;
      }
      const int lca = (P.dis1 == 1) ? block_lca(K, C.mem1, m, ctl) : C.cl_id[bp];
      for (int i = tid; i < m; i += NT) K.meld[C.mbase + i] = C.mem1[i];
      for (int g = tid; g < G; g += NT) {  // set_synteny_one (:495-509) of the best
        const double s = C.S[(int64_t)bp * G + g];
        K.syn[C.l0 + g] = C.ign[g] ? '~' : (s >= P.k1 ? 'A' : '!');
      }
      STAMP(11);
      if (tid == 0) {
        double crit, rank;
        score_one(bp, crit, rank);
        K.call[c] = WF_CALL_NO_LGT;
        K.crit[c] = crit;
        K.rank[c] = br;
        K.c1[c] = lca;
        K.c2[c] = -1;
        K.nm1[c] = m;
        K.iters[c] = (int16_t)iteration;
        K.pair_evals[c] = pair_evals;
      }
      return kDecDone;
    }
  }

  return kDecNext;
}

// explain_two + LGT filters + meld_two (orgscorer.py:599-619, 633-744), then the roll-up
// decision: kDecDone (written), kDecStop (unclassified) or kDecRaise.
template <int NT>
__device__ __forceinline__ int decide_two(const KArgs& K, const Contig& C, Ctl& ctl, int c, int Pn,
                                          int iteration, int64_t& pair_evals) {
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, w = wave_id();
  const DevParams& P = K.p;
  const int G = C.G;
  const int Gu = ctl.Gu;
  (void)w; (void)NW;
  // ================= explain_two (orgscorer.py:599-619) ============================
  {
    // potential clades: max over ALL loci >= k2 (:603-605)
    int flag_local = 0;
    const int per = (Pn + NT - 1) / NT;
    const int pb0 = min(Pn, tid * per), pe0 = min(Pn, pb0 + per);
    auto potential = [&](int p) -> bool {
      const double* row = C.S + (int64_t)p * G;
      double mx = row[0];
#pragma unroll 8
      for (int g = 1; g < G; ++g) mx = row[g] > mx ? row[g] : mx;
      return mx >= P.k2;
    };
    for (int p = pb0; p < pe0; ++p) flag_local += potential(p) ? 1 : 0;
    int Pp;
    int pos = block_scan<NT>(flag_local, &Pp, ctl);
    for (int p = pb0; p < pe0; ++p)
      if (potential(p)) C.pot[pos++] = p;
    pair_evals += (int64_t)Pp * (Pp - 1) / 2;
    if (threadIdx.x == 0) note_ppot(K, c, iteration, Pp);
    STAMP_SYNC();
    STAMP(16);
    const bool use_mask = Gu <= 64;
    const uint64_t full = (Gu >= 64) ? ~0ull : ((1ull << Gu) - 1ull);
    __syncthreads();
    if (use_mask) {
      for (int i = tid; i < Pp; i += NT) {
        const double* row = C.S + (int64_t)C.pot[i] * G;
        uint64_t m = 0;
#pragma unroll 8
        for (int u = 0; u < Gu; ++u)
          if (row[C.um[u]] >= P.k2) m |= 1ull << u;
        C.mask[i] = m;
      }
    }
    __syncthreads();
    STAMP(17);
    // pass 1: best pair over all pairs clade1 < clade2 (name order == index order)
    double br = -__builtin_inf();
    long long bk = -1;
    auto candidate = [&](int i, int j) -> bool {
      if (use_mask) return (C.mask[i] | C.mask[j]) == full;
      return pair_crit(C, C.pot[i], C.pot[j], Gu) >= P.k2;
    };
    auto consider = [&](int i, int j) {
      const double r = pair_rank(C, C.pot[i], C.pot[j], Gu);
      const long long key = (long long)i * Pp + j;
      if (better(r, key, br, bk)) { br = r; bk = key; }
    };
    MaskClasses mcls;
    const bool use_cls = use_mask && build_mask_classes<NT>(C, ctl, Pp, Gu, full, mcls);
    if (use_cls) for_each_candidate_cls<NT>(mcls, consider);
    else for_each_candidate<NW>(C.mask, use_mask, Pp, full, candidate, consider);
    block_argmax<NT>(br, bk, ctl);
    STAMP(18);
    bool have_ok = false;
    if (bk >= 0) {
      if (P.sister_on) {                 // sister checks read listed parents per clade
        for (int q = tid; q < Pn; q += NT) {
          C.sib_of[q] = K.sibp[C.cl_id[q]];
          if (C.hm) {
            const double* row = C.S + (int64_t)q * G;
            uint64_t m = 0;
            for (int g = 0; g < G; ++g)
              if (row[g] >= P.sister_thr) m |= 1ull << g;
            C.hm[q] = m;
          }
        }
        __syncthreads();
      }
      const int bi = (int)(bk / Pp), bj = (int)(bk % Pp);
      for (int i = tid; i < (Pn + 31) / 32; i += NT) { C.bm1[i] = 0; C.bm2[i] = 0; }
      if (tid == 0) {
        OptEval e = eval_two(K, C, Pn, C.pot[bi], C.pot[bj], nullptr, C.best_syn);
        ctl.best_ok = e.ok; ctl.best_dir = e.dir;
        ctl.best_c1p = e.c1p; ctl.best_c2p = e.c2p;
        ctl.best_crit = pair_crit(C, C.pot[bi], C.pot[bj], Gu);
        ctl.n_in = 0; ctl.all_ok = 1; ctl.all_same = 1;
      }
      __syncthreads();
      // pass 2: options within --range of the best get the LGT filters (:636-639)
      auto within = [&](int i, int j) {
        const double r = pair_rank(C, C.pot[i], C.pot[j], Gu);
        if (!((br - r) <= P.range)) return;
        OptEval e = eval_two(K, C, Pn, C.pot[i], C.pot[j], C.best_syn, nullptr);
        atomicAdd(&ctl.n_in, 1);
        if (!e.ok) atomicAnd(&ctl.all_ok, 0);
        if (!e.same) atomicAnd(&ctl.all_same, 0);
        atomicOr(&C.bm1[e.c1p >> 5], 1u << (e.c1p & 31));
        atomicOr(&C.bm2[e.c2p >> 5], 1u << (e.c2p & 31));
      };
      if (use_cls) for_each_candidate_cls<NT>(mcls, within);
      else for_each_candidate<NW>(C.mask, use_mask, Pp, full, candidate, within);
      __syncthreads();
      // meld_two (:640-669)
      if (tid == 0) {
        int kind;   // 0 none, 1 best as is, 2 meld, 3 unchecked best, 4 upstream crash
        if (ctl.n_in == 0) kind = (P.dis2 == 0) ? 3 : (P.dis2 == 1 ? 0 : 4);  // --range < 0
        else if (ctl.n_in == 1 || P.dis2 == 0) kind = 1;
        else if (P.dis2 == 1) kind = 0;
        else kind = (ctl.all_ok && ctl.all_same) ? 2 : 0;
        ctl.res_kind = kind;
        ctl.cnt = 0;
        ctl.cnt2 = 0;
      }
      __syncthreads();
      const int kind = ctl.res_kind;
      if (kind == 4) {
        if (tid == 0) K.status[c] = WF_E_BADINPUT;
        return kDecDone;
      }
      int lca1 = -1, lca2v = -1, m1 = 0, m2 = 0;
      if (kind == 2) {
        for (int p = tid; p < Pn; p += NT) {
          if (C.bm1[p >> 5] & (1u << (p & 31))) C.mem1[atomicAdd(&ctl.cnt, 1)] = C.cl_id[p];
          if (C.bm2[p >> 5] & (1u << (p & 31))) C.mem2[atomicAdd(&ctl.cnt2, 1)] = C.cl_id[p];
        }
        __syncthreads();
        m1 = ctl.cnt;
        m2 = ctl.cnt2;
        __syncthreads();
        lca1 = block_lca(K, C.mem1, m1, ctl);
        lca2v = block_lca(K, C.mem2, m2, ctl);
        bool keep = true;
        if (!P.allow_lca) {
          const int nl = lca2(K, lca1, lca2v);
          keep = !(nl == lca1 || nl == lca2v);
        }
        have_ok = keep;   // melded options are all OK
      } else if (kind == 1) {
        have_ok = ctl.best_ok != 0;
      } else if (kind == 3) {
        have_ok = true;
      }
      if (have_ok) {
        for (int g = tid; g < G; g += NT) K.syn[C.l0 + g] = C.best_syn[g];
        if (kind == 2) {
          for (int i = tid; i < m1; i += NT) K.meld[C.mbase + i] = C.mem1[i];
          for (int i = tid; i < m2; i += NT) K.meld[C.mbase + m1 + i] = C.mem2[i];
        }
        if (tid == 0) {
          K.call[c] = WF_CALL_LGT;
          K.crit[c] = ctl.best_crit;
          K.rank[c] = br;
          K.dir[c] = (int8_t)ctl.best_dir;
          K.c1[c] = (kind == 2) ? lca1 : C.cl_id[ctl.best_c1p];
          K.c2[c] = (kind == 2) ? lca2v : C.cl_id[ctl.best_c2p];
          K.nm1[c] = (kind == 2) ? m1 : 0;
          K.nm2[c] = (kind == 2) ? m2 : 0;
          K.iters[c] = (int16_t)iteration;
          K.pair_evals[c] = pair_evals;
        }
        return kDecDone;
      }
    }
  }

  STAMP(12);
  __syncthreads();
  return (Pn == 0 || ctl.root_present) ? kDecStop : kDecRaise;
}

template <int NT>
__device__ __forceinline__ int decide_level(const KArgs& K, const Contig& C, Ctl& ctl, int c, int Pn,
                                            int iteration, bool& first, int64_t& pair_evals) {
  int d = decide_prologue<NT>(K, C, ctl, Pn, first);
  if (d != kDecNext) return d;
  d = decide_one<NT>(K, C, ctl, c, Pn, iteration, pair_evals);
  if (d != kDecNext) return d;
  return decide_two<NT>(K, C, ctl, c, Pn, iteration, pair_evals);
}

}  // namespace
}  // namespace wf
