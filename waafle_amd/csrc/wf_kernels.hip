// HIP kernels for the waafle_orgscorer contig-scoring hot path (gfx950 / MI355X), fused
// form: one workgroup scores one contig end to end -- hit->locus attachment
// (orgscorer.py:359-392), per-(clade, locus) site-score means in numpy's exact pairwise
// float64 order (:394-429), the taxonomy roll-up loop (:431-445, :566-583), the one-clade
// search + meld (:585-597, :621-631) and the all-pairs two-clade search + meld + LGT
// filters (:599-619, :633-744).  The per-contig state lives in LDS (k_contig_lds);
// contigs whose state does not fit are re-run by k_contig_big with the same code on a
// per-workgroup HBM workspace slot.
#include "wf_device.h"

namespace wf {

namespace {

// --------------------------------------------------------------------------
// the contig workgroup
// --------------------------------------------------------------------------

template <int NT, bool BIG>
__device__ __forceinline__ void process_contig(const KArgs& K, int c, char* abase, int64_t acap, Ctl& ctl) {
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x;
  const DevParams& P = K.p;
  const int nsys = K.n_sys;
  Contig C;
  C.h0 = K.hit_off[c];
  C.H = (int)(K.hit_off[c + 1] - C.h0);
  C.l0 = K.loc_off[c];
  C.G = (int)(K.loc_off[c + 1] - C.l0);
  C.mbase = 2 * C.h0 + 2 * (int64_t)c;
  const int H = C.H, G = C.G;

  if (tid == 0) {
    ctl.overflow = 0; ctl.status = 0; ctl.need = 0;
    K.call[c] = WF_CALL_UNCLASSIFIED;
    K.crit[c] = 0.0; K.rank[c] = 0.0; K.c1[c] = -1; K.c2[c] = -1; K.dir[c] = 0;
    K.iters[c] = 0; K.nm1[c] = 0; K.nm2[c] = 0; K.pair_evals[c] = 0; K.status[c] = 0;
    K.need[c] = 0;
  }
  for (int i = tid; i < G * nsys; i += NT) K.annot[C.l0 * nsys + i] = -1;
  if (H == 0 || G == 0) return;  // never evaluated -> unclassified (orgscorer.py:959)
  STAMP_INIT();
  STAMP(20);
  Arena ar{abase, acap, 0};
  // ---- loci and their pairwise-sum leaf tables ------------------------------------
  C.loc_lo = ar.take<int>(G);
  C.loc_len = ar.take<int>(G);
  C.loc_st = ar.take<int>(G);
  C.leaf_off = ar.take<int>(G + 1);
  C.loc_grp = ar.take<int>(G);
  C.loc_steps = ar.take<int>(G);
  C.sched_off = ar.take<int>(G + 1);
  C.maxes = ar.take<uint64_t>(G);
  C.ign = ar.take<int>(G);
  C.um = ar.take<int>(G);
  if (!ar.fits()) {
    if (tid == 0) { ctl.overflow = 1; ctl.need = ar.used + 4096; }
    __syncthreads();
    return;
  }
  for (int g = tid; g < G; g += NT) {
    int s = K.lstart[C.l0 + g], e = K.lend[C.l0 + g];
    int lo = min(s, e), hi = max(s, e);
    C.loc_lo[g] = lo;
    C.loc_len[g] = hi - lo + 1;                 // len(Locus) (utils.py:321-322)
    C.loc_st[g] = K.lstrand[C.l0 + g];
    const int n = hi - lo + 1, nl = leaves_of_length(n);
    C.leaf_off[g + 1] = nl;
    // lane-group size for the parallel site means (0: serial path)
    const int gs = (n > kNpyBuf || nl > kGroupMax) ? 0 : nl <= 8 ? 8 : nl <= 16 ? 16 : nl <= 32 ? 32 : 64;
    C.loc_grp[g] = gs;
    C.sched_off[g + 1] = gs;
  }
  __syncthreads();
  if (tid == 0) {
    C.leaf_off[0] = 0;
    C.sched_off[0] = 0;
    for (int g = 0; g < G; ++g) {
      C.leaf_off[g + 1] += C.leaf_off[g];
      C.sched_off[g + 1] += C.sched_off[g];
    }
    ctl.cnt = C.leaf_off[G];
    ctl.cnt2 = C.sched_off[G];
  }
  __syncthreads();
  STAMP(0);
  const int NL = ctl.cnt, NSCH = ctl.cnt2;
  C.leaves = ar.take<int4>(NL);
  C.sched = ar.take<uint64_t>(NSCH);

  // ---- attach hits to loci: count (orgscorer.py:359-369, :559-564; utils.py:487-500) ---
  auto attaches = [&](int qlo, int qhi, int hs, int g) -> bool {
    if (P.stranded && hs != C.loc_st[g]) return false;
    const int l1 = C.loc_lo[g], l2 = l1 + C.loc_len[g] - 1;
    if (l1 > qhi || qlo > l2) return 0.0 >= P.min_overlap;   // calc_overlap -> int 0
    const int ov = min(qhi, l2) - max(qlo, l1) + 1;
    const int den = min(qhi - qlo + 1, l2 - l1 + 1);
    return (double)ov / (double)den >= P.min_overlap;
  };
  int local = 0;
  for (int i = tid; i < H; i += NT) {
    const int64_t hi_ = C.h0 + i;
    if (!(K.scov[hi_] >= P.min_scov)) continue;
    const int qlo = K.qlo[hi_], qhi = K.qhi[hi_], hs = K.hstrand[hi_];
    for (int g = 0; g < G; ++g) local += attaches(qlo, qhi, hs, g) ? 1 : 0;
  }
  int A;
  int off = block_scan<NT>(local, &A, ctl);
  STAMP(1);
  const int virt = (P.weak == 2) ? 1 : 0;       // assign-unknown adds "Unknown" (:416-418)
  const int A1 = A + virt;
  C.alo = ar.take<int>(A);
  C.ahi = ar.take<int>(A);
  C.aloc = ar.take<int>(A);
  C.acl = ar.take<int>(A);
  C.asc = ar.take<double>(A);
  const int64_t persist_mark = ar.used;
  C.ahit = ar.take<int>(A);                     // temporary: annotations only
  if (!ar.fits() || A >= (1 << 24) || G >= kLocVirtual) {
    if (tid == 0) {
      ctl.overflow = 1;
      ctl.status = (A >= (1 << 24) || G >= kLocVirtual) ? WF_E_BADINPUT : 0;
      ctl.need = ar.used + (int64_t)A1 * (48 + 8 * G) + 8192;
    }
    __syncthreads();
    return;
  }
  // leaf tables and combine schedules
  for (int i = tid; i < NSCH; i += NT) C.sched[i] = ~0ull;
  __syncthreads();
  for (int g = tid; g < G; g += NT) {
    int k = C.leaf_off[g];
    const int n = C.loc_len[g], gs = C.loc_grp[g];
    int8_t* sch = gs ? reinterpret_cast<int8_t*>(C.sched + C.sched_off[g]) : nullptr;
    for (int o = 0; o < n; o += kNpyBuf)
      k += gen_leaves(o, min(kNpyBuf, n - o), C.leaves + k, sch, gs);
    int steps = 0;
    for (int d = 0; d < kMaxDepth && sch; ++d)
      for (int i = 0; i < gs; ++i)
        if (sch[i * 8 + d] >= 0) steps = d + 1;
    C.loc_steps[g] = steps;
  }
  // ---- attach: fill, with the python-slice site range (orgscorer.py:371-382) ---------
  for (int i = tid; i < H; i += NT) {
    const int64_t hi_ = C.h0 + i;
    if (!(K.scov[hi_] >= P.min_scov)) continue;
    const int qlo = K.qlo[hi_], qhi = K.qhi[hi_], hs = K.hstrand[hi_];
    for (int g = 0; g < G; ++g) {
      if (!attaches(qlo, qhi, hs, g)) continue;
      const int len = C.loc_len[g], l1 = C.loc_lo[g];
      const int h1 = max(0, qlo - l1);
      const int h2 = min(len - 1, qhi - l1);
      const int start = min(h1, len);
      int stop = h2 + 1;                         // site[h1:h2+1], python slice rules
      if (stop < 0) { stop += len; if (stop < 0) stop = 0; }
      C.alo[off] = start;
      C.ahi[off] = stop;                         // empty when stop <= start
      C.ahit[off] = i;
      C.aloc[off] = g;
      C.acl[off] = K.taxon[hi_];
      C.asc[off] = K.score[hi_];
      ++off;
    }
  }
  __syncthreads();
  STAMP(2);

  // ---- annotation transfer (orgscorer.py:383-392): per (locus, system) the last hit in
  // file order whose score equals the running maximum >= threshold ---------------------
  if (nsys > 0) {
    ar.used = persist_mark + (int64_t)A * 4 + 16;
    uint64_t* abest = ar.take<uint64_t>((int64_t)G * nsys);
    int* aidx = ar.take<int>((int64_t)G * nsys);
    if (!ar.fits()) {
      if (tid == 0) { ctl.overflow = 1; ctl.need = ar.used + (int64_t)A1 * (48 + 8 * G) + 8192; }
      __syncthreads();
      return;
    }
    for (int i = tid; i < G * nsys; i += NT) { abest[i] = 0; aidx[i] = -1; }
    __syncthreads();
    for (int a = tid; a < A; a += NT) {
      const uint32_t m = K.sysmask[C.h0 + C.ahit[a]];
      const double s = C.asc[a];
      if (m == 0 || !(s >= P.annot_ref)) continue;
      for (int b = 0; b < nsys; ++b)
        if (m & (1u << b)) atomicMax((unsigned long long*)&abest[C.aloc[a] * nsys + b], dbits(s));
    }
    __syncthreads();
    for (int a = tid; a < A; a += NT) {
      const uint32_t m = K.sysmask[C.h0 + C.ahit[a]];
      const double s = C.asc[a];
      if (m == 0 || !(s >= P.annot_ref)) continue;
      for (int b = 0; b < nsys; ++b)
        if ((m & (1u << b)) && abest[C.aloc[a] * nsys + b] == dbits(s))
          atomicMax(&aidx[C.aloc[a] * nsys + b], C.ahit[a]);
    }
    __syncthreads();
    for (int i = tid; i < G * nsys; i += NT)
      K.annot[C.l0 * nsys + i] = aidx[i] >= 0 ? (int)(C.h0 + aidx[i]) : -1;
    __syncthreads();
    ar.used = persist_mark;
  }

  // ---- initial jumps (orgscorer.py:955-957) ---------------------------------------
  if (P.jump > 0) {
    for (int a = tid; a < A; a += NT) {
      int x = C.acl[a];
      for (int j = 0; j < P.jump; ++j) x = K.parent[x];
      C.acl[a] = x;
    }
  }
  __syncthreads();
  STAMP(3);

  int iteration = 1;
  bool first = true;
  int64_t pair_evals = 0;

  for (;;) {
    // ================= build the gene-score matrix of this level ===================
    ar.used = persist_mark;
    int npow = 1;
    while (npow < A1) npow <<= 1;
    C.keys = ar.take<uint64_t>(npow);
    C.seg_start = ar.take<int>(A1 + 1);
    C.seg_cl = ar.take<int>(A1 + 1);
    C.sorder = ar.take<int>(A1 + 1);
    const int64_t dead_end = ar.used;             // keys + segments: dead after site means
    C.cl_id = ar.take<int>(A1 + 1);
    if (!ar.fits()) {
      if (tid == 0) { ctl.overflow = 1; ctl.need = ar.used + (int64_t)A1 * (48 + 8 * G) + 8192; }
      __syncthreads();
      return;
    }
    for (int t = tid; t < npow; t += NT) {
      uint64_t key = kKeyPad;
      if (t < A)
        key = ((uint64_t)(uint32_t)C.acl[t] << 40) | ((uint64_t)C.aloc[t] << 24) | (uint64_t)t;
      else if (t < A1)
        key = ((uint64_t)(uint32_t)K.unknown << 40) | ((uint64_t)kLocVirtual << 24) | 0xFFFFFFull;
      C.keys[t] = key;
    }
    __syncthreads();
    STAMP(4);
    bitonic_sort<NT>(C.keys, npow);
    STAMP(5);
    STAMP(21);
    // segments = distinct (clade, locus); clades = distinct clade (sorted = name order)
    {
      const int per = (A1 + NT - 1) / NT;
      const int b = min(A1, tid * per), e = min(A1, b + per);
      int ns = 0, nc = 0;
      for (int t = b; t < e; ++t) {
        const uint64_t k = C.keys[t];
        if (t == 0 || (k >> 24) != (C.keys[t - 1] >> 24)) ++ns;
        if (t == 0 || (k >> 40) != (C.keys[t - 1] >> 40)) ++nc;
      }
      int ps, pc, ts, tc;
      block_scan2<NT>(ns, nc, &ps, &pc, &ts, &tc, ctl);
      int si = ps - 1, ci = pc - 1;
      for (int t = b; t < e; ++t) {
        const uint64_t k = C.keys[t];
        if (t == 0 || (k >> 40) != (C.keys[t - 1] >> 40)) {
          ++ci;
          const int id = (int)(k >> 40);
          C.cl_id[ci] = id;
          if (id == K.unknown) ctl.p_unk = ci;
        }
        if (t == 0 || (k >> 24) != (C.keys[t - 1] >> 24)) {
          ++si;
          C.seg_start[si] = t;
          C.seg_cl[si] = ci;
        }
      }
      if (tid == 0) {
        ctl.S_n = ts;
        ctl.P = tc;
        C.seg_start[ts] = A1;
      }
    }
    __syncthreads();
    STAMP(6);
    const int S_n = ctl.S_n, Pn = ctl.P;
    C.S = ar.take<double>((int64_t)Pn * G);
    {
      // explain scratch: overlays the sort keys / segment tables when they fit (both are
      // dead once the gene-score matrix exists), else follows S
      Arena ex{abase, acap, persist_mark};
      const int64_t need_ex = (int64_t)Pn * 24 + 8 * ((Pn + 31) / 32) + G + 7 * 16;
      if (persist_mark + need_ex > dead_end) ex.used = ar.used;
      C.pot = ex.take<int>(Pn);
      C.mask = ex.take<uint64_t>(Pn);
      C.mem1 = ex.take<int>(Pn);
      C.mem2 = ex.take<int>(Pn);
      C.bm1 = ex.take<unsigned>((Pn + 31) / 32);
      C.bm2 = ex.take<unsigned>((Pn + 31) / 32);
      C.best_syn = ex.take<uint8_t>(G);
      C.sib_of = ex.take<int>(Pn);
      if (ex.used > ar.used) ar.used = ex.used;
    }
    if (!ar.fits()) {
      if (tid == 0) { ctl.overflow = 1; ctl.need = ar.used + (int64_t)A1 * (48 + 8 * G) + 8192; }
      __syncthreads();
      return;
    }
    for (int i = tid; i < Pn * G; i += NT) C.S[i] = 0.0;
    __syncthreads();
    STAMP(7);
    // ---- site-score means (orgscorer.py:399-406) -------------------------------------
    // segments grouped by their locus' lane-group class (8/16/32/64 lanes; 4 = serial)
    if (tid < 5) ctl.cls_cnt[tid] = 0;
    __syncthreads();
    auto seg_class = [&](int s) -> int {
      const int g = (int)((C.keys[C.seg_start[s]] >> 24) & 0xFFFF);
      if (g == kLocVirtual) return -1;
      const int gs = C.loc_grp[g];
      return gs == 8 ? 0 : gs == 16 ? 1 : gs == 32 ? 2 : gs == 64 ? 3 : 4;
    };
    for (int s = tid; s < S_n; s += NT) {
      const int cls = seg_class(s);
      if (cls >= 0) atomicAdd(&ctl.cls_cnt[cls], 1);
    }
    __syncthreads();
    if (tid == 0) {
      int acc = 0;
      for (int q = 0; q < 5; ++q) { ctl.cls_off[q] = acc; acc += ctl.cls_cnt[q]; ctl.cls_cnt[q] = 0; }
    }
    __syncthreads();
    for (int s = tid; s < S_n; s += NT) {
      const int cls = seg_class(s);
      if (cls >= 0) C.sorder[ctl.cls_off[cls] + atomicAdd(&ctl.cls_cnt[cls], 1)] = s;
    }
    __syncthreads();
    STAMP(22);
    for (int q = 0; q < 4; ++q) {
      site_means_grouped<NW>(C, C.sorder + ctl.cls_off[q], ctl.cls_cnt[q], 8 << q);
      STAT(27 + q, ctl.cls_cnt[q]);
      STAMP_SYNC();
      STAMP(23 + q);
    }
    STAT(31, ctl.cls_cnt[4]);
    for (int i = tid; i < ctl.cls_cnt[4]; i += NT) {
      const int s = C.sorder[ctl.cls_off[4] + i];
      const int kb = C.seg_start[s], ke = C.seg_start[s + 1];
      const int g = (int)((C.keys[kb] >> 24) & 0xFFFF);
      C.S[(int64_t)C.seg_cl[s] * G + g] = segment_mean(C, g, kb, ke);
    }
    __syncthreads();
    STAMP(8);
    {
      const int dec = decide_level<NT>(K, C, ctl, c, Pn, iteration, first, pair_evals);
      if (dec == kDecDone) return;
      if (dec == kDecStop) break;
    }
    for (int a = tid; a < A; a += NT) C.acl[a] = K.parent[C.acl[a]];
    ++iteration;
    if (iteration > kMaxIter) {
      if (tid == 0) ctl.status = WF_E_RUNAWAY;
      __syncthreads();
      break;
    }
    __syncthreads();
  }
  // unclassified after evaluation
  if (tid == 0) {
    K.iters[c] = (int16_t)min(iteration, 32767);
    K.pair_evals[c] = pair_evals;
    K.status[c] = ctl.status;
  }
}

}  // namespace

// Tiers 1 and 2: state in LDS.  Tier 1 (LIST = false) runs one workgroup per contig of the
// batch -- NT = 64, one wave per contig, suits the small contigs of typical assemblies.
// Tier 2 (LIST = true, NT = 256, a larger LDS budget) drains the contigs tier 1 could not
// hold, as a persistent grid over the work list.  Whatever still does not fit goes to the
// tier-3 HBM-workspace kernel.
// Kernel arguments live in device memory (one KArgs block per tier, uploaded per call) so
// every field is a scalar load; a by-value struct argument whose address is taken would be
// copied to scratch and re-read from there on every access.
#ifndef WF_LDS_OCC
#define WF_LDS_OCC 2   // min waves per SIMD the register allocator must leave room for
#endif
template <int NT, bool LIST>
__global__ __launch_bounds__(NT, WF_LDS_OCC) void k_contig_lds(const KArgs* __restrict__ kp) {
  const KArgs& K = *kp;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ Ctl ctl;
  const int count = LIST ? *K.work_count : K.n_contigs;
  for (int i = blockIdx.x; i < count; i += gridDim.x) {
    const int c = LIST ? K.work_list[i] : i;
    process_contig<NT, false>(K, c, smem, K.lds_bytes, ctl);
    __syncthreads();
    if (threadIdx.x == 0 && ctl.overflow) {
      if (ctl.status != 0) {
        K.status[c] = ctl.status;
      } else {
        const int slot = atomicAdd(K.ovf_count, 1);
        K.ovf_list[slot] = c;
        K.status[c] = kPending;
        K.need[c] = ctl.need;
      }
    }
    __syncthreads();
  }
}

// Tier 3: the same contig program on a per-workgroup HBM workspace slot.
__global__ __launch_bounds__(kBlock, 2) void k_contig_big(const KArgs* __restrict__ kp) {
  const KArgs& K = *kp;
  __shared__ Ctl ctl;
  const int count = *K.work_count;
  char* base = K.big_ws + (int64_t)blockIdx.x * K.slot_bytes;
  for (int i = blockIdx.x; i < count; i += gridDim.x) {
    const int c = K.work_list[i];
    process_contig<kBlock, true>(K, c, base, K.slot_bytes, ctl);
    __syncthreads();
    if (threadIdx.x == 0 && ctl.overflow) {
      K.status[c] = ctl.status != 0 ? ctl.status : WF_E_NOMEM;
      K.need[c] = ctl.need;
    }
    __syncthreads();
  }
}

template <int NT, bool LIST>
static hipError_t launch_lds(const KArgs& k, const KArgs* dk, int grid, hipStream_t s) {
  if (k.lds_bytes > 64 * 1024) {
    static hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&k_contig_lds<NT, LIST>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 1024);
    if (attr != hipSuccess) return attr;
  }
  hipLaunchKernelGGL((k_contig_lds<NT, LIST>), dim3(grid), dim3(NT), (size_t)k.lds_bytes, s, dk);
  return hipGetLastError();
}

hipError_t launch_lds_kernel(const KArgs& k, const KArgs* dk, hipStream_t s) {
  if (k.n_contigs <= 0) return hipSuccess;
  if (k.lds_threads == 64) return launch_lds<64, false>(k, dk, k.n_contigs, s);
  if (k.lds_threads == 128) return launch_lds<128, false>(k, dk, k.n_contigs, s);
  return launch_lds<256, false>(k, dk, k.n_contigs, s);
}

hipError_t launch_lds_list_kernel(const KArgs& k, const KArgs* dk, int grid, hipStream_t s) {
  if (grid <= 0) return hipSuccess;
  return launch_lds<256, true>(k, dk, grid, s);
}

hipError_t launch_big_kernel(const KArgs* dk, int grid, hipStream_t s) {
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_contig_big, dim3(grid), dim3(kBlock), 0, s, dk);
  return hipGetLastError();
}

#ifdef WF_STAMPS
extern "C" int wf_stamps_read(unsigned long long* out, int n) {
  if (n > 32) n = 32;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * n) == hipSuccess
             ? 0 : -2;
}
extern "C" int wf_stamps_reset(void) {
  unsigned long long z[32] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof z) == hipSuccess ? 0 : -2;
}
#endif
}  // namespace wf
