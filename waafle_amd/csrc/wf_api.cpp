// C-ABI of libwaafle_hip.so (see include/waafle_hip.h): context/device management,
// taxonomy upload, batch staging and the staged kernel sequence (wf_staged.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "waafle_hip.h"
#include "wf_internal.h"

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

struct wf_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  // taxonomy
  int32_t tax_n = 0, root = -1, unknown = -1;
  DevBuf parent, depth, sibp, leaves, lin;
  // genecaller staging (host-resident calls)
  DevBuf gc_off, gc_qlo, gc_qhi, gc_strand, gc_scov, gc_ngenes, gc_gstart, gc_gstop, gc_gstrand, gc_status;
  // waafle_junctions staging and scratch
  DevBuf jn_site_off, jn_loc_off, jn_loc_contig, jn_lstart, jn_lend, jn_pc, jn_m1s, jn_m1e, jn_m2s, jn_m2e;
  DevBuf jn_diff, jn_cov, jn_prefix, jn_hits, jn_lhits, jn_c1, jn_c2, jn_cj, jn_ratio, jn_tmp;
  DevBuf jn_pfirst, jn_pmask, jn_ovf;
  bool have_lin = false;
  int64_t lds_bytes = 24 * 1024;   // decision arena per workgroup (wf_set_lds_bytes)
  // staging for host-resident batches
  DevBuf b_hit_off, b_qlo, b_qhi, b_taxon, b_hstrand, b_score, b_scov, b_sysmask;
  DevBuf b_loc_off, b_lstart, b_lend, b_lstrand, b_hkey;
  DevBuf r_call, r_crit, r_rank, r_c1, r_c2, r_dir, r_iters, r_syn, r_nm1, r_nm2, r_meld,
      r_annot, r_pairs, r_status, r_need, r_ppot;
  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, int>> ev_lds;   // indices into ev_pool (one pair per pass)
  int64_t launches = 0;
  bool lds_set = false;            // wf_set_lds_bytes called: also the staged decision arena
  int mode = WF_MODE_LEVEL0;       // wf_set_mode
  int sparse_big = 3;              // wf_set_option(WF_OPT_SPARSE_BIG)
  int64_t att_limit = (int64_t(1) << 31) - 1;   // wf_set_option(WF_OPT_ATT_LIMIT)
  int64_t dump_cap = 0;            // wf_set_option(WF_OPT_DUMP_CAP), 0: the default size
  int triage = 1;                  // wf_set_option(WF_OPT_TRIAGE)
  wf::StagedState* staged = nullptr;
  // --write-details
  bool details_on = false;
  wf::DetailsSink det;
  std::vector<int32_t> d_eval_contig, d_eval_level, d_level, d_contig, d_clade, d_locus, d_nspan, d_spans;
  std::vector<double> d_mean;
  std::vector<int64_t> d_span_off;
};

namespace {

int fail(wf_ctx* ctx, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  return code;
}

#define HIP_TRY(ctx, expr)                                                             \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail(ctx, WF_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));       \
  } while (0)

int ensure(wf_ctx* ctx, DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.bytes >= bytes) return WF_OK;
  if (b.p) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
  }
  size_t want = std::max(bytes, b.bytes * 3 / 2);
  hipError_t e = hipMalloc(&b.p, want);
  if (e != hipSuccess) {
    e = hipMalloc(&b.p, bytes);
    want = bytes;
  }
  if (e != hipSuccess)
    return fail(ctx, WF_E_HIP, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
  b.bytes = want;
  return WF_OK;
}

void release(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

template <class T>
int upload(wf_ctx* ctx, DevBuf& b, const T* src, int64_t count, const T** dst) {
  int rc = ensure(ctx, b, sizeof(T) * (size_t)std::max<int64_t>(count, 1));
  if (rc) return rc;
  if (count > 0) {
    hipError_t e = hipMemcpyAsync(b.p, src, sizeof(T) * count, hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) return fail(ctx, WF_E_HIP, "H2D copy failed: %s", hipGetErrorString(e));
  }
  *dst = static_cast<const T*>(b.p);
  return WF_OK;
}

template <class T>
int alloc_out(wf_ctx* ctx, DevBuf& b, int64_t count, T** dst) {
  int rc = ensure(ctx, b, sizeof(T) * (size_t)std::max<int64_t>(count, 1));
  if (rc) return rc;
  *dst = static_cast<T*>(b.p);
  return WF_OK;
}

template <class T>
int download(wf_ctx* ctx, T* host, const T* dev, int64_t count) {
  if (count <= 0) return WF_OK;
  hipError_t e = hipMemcpyAsync(host, dev, sizeof(T) * count, hipMemcpyDeviceToHost, ctx->stream);
  if (e != hipSuccess) return fail(ctx, WF_E_HIP, "D2H copy failed: %s", hipGetErrorString(e));
  return WF_OK;
}

int take_event_pair(wf_ctx* ctx, std::vector<std::pair<int, int>>& list) {
  for (int k = 0; k < 2; ++k) {
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) return -1;
    ctx->ev_pool.push_back(ev);
  }
  int a = (int)ctx->ev_pool.size() - 2;
  list.push_back({a, a + 1});
  return a;
}

wf::DevParams derive_params(const wf_params& p) {
  wf::DevParams d{};
  d.k1 = p.k1;
  d.k2 = p.k2;
  d.kmin = std::min(p.k1, p.k2);   // orgscorer.py:338-339
  const double kmax = std::max(p.k1, p.k2);
  const double eps = 1e-6;          // c_eps, orgscorer.py:58
  d.k_amb = p.ambiguous_threshold == 0 ? eps : (p.ambiguous_threshold == 1 ? d.kmin : kmax);
  d.sister_thr = p.sister_penalty == 1 ? kmax : d.kmin;   // lenient: max, strict: min
  d.sister_on = p.sister_penalty != 0;
  d.annot_ref = p.annotation_threshold == 0 ? eps : (p.annotation_threshold == 1 ? d.kmin : kmax);
  d.range = p.range;
  d.min_overlap = p.min_overlap;
  d.min_scov = p.min_scov;
  d.amb_frac = p.ambiguous_fraction;
  d.dis1 = p.disambiguate_one;
  d.dis2 = p.disambiguate_two;
  d.jump = p.jump_taxonomy > 0 ? p.jump_taxonomy : 0;
  d.allow_lca = p.allow_lca;
  d.clade_genes = p.clade_genes;
  d.clade_leaves = p.clade_leaves;
  d.weak = p.weak_loci;
  d.stranded = p.stranded;
  return d;
}

}  // namespace

extern "C" {

int wf_abi_version(void) { return WF_ABI_VERSION; }

int wf_device_count(int* count) {
  if (!count) return WF_E_BADINPUT;
  hipError_t e = hipGetDeviceCount(count);
  if (e != hipSuccess) {
    *count = 0;
    return WF_E_HIP;
  }
  return WF_OK;
}

int wf_init(int device, wf_ctx** out) {
  if (!out) return WF_E_BADINPUT;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return WF_E_HIP;
  if (device < 0 || device >= n) return WF_E_BADINPUT;
  wf_ctx* ctx = new (std::nothrow) wf_ctx();
  if (!ctx) return WF_E_NOMEM;
  ctx->device = device;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return WF_E_HIP;
  }
  ctx->stream = ctx->own_stream;
  *out = ctx;
  return WF_OK;
}

void wf_free(wf_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  DevBuf* bufs[] = {&ctx->parent, &ctx->depth, &ctx->sibp, &ctx->leaves, &ctx->lin, &ctx->gc_off,
                    &ctx->gc_qlo, &ctx->gc_qhi, &ctx->gc_strand, &ctx->gc_scov, &ctx->gc_ngenes,
                    &ctx->gc_gstart, &ctx->gc_gstop, &ctx->gc_gstrand, &ctx->gc_status,
                    &ctx->jn_site_off, &ctx->jn_loc_off, &ctx->jn_loc_contig, &ctx->jn_lstart,
                    &ctx->jn_lend, &ctx->jn_pc, &ctx->jn_m1s, &ctx->jn_m1e, &ctx->jn_m2s,
                    &ctx->jn_m2e, &ctx->jn_diff, &ctx->jn_cov, &ctx->jn_prefix, &ctx->jn_hits,
                    &ctx->jn_lhits, &ctx->jn_c1, &ctx->jn_c2, &ctx->jn_cj, &ctx->jn_ratio,
                    &ctx->jn_tmp, &ctx->jn_pfirst, &ctx->jn_pmask, &ctx->jn_ovf,
                    &ctx->b_hit_off, &ctx->b_qlo, &ctx->b_qhi, &ctx->b_taxon, &ctx->b_hstrand,
                    &ctx->b_score, &ctx->b_scov, &ctx->b_sysmask, &ctx->b_hkey, &ctx->b_loc_off,
                    &ctx->b_lstart, &ctx->b_lend, &ctx->b_lstrand, &ctx->r_call, &ctx->r_crit,
                    &ctx->r_rank, &ctx->r_c1, &ctx->r_c2, &ctx->r_dir, &ctx->r_iters,
                    &ctx->r_syn, &ctx->r_nm1, &ctx->r_nm2, &ctx->r_meld, &ctx->r_annot,
                    &ctx->r_pairs, &ctx->r_status, &ctx->r_need, &ctx->r_ppot};
  for (DevBuf* b : bufs) release(*b);
  if (ctx->staged) wf::staged_destroy(ctx->staged);
  for (hipEvent_t ev : ctx->ev_pool) (void)hipEventDestroy(ev);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  delete ctx;
}

const char* wf_last_error(const wf_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int wf_set_stream(wf_ctx* ctx, void* hip_stream) {
  if (!ctx) return WF_E_BADINPUT;
  ctx->stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->own_stream;
  return WF_OK;
}

int wf_set_lds_bytes(wf_ctx* ctx, int64_t bytes) {
  if (!ctx) return WF_E_BADINPUT;
  if (bytes < 4096 || bytes > 152 * 1024)
    return fail(ctx, WF_E_BADINPUT, "LDS budget %lld out of [4096, 155648]", (long long)bytes);
  ctx->lds_bytes = bytes;
  ctx->lds_set = true;
  return WF_OK;
}

int wf_set_mode(wf_ctx* ctx, int mode) {
  if (!ctx) return WF_E_BADINPUT;
  if (mode != WF_MODE_STAGED && mode != WF_MODE_LEVEL0 && mode != WF_MODE_WAVES)
    return fail(ctx, WF_E_BADINPUT, "mode must be WF_MODE_LEVEL0 (2), WF_MODE_WAVES (3) or WF_MODE_STAGED (0)");
  ctx->mode = mode;
  return WF_OK;
}

int wf_set_option(wf_ctx* ctx, int option, int64_t value) {
  if (!ctx) return WF_E_BADINPUT;
  switch (option) {
    case WF_OPT_SPARSE_BIG:
      // (0 and 1, the dense decision forms for <= 63 loci, are retired: round 4)
      if (value < 2 || value > 3) return fail(ctx, WF_E_BADINPUT, "WF_OPT_SPARSE_BIG is 2 or 3");
      ctx->sparse_big = (int)value;
      return WF_OK;
    case WF_OPT_ATT_LIMIT:
      if (value < 1 || value > (int64_t(1) << 31) - 1)
        return fail(ctx, WF_E_BADINPUT, "WF_OPT_ATT_LIMIT %lld out of [1, 2^31 - 1]", (long long)value);
      ctx->att_limit = value;
      return WF_OK;
    case WF_OPT_WAVE_TWO:        // (0, the round-3 hand-over flow, retired in ABI 6)
      if (value != 1) return fail(ctx, WF_E_BADINPUT, "WF_OPT_WAVE_TWO is 1 (0 is retired)");
      return WF_OK;
    case WF_OPT_DUMP_CAP:
      if (value < 0 || value > (int64_t(1) << 31) - 4096)
        return fail(ctx, WF_E_BADINPUT, "WF_OPT_DUMP_CAP %lld out of [0, 2^31 - 4096]", (long long)value);
      ctx->dump_cap = value;
      return WF_OK;
    case WF_OPT_TRIAGE:
      if (value < 0 || value > 1) return fail(ctx, WF_E_BADINPUT, "WF_OPT_TRIAGE is 0 or 1");
      ctx->triage = (int)value;
      return WF_OK;
    default:
      return fail(ctx, WF_E_BADINPUT, "unknown option %d", option);
  }
}

int wf_set_taxonomy(wf_ctx* ctx, const wf_taxonomy* t) {
  if (!ctx || !t) return WF_E_BADINPUT;
  if (t->n <= 0 || !t->parent || !t->depth || !t->sib_parent || !t->leaf_count)
    return fail(ctx, WF_E_BADINPUT, "taxonomy arrays missing");
  if (t->n >= (1 << 24)) return fail(ctx, WF_E_BADINPUT, "more than 2^24-1 taxonomy names");
  if (t->root < 0 || t->root >= t->n || t->unknown < 0 || t->unknown >= t->n)
    return fail(ctx, WF_E_BADINPUT, "root/unknown ids out of range");
  for (int32_t i = 0; i < t->n; ++i) {   // parent ids valid; depth consistent with parents
    const int32_t p = t->parent[i];
    if (p < 0 || p >= t->n) return fail(ctx, WF_E_BADINPUT, "parent id out of range at %d", i);
    if (i == t->root ? t->depth[i] != 0 : t->depth[i] != t->depth[p] + 1)
      return fail(ctx, WF_E_BADINPUT, "depth inconsistent with parent at %d", i);
  }
  (void)hipSetDevice(ctx->device);
  const int32_t *dp, *dd, *ds;
  const int64_t* dl;
  int rc;
  if ((rc = upload(ctx, ctx->parent, t->parent, t->n, &dp)) ||
      (rc = upload(ctx, ctx->depth, t->depth, t->n, &dd)) ||
      (rc = upload(ctx, ctx->sibp, t->sib_parent, t->n, &ds)) ||
      (rc = upload(ctx, ctx->leaves, t->leaf_count, t->n, &dl)))
    return rc;
  // lineage rows (utils.py:392-399 as a table): LCA becomes one row compare instead of a
  // parent walk of dependent loads
  int32_t max_depth = 0;
  for (int32_t i = 0; i < t->n; ++i) max_depth = std::max(max_depth, t->depth[i]);
  ctx->have_lin = max_depth < wf::kLin;
  if (ctx->have_lin) {
    std::vector<int32_t> lin((size_t)t->n * wf::kLin, -1);
    std::vector<int32_t> order(t->n);
    for (int32_t i = 0; i < t->n; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(),
                     [&](int32_t a, int32_t b) { return t->depth[a] < t->depth[b]; });
    for (int32_t i : order) {
      int32_t* row = &lin[(size_t)i * wf::kLin];
      if (i != t->root) std::copy_n(&lin[(size_t)t->parent[i] * wf::kLin], wf::kLin, row);
      row[t->depth[i]] = i;
    }
    const int32_t* dlin;
    if ((rc = upload(ctx, ctx->lin, lin.data(), (int64_t)lin.size(), &dlin))) return rc;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));   // `lin` is a pageable local
  }
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  ctx->tax_n = t->n;
  ctx->root = t->root;
  ctx->unknown = t->unknown;
  return WF_OK;
}

static int check_batch(wf_ctx* ctx, const wf_batch* b, const wf_params* p, const wf_result* r) {
  if (!b || !p || !r) return fail(ctx, WF_E_BADINPUT, "null batch/params/result");
  if (ctx->tax_n <= 0) return fail(ctx, WF_E_STATE, "wf_set_taxonomy must precede wf_score");
  if (b->n_contigs < 0 || b->n_hits < 0 || b->n_loci < 0)
    return fail(ctx, WF_E_BADINPUT, "negative sizes");
  if (b->n_systems < 0 || b->n_systems > 32)
    return fail(ctx, WF_E_BADINPUT, "n_systems %d not in [0, 32]", b->n_systems);
  if (b->n_hits >= (int64_t)1 << 31) return fail(ctx, WF_E_BADINPUT, "n_hits must be < 2^31");
  if (b->max_loci >= 0xFFFF) return fail(ctx, WF_E_BADINPUT, "more than 65534 loci in a contig");
  if (p->disambiguate_one < 0 || p->disambiguate_one > 1 || p->disambiguate_two < 0 ||
      p->disambiguate_two > 2 || p->ambiguous_threshold < 0 || p->ambiguous_threshold > 2 ||
      p->sister_penalty < 0 || p->sister_penalty > 2 || p->weak_loci < 0 || p->weak_loci > 2 ||
      p->annotation_threshold < 0 || p->annotation_threshold > 2)
    return fail(ctx, WF_E_BADINPUT, "parameter enum out of range");
  if (b->n_contigs > 0 && (!b->hit_off || !b->loc_off))
    return fail(ctx, WF_E_BADINPUT, "null offsets");
  if (b->n_hits > 0 && (!b->hit_qlo || !b->hit_qhi || !b->hit_taxon || !b->hit_strand ||
                        !b->hit_score || !b->hit_scov || !b->hit_sysmask))
    return fail(ctx, WF_E_BADINPUT, "null hit arrays");
  if (b->n_loci > 0 && (!b->loc_start || !b->loc_end || !b->loc_strand))
    return fail(ctx, WF_E_BADINPUT, "null locus arrays");
  if (!r->call || !r->crit || !r->rank || !r->clade1 || !r->clade2 || !r->direction ||
      !r->iterations || !r->synteny || !r->n_meld1 || !r->n_meld2 || !r->meld ||
      !r->annot_hit || !r->pair_evals || !r->status || !r->need_bytes)
    return fail(ctx, WF_E_BADINPUT, "null result arrays");
  if (!b->device_resident) {   // host batches: validate CSR and ids before any launch
    const int64_t* ho = b->hit_off;
    const int64_t* lo = b->loc_off;
    if (ho[0] != 0 || lo[0] != 0 || ho[b->n_contigs] != b->n_hits || lo[b->n_contigs] != b->n_loci)
      return fail(ctx, WF_E_BADINPUT, "CSR offsets inconsistent with sizes");
    for (int32_t c = 0; c < b->n_contigs; ++c) {
      if (ho[c + 1] < ho[c] || lo[c + 1] < lo[c]) return fail(ctx, WF_E_BADINPUT, "offsets decrease");
      if (ho[c + 1] - ho[c] > b->max_hits || lo[c + 1] - lo[c] > b->max_loci)
        return fail(ctx, WF_E_BADINPUT, "max_hits/max_loci understate contig %d", c);
    }
    for (int64_t i = 0; i < b->n_hits; ++i)
      if (b->hit_taxon[i] < 0 || b->hit_taxon[i] >= ctx->tax_n)
        return fail(ctx, WF_E_BADINPUT, "hit %lld taxon id out of range", (long long)i);
    if (b->hit_key)                // the packed words must say what the arrays say
      for (int64_t i = 0; i < b->n_hits; ++i) {
        const uint32_t k = b->hit_key[i];
        const uint32_t want = (uint32_t)b->hit_taxon[i] | (uint32_t)(b->hit_scov[i] >= p->min_scov) << 24 |
                              (uint32_t)(b->hit_strand[i] == 1) << 25 | (b->hit_sysmask[i] & 63u) << 26;
        if (k != want)
          return fail(ctx, WF_E_BADINPUT, "hit %lld: hit_key 0x%08x, its arrays (min_scov %g) give 0x%08x",
                      (long long)i, k, p->min_scov, want);
      }
  }
  return WF_OK;
}

// The staged sequence on the context stream (wf_staged.hip), bracketed by timing events.
static int run_kernels(wf_ctx* ctx, wf::KArgs& K, const wf_batch* b) {
  K.root = ctx->root;
  K.unknown = ctx->unknown;
  if (!ctx->staged) ctx->staged = wf::staged_create(ctx->device);
  if (ctx->lds_set) wf::staged_set_lds(ctx->staged, ctx->lds_bytes);
  wf::staged_set_level0(ctx->staged, ctx->mode != WF_MODE_STAGED, ctx->mode == WF_MODE_WAVES);
  wf::staged_set_options(ctx->staged, ctx->sparse_big, ctx->att_limit, ctx->dump_cap,
                         ctx->triage);
  std::pair<int, int> el{-1, -1};
  if (ctx->timing) {
    if (take_event_pair(ctx, ctx->ev_lds) < 0) return fail(ctx, WF_E_HIP, "hipEventCreate failed");
    el = ctx->ev_lds.back();
    HIP_TRY(ctx, hipEventRecord(ctx->ev_pool[el.first], ctx->stream));
  }
  std::string err;
  const int rc = wf::staged_score(ctx->staged, K, ctx->tax_n, b->max_loci, b->max_hits, b->n_hits, b->n_loci, ctx->stream,
                                  &err, ctx->details_on ? &ctx->det : nullptr);
  if (rc) return fail(ctx, rc == -1 ? WF_E_BADINPUT : (rc == WF_E_TOOBIG ? WF_E_TOOBIG : WF_E_HIP), "%s", err.c_str());
  HIP_TRY(ctx, wf::finish_ppot(K, ctx->stream));
  if (el.first >= 0) HIP_TRY(ctx, hipEventRecord(ctx->ev_pool[el.second], ctx->stream));
  ++ctx->launches;
  return WF_OK;
}

int wf_score(wf_ctx* ctx, const wf_batch* b, const wf_params* p, wf_result* r) {
  if (!ctx) return WF_E_BADINPUT;
  int rc = check_batch(ctx, b, p, r);
  if (rc) return rc;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  wf::KArgs K{};
  K.n_contigs = b->n_contigs;
  K.n_sys = b->n_systems;
  K.parent = static_cast<const int32_t*>(ctx->parent.p);
  K.depth = static_cast<const int32_t*>(ctx->depth.p);
  K.sibp = static_cast<const int32_t*>(ctx->sibp.p);
  K.leaves = static_cast<const int64_t*>(ctx->leaves.p);
  K.lin = ctx->have_lin ? static_cast<const int32_t*>(ctx->lin.p) : nullptr;
  K.p = derive_params(*p);
  const int64_t N = b->n_contigs, NH = b->n_hits, NL = b->n_loci;
  const int64_t n_meld = 2 * NH + 2 * N, n_annot = NL * b->n_systems;

  if (b->device_resident) {
    K.hit_off = b->hit_off; K.qlo = b->hit_qlo; K.qhi = b->hit_qhi; K.taxon = b->hit_taxon;
    K.hstrand = b->hit_strand; K.score = b->hit_score; K.scov = b->hit_scov;
    K.sysmask = b->hit_sysmask; K.loc_off = b->loc_off; K.lstart = b->loc_start;
    K.lend = b->loc_end; K.lstrand = b->loc_strand; K.hkey = b->hit_key;
    K.call = r->call; K.crit = r->crit; K.rank = r->rank; K.c1 = r->clade1; K.c2 = r->clade2;
    K.dir = r->direction; K.iters = r->iterations; K.syn = r->synteny; K.nm1 = r->n_meld1;
    K.nm2 = r->n_meld2; K.meld = r->meld; K.annot = r->annot_hit; K.pair_evals = r->pair_evals;
    K.status = r->status; K.need = r->need_bytes; K.ppot = r->ppot_sum;
    return run_kernels(ctx, K, b);
  }

  // host-resident: stage, run, copy back
  if ((rc = upload(ctx, ctx->b_hit_off, b->hit_off, N + 1, &K.hit_off)) ||
      (rc = upload(ctx, ctx->b_qlo, b->hit_qlo, NH, &K.qlo)) ||
      (rc = upload(ctx, ctx->b_qhi, b->hit_qhi, NH, &K.qhi)) ||
      (rc = upload(ctx, ctx->b_taxon, b->hit_taxon, NH, &K.taxon)) ||
      (rc = upload(ctx, ctx->b_hstrand, b->hit_strand, NH, &K.hstrand)) ||
      (rc = upload(ctx, ctx->b_score, b->hit_score, NH, &K.score)) ||
      (rc = upload(ctx, ctx->b_scov, b->hit_scov, NH, &K.scov)) ||
      (rc = upload(ctx, ctx->b_sysmask, b->hit_sysmask, NH, &K.sysmask)) ||
      (rc = upload(ctx, ctx->b_loc_off, b->loc_off, N + 1, &K.loc_off)) ||
      (rc = upload(ctx, ctx->b_lstart, b->loc_start, NL, &K.lstart)) ||
      (rc = upload(ctx, ctx->b_lend, b->loc_end, NL, &K.lend)) ||
      (rc = upload(ctx, ctx->b_lstrand, b->loc_strand, NL, &K.lstrand)))
    return rc;
  K.hkey = nullptr;
  if (b->hit_key && (rc = upload(ctx, ctx->b_hkey, b->hit_key, NH, &K.hkey))) return rc;
  if ((rc = alloc_out(ctx, ctx->r_call, N, &K.call)) ||
      (rc = alloc_out(ctx, ctx->r_crit, N, &K.crit)) ||
      (rc = alloc_out(ctx, ctx->r_rank, N, &K.rank)) ||
      (rc = alloc_out(ctx, ctx->r_c1, N, &K.c1)) || (rc = alloc_out(ctx, ctx->r_c2, N, &K.c2)) ||
      (rc = alloc_out(ctx, ctx->r_dir, N, &K.dir)) ||
      (rc = alloc_out(ctx, ctx->r_iters, N, &K.iters)) ||
      (rc = alloc_out(ctx, ctx->r_syn, NL, &K.syn)) ||
      (rc = alloc_out(ctx, ctx->r_nm1, N, &K.nm1)) ||
      (rc = alloc_out(ctx, ctx->r_nm2, N, &K.nm2)) ||
      (rc = alloc_out(ctx, ctx->r_meld, n_meld, &K.meld)) ||
      (rc = alloc_out(ctx, ctx->r_annot, n_annot, &K.annot)) ||
      (rc = alloc_out(ctx, ctx->r_pairs, N, &K.pair_evals)) ||
      (rc = alloc_out(ctx, ctx->r_status, N, &K.status)) ||
      (rc = alloc_out(ctx, ctx->r_need, N, &K.need)))
    return rc;
  K.ppot = nullptr;
  if (r->ppot_sum && (rc = alloc_out(ctx, ctx->r_ppot, N, &K.ppot))) return rc;
  if ((rc = run_kernels(ctx, K, b))) return rc;
  if ((rc = download(ctx, r->status, K.status, N)) || (rc = download(ctx, r->need_bytes, K.need, N)))
    return rc;
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));

  if ((rc = download(ctx, r->call, K.call, N)) || (rc = download(ctx, r->crit, K.crit, N)) ||
      (rc = download(ctx, r->rank, K.rank, N)) || (rc = download(ctx, r->clade1, K.c1, N)) ||
      (rc = download(ctx, r->clade2, K.c2, N)) || (rc = download(ctx, r->direction, K.dir, N)) ||
      (rc = download(ctx, r->iterations, K.iters, N)) ||
      (rc = download(ctx, r->synteny, K.syn, NL)) || (rc = download(ctx, r->n_meld1, K.nm1, N)) ||
      (rc = download(ctx, r->n_meld2, K.nm2, N)) || (rc = download(ctx, r->meld, K.meld, n_meld)) ||
      (rc = download(ctx, r->annot_hit, K.annot, n_annot)) ||
      (rc = download(ctx, r->pair_evals, K.pair_evals, N)))
    return rc;
  if (K.ppot && (rc = download(ctx, r->ppot_sum, K.ppot, N))) return rc;
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  for (int32_t c = 0; c < b->n_contigs; ++c)
    if (r->status[c] != 0)
      return fail(ctx, r->status[c], "contig %d failed with status %d", c, r->status[c]);
  return WF_OK;
}

int wf_pack_hit_keys(int64_t n_hits, const int32_t* taxon, const int8_t* strand, const double* scov,
                     const uint32_t* sysmask, double min_scov, uint32_t* out) {
  if (n_hits < 0 || (n_hits > 0 && (!taxon || !strand || !scov || !sysmask || !out))) return WF_E_BADINPUT;
  for (int64_t i = 0; i < n_hits; ++i) {
    if (taxon[i] < 0 || taxon[i] >= (1 << 24) || (strand[i] != 0 && strand[i] != 1)) return WF_E_BADINPUT;
    out[i] = (uint32_t)taxon[i] | (uint32_t)(scov[i] >= min_scov) << 24 | (uint32_t)(strand[i] == 1) << 25 |
             (sysmask[i] & 63u) << 26;
  }
  return WF_OK;
}

int wf_genecall(wf_ctx* ctx, const wf_gc_batch* b, const wf_gc_params* p, wf_gc_result* r) {
  if (!ctx) return WF_E_BADINPUT;
  if (!b || !p || !r) return fail(ctx, WF_E_BADINPUT, "null batch/params/result");
  if (b->n_groups < 0 || b->n_hits < 0) return fail(ctx, WF_E_BADINPUT, "negative sizes");
  if (!b->hit_off || (b->n_hits > 0 && (!b->hit_qlo || !b->hit_qhi || !b->hit_strand || !b->hit_scov)))
    return fail(ctx, WF_E_BADINPUT, "null hit arrays");
  if (!r->n_genes || !r->gene_start || !r->gene_stop || !r->gene_strand)
    return fail(ctx, WF_E_BADINPUT, "null result arrays");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  const int64_t G = b->n_groups, NH = b->n_hits;
  if (G == 0) return WF_OK;
  // largest group (LDS capacity of the kernel): from the offsets, on the host
  std::vector<int64_t> off;
  const int64_t* hoff = b->hit_off;
  if (b->device_resident) {
    off.resize(G + 1);
    HIP_TRY(ctx, hipMemcpyAsync(off.data(), b->hit_off, sizeof(int64_t) * (G + 1), hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    hoff = off.data();
  }
  if (hoff[0] != 0 || hoff[G] != NH) return fail(ctx, WF_E_BADINPUT, "hit_off must span [0, n_hits]");
  int64_t mx = 0;
  for (int64_t g = 0; g < G; ++g) {
    if (hoff[g + 1] < hoff[g]) return fail(ctx, WF_E_BADINPUT, "hit_off decreases at group %lld", (long long)g);
    mx = std::max(mx, hoff[g + 1] - hoff[g]);
  }
  constexpr int64_t kCapMax = 4096;
  wf::GcArgs a{};
  a.n_groups = (int)G;
  a.cap = 64;
  while (a.cap < std::min(mx, kCapMax)) a.cap <<= 1;
  a.min_overlap = p->min_overlap;
  a.min_scov = p->min_scov;
  a.min_gene_length = p->min_gene_length;
  int rc;
  if (b->device_resident) {
    a.hit_off = b->hit_off; a.qlo = b->hit_qlo; a.qhi = b->hit_qhi; a.strand = b->hit_strand;
    a.scov = b->hit_scov;
    a.n_genes = r->n_genes; a.gene_start = r->gene_start; a.gene_stop = r->gene_stop;
    a.gene_strand = r->gene_strand;
  } else {
    if ((rc = upload(ctx, ctx->gc_off, b->hit_off, G + 1, &a.hit_off)) ||
        (rc = upload(ctx, ctx->gc_qlo, b->hit_qlo, NH, &a.qlo)) ||
        (rc = upload(ctx, ctx->gc_qhi, b->hit_qhi, NH, &a.qhi)) ||
        (rc = upload(ctx, ctx->gc_strand, b->hit_strand, NH, &a.strand)) ||
        (rc = upload(ctx, ctx->gc_scov, b->hit_scov, NH, &a.scov)) ||
        (rc = alloc_out(ctx, ctx->gc_ngenes, G, &a.n_genes)) ||
        (rc = alloc_out(ctx, ctx->gc_gstart, NH, &a.gene_start)) ||
        (rc = alloc_out(ctx, ctx->gc_gstop, NH, &a.gene_stop)) ||
        (rc = alloc_out(ctx, ctx->gc_gstrand, NH, &a.gene_strand)))
      return rc;
  }
  if ((rc = alloc_out(ctx, ctx->gc_status, G, &a.status))) return rc;
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, ctx->device) == hipSuccess) cus = prop.multiProcessorCount;
  HIP_TRY(ctx, wf::launch_genecall(a, cus, ctx->stream));
  std::vector<int32_t> status(G);
  if ((rc = download(ctx, status.data(), a.status, G))) return rc;
  if (!b->device_resident) {
    if ((rc = download(ctx, r->n_genes, a.n_genes, G)) ||
        (rc = download(ctx, r->gene_start, a.gene_start, NH)) ||
        (rc = download(ctx, r->gene_stop, a.gene_stop, NH)) ||
        (rc = download(ctx, r->gene_strand, a.gene_strand, NH)))
      return rc;
  }
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  for (int64_t g = 0; g < G; ++g)
    if (status[g] != 0)
      return fail(ctx, WF_E_NOMEM, "contig group %lld has more than %lld intervals", (long long)g,
                  (long long)kCapMax);
  return WF_OK;
}

int wf_junctions(wf_ctx* ctx, const wf_jn_batch* b, const wf_jn_params* p, wf_jn_result* r) {
  if (!ctx) return WF_E_BADINPUT;
  if (!b || !p || !r) return fail(ctx, WF_E_BADINPUT, "null batch/params/result");
  if (b->n_contigs < 0 || b->n_pairs < 0 || b->n_loci < 0) return fail(ctx, WF_E_BADINPUT, "negative sizes");
  if (b->device_resident) return fail(ctx, WF_E_BADINPUT, "wf_junctions takes host arrays");
  if (b->n_contigs > 0 && (!b->contig_length || !b->loc_off))
    return fail(ctx, WF_E_BADINPUT, "null contig arrays");
  if (b->n_loci > 0 && (!b->loc_start || !b->loc_end)) return fail(ctx, WF_E_BADINPUT, "null locus arrays");
  if (b->n_pairs > 0 && (!b->pair_contig || !b->m1_start || !b->m1_end || !b->m2_start || !b->m2_end))
    return fail(ctx, WF_E_BADINPUT, "null pair arrays");
  if (!r->junction_hits || !r->coverage_gene1 || !r->coverage_gene2 || !r->coverage_junction || !r->ratio)
    return fail(ctx, WF_E_BADINPUT, "null result arrays");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  const int64_t N = b->n_contigs, NL = b->n_loci, NP = b->n_pairs;
  if (N == 0) return WF_OK;
  // host-side layout: site offsets (len + 1 slots per contig), locus -> contig, validation
  std::vector<int64_t> site_off(N + 1, 0);
  std::vector<int32_t> loc_contig((size_t)std::max<int64_t>(NL, 1), 0);
  if (b->loc_off[0] != 0 || b->loc_off[N] != NL) return fail(ctx, WF_E_BADINPUT, "loc_off must span [0, n_loci]");
  int forward = 1;
  for (int64_t c = 0; c < N; ++c) {
    if (b->contig_length[c] < 0) return fail(ctx, WF_E_BADINPUT, "negative contig length");
    site_off[c + 1] = site_off[c] + b->contig_length[c] + 1;
    if (b->loc_off[c + 1] < b->loc_off[c]) return fail(ctx, WF_E_BADINPUT, "loc_off decreases");
    for (int64_t l = b->loc_off[c]; l < b->loc_off[c + 1]; ++l) {
      loc_contig[l] = (int32_t)c;
      if (b->loc_start[l] > b->loc_end[l]) forward = 0;
      if (l > b->loc_off[c] && b->loc_start[l] < b->loc_start[l - 1])
        return fail(ctx, WF_E_BADINPUT, "loci of contig %lld are not sorted by start", (long long)c);
    }
  }
  const int64_t S = site_off[N];
  if (S >= ((int64_t)1 << 31) - 1) return fail(ctx, WF_E_BADINPUT, "contigs longer than 2^31 sites in total");
  for (int64_t i = 0; i < NP; ++i)
    if (b->pair_contig[i] < 0 || b->pair_contig[i] >= N)
      return fail(ctx, WF_E_BADINPUT, "pair %lld contig out of range", (long long)i);
  wf::JnArgs a{};
  a.n_contigs = (int)N;
  // the early exit past the pair's right end holds only while a disjoint locus misses
  // (overlap 0 < min_sites); with --min-overlap-sites <= 0 every locus is hit (:277-286)
  a.loc_forward = forward && p->min_overlap_sites > 0;
  a.n_pairs = NP;
  a.n_loci = NL;
  a.n_sites = S;
  a.min_sites = p->min_overlap_sites;
  int rc;
  const int64_t* d_site_off;
  const int32_t* d_loc_contig;
  if ((rc = upload(ctx, ctx->jn_site_off, site_off.data(), N + 1, &d_site_off)) ||
      (rc = upload(ctx, ctx->jn_loc_off, b->loc_off, N + 1, &a.loc_off)) ||
      (rc = upload(ctx, ctx->jn_loc_contig, loc_contig.data(), NL, &d_loc_contig)) ||
      (rc = upload(ctx, ctx->jn_lstart, b->loc_start, NL, &a.loc_start)) ||
      (rc = upload(ctx, ctx->jn_lend, b->loc_end, NL, &a.loc_end)) ||
      (rc = upload(ctx, ctx->jn_pc, b->pair_contig, NP, &a.pair_contig)) ||
      (rc = upload(ctx, ctx->jn_m1s, b->m1_start, NP, &a.m1_start)) ||
      (rc = upload(ctx, ctx->jn_m1e, b->m1_end, NP, &a.m1_end)) ||
      (rc = upload(ctx, ctx->jn_m2s, b->m2_start, NP, &a.m2_start)) ||
      (rc = upload(ctx, ctx->jn_m2e, b->m2_end, NP, &a.m2_end)) ||
      (rc = alloc_out(ctx, ctx->jn_diff, S, &a.diff)) ||
      (rc = alloc_out(ctx, ctx->jn_cov, S, &a.coverage)) ||
      (rc = alloc_out(ctx, ctx->jn_prefix, S, &a.prefix)) ||
      (rc = alloc_out(ctx, ctx->jn_hits, NL, &a.junction_hits)) ||
      (rc = alloc_out(ctx, ctx->jn_c1, NL, &a.cov1)) || (rc = alloc_out(ctx, ctx->jn_c2, NL, &a.cov2)) ||
      (rc = alloc_out(ctx, ctx->jn_cj, NL, &a.covj)) || (rc = alloc_out(ctx, ctx->jn_ratio, NL, &a.ratio)))
    return rc;
  a.site_off = d_site_off;
  a.loc_contig = d_loc_contig;
  if (r->locus_hits && (rc = alloc_out(ctx, ctx->jn_lhits, NL, &a.locus_hits))) return rc;
  if (r->pair_first || r->pair_mask) {
    if (!r->pair_first || !r->pair_mask) return fail(ctx, WF_E_BADINPUT, "pair_first and pair_mask go together");
    if ((rc = alloc_out(ctx, ctx->jn_pfirst, NP, &a.pair_first)) ||
        (rc = alloc_out(ctx, ctx->jn_pmask, NP, &a.pair_mask)) ||
        (rc = alloc_out(ctx, ctx->jn_ovf, 1, &a.overflow)))
      return rc;
  }
  const size_t tb = wf::junctions_tmp_bytes(S);
  if ((rc = ensure(ctx, ctx->jn_tmp, tb))) return rc;
  std::string err;
  if (wf::junctions_run(a, ctx->jn_tmp.p, ctx->jn_tmp.bytes, ctx->stream, &err))
    return fail(ctx, WF_E_HIP, "%s", err.c_str());
  if ((rc = download(ctx, r->junction_hits, a.junction_hits, NL)) ||
      (rc = download(ctx, r->coverage_gene1, a.cov1, NL)) ||
      (rc = download(ctx, r->coverage_gene2, a.cov2, NL)) ||
      (rc = download(ctx, r->coverage_junction, a.covj, NL)) ||
      (rc = download(ctx, r->ratio, a.ratio, NL)))
    return rc;
  if (r->locus_hits && (rc = download(ctx, r->locus_hits, a.locus_hits, NL))) return rc;
  unsigned overflow = 0;
  if (a.pair_first && ((rc = download(ctx, r->pair_first, a.pair_first, NP)) ||
                       (rc = download(ctx, r->pair_mask, a.pair_mask, NP)) ||
                       (rc = download(ctx, &overflow, a.overflow, 1))))
    return rc;
  if (r->coverage) {   // drop the sentinel slot of each contig
    for (int64_t c = 0; c < N; ++c) {
      const int64_t n = b->contig_length[c];
      if (n > 0 && (rc = download(ctx, r->coverage + (site_off[c] - c), a.coverage + site_off[c], n))) return rc;
    }
  }
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  if (overflow)
    return fail(ctx, WF_E_NOMEM, "%u read pairs hit loci more than 64 apart (pair_mask holds 64)", overflow);
  return WF_OK;
}

int wf_details_enable(wf_ctx* ctx, int on) {
  if (!ctx) return WF_E_BADINPUT;
  ctx->details_on = on != 0;
  ctx->det.levels.clear();
  return WF_OK;
}

int wf_details_read(wf_ctx* ctx, wf_details* out) {
  if (!ctx || !out) return WF_E_BADINPUT;
  if (!ctx->details_on) return fail(ctx, WF_E_STATE, "details are not enabled");
  ctx->d_eval_contig.clear(); ctx->d_eval_level.clear();
  ctx->d_level.clear(); ctx->d_contig.clear(); ctx->d_clade.clear(); ctx->d_locus.clear();
  ctx->d_nspan.clear(); ctx->d_spans.clear(); ctx->d_mean.clear(); ctx->d_span_off.assign(1, 0);
  for (const wf::DetailsLevel& L : ctx->det.levels) {
    for (int32_t c : L.act) { ctx->d_eval_contig.push_back(c); ctx->d_eval_level.push_back(L.level); }
    const size_t ns = L.seg_crank.size();
    for (size_t i = 0; i < ns; ++i) {
      ctx->d_level.push_back(L.level);
      ctx->d_contig.push_back(L.act[L.seg_crank[i]]);
      ctx->d_clade.push_back(L.seg_cg[2 * i]);
      ctx->d_locus.push_back(L.seg_cg[2 * i + 1]);
      ctx->d_mean.push_back(L.seg_mean[i]);
      const int n = L.span_cnt[i];
      ctx->d_nspan.push_back(n);
      const size_t at = 2 * (size_t)L.seg_start[i];
      for (int r = 0; r < 2 * n; ++r) ctx->d_spans.push_back(L.spans[at + r]);
      ctx->d_span_off.push_back(ctx->d_span_off.back() + (n > 0 ? n : 0));
    }
  }
  out->n_evals = (int64_t)ctx->d_eval_contig.size();
  out->eval_contig = ctx->d_eval_contig.data();
  out->eval_level = ctx->d_eval_level.data();
  out->n_segs = (int64_t)ctx->d_contig.size();
  out->seg_level = ctx->d_level.data();
  out->seg_contig = ctx->d_contig.data();
  out->seg_clade = ctx->d_clade.data();
  out->seg_locus = ctx->d_locus.data();
  out->seg_mean = ctx->d_mean.data();
  out->seg_nspan = ctx->d_nspan.data();
  out->span_off = ctx->d_span_off.data();
  out->spans = ctx->d_spans.data();
  return WF_OK;
}

int wf_synchronize(wf_ctx* ctx) {
  if (!ctx) return WF_E_BADINPUT;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return WF_OK;
}

int wf_timing_enable(wf_ctx* ctx, int on) {
  if (!ctx) return WF_E_BADINPUT;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  for (hipEvent_t ev : ctx->ev_pool) (void)hipEventDestroy(ev);
  ctx->ev_pool.clear();
  ctx->ev_lds.clear();
  ctx->launches = 0;
  ctx->timing = on != 0;
  if (!ctx->staged) ctx->staged = wf::staged_create(ctx->device);
  wf::staged_timing(ctx->staged, ctx->timing);
  return WF_OK;
}

int wf_timing_read(wf_ctx* ctx, wf_timing* out) {
  if (!ctx || !out) return WF_E_BADINPUT;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  double total = 0.0;
  for (auto& pr : ctx->ev_lds) {
    float ms = 0.f;
    HIP_TRY(ctx, hipEventElapsedTime(&ms, ctx->ev_pool[pr.first], ctx->ev_pool[pr.second]));
    total += ms;
  }
  out->pass_ms = total;
  out->passes = (int64_t)ctx->ev_lds.size();
  for (int i = 0; i < WF_N_PHASES; ++i) { out->phase_ms[i] = 0.0; out->phase_spans[i] = 0; }
  if (ctx->staged) wf::staged_timing_read(ctx->staged, out->phase_ms, out->phase_spans, WF_N_PHASES);
  return WF_OK;
}

}  // extern "C"
