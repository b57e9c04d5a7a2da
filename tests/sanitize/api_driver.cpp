// Host-sanitizer driver for the C-ABI of libwaafle_hip (wf_api.cpp and the host halves of
// wf_staged.hip / wf_genecall.hip / wf_junctions.hip).  Built by scripts/build_api_asan.sh
// with AddressSanitizer + UndefinedBehaviorSanitizer on the HOST code only
// (-Xarch_host -fsanitize=...; device code is compiled normally), run on the GPU box.
//
// It drives every entry point through its validation paths (null pointers, bad sizes, bad
// enums, call order) and through real runs: host-resident scoring batches that grow and
// shrink (scratch reallocation), a second context on the same device, the genecaller and
// the junction table.  Results are checked for internal consistency only (parity lives in
// the pytest suite); the point is a clean sanitizer log.
#include <sanitizer/lsan_interface.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "waafle_hip.h"

#define CHECK(x)                                                                  \
  do {                                                                            \
    if (!(x)) { std::fprintf(stderr, "FAILED: %s (line %d)\n", #x, __LINE__); std::exit(1); } \
  } while (0)

struct Batch {
  std::vector<int64_t> hit_off, loc_off;
  std::vector<int32_t> qlo, qhi, taxon, lstart, lend;
  std::vector<int8_t> hstrand, lstrand;
  std::vector<double> score, scov;
  std::vector<uint32_t> sysmask;
  int32_t max_hits = 0, max_loci = 0;
};

// taxonomy ids: 0 r__Root, 1 Unknown, 2..3 genera, 4..11 species (4 per genus)
static void make_taxonomy(std::vector<int32_t>& parent, std::vector<int32_t>& depth,
                          std::vector<int32_t>& sib, std::vector<int64_t>& leaves) {
  parent = {0, 0, 0, 0, 2, 2, 2, 2, 3, 3, 3, 3};
  depth = {0, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2};
  sib = {-1, -1, 0, 0, 2, 2, 2, 2, 3, 3, 3, 3};
  leaves = {8, 1, 4, 4, 1, 1, 1, 1, 1, 1, 1, 1};
}

static Batch make_batch(int n, int genes, int hits_per_gene, unsigned seed) {
  std::mt19937 rng(seed);
  Batch b;
  b.hit_off.push_back(0);
  b.loc_off.push_back(0);
  for (int c = 0; c < n; ++c) {
    int pos = 1;
    const int owner = 4 + (int)(rng() % 8);
    std::vector<std::pair<int, int>> genes_at;
    for (int g = 0; g < genes; ++g) {
      const int len = 250 + (int)(rng() % 1200);
      b.lstart.push_back(pos);
      b.lend.push_back(pos + len - 1);
      b.lstrand.push_back((int8_t)(rng() % 2));
      genes_at.push_back({pos, pos + len - 1});
      pos += len + 5 + (int)(rng() % 100);
    }
    for (auto [s, e] : genes_at)
      for (int h = 0; h < hits_per_gene; ++h) {
        const int a = s + (h ? (int)(rng() % 50) : 0), z = e - (h ? (int)(rng() % 50) : 0);
        b.qlo.push_back(a);
        b.qhi.push_back(z);
        b.taxon.push_back(h ? 4 + (int)(rng() % 8) : owner);
        b.hstrand.push_back((int8_t)(rng() % 2));
        b.scov.push_back(0.8 + 0.2 * (rng() % 1000) / 1000.0);
        b.score.push_back(0.7 + 0.3 * (rng() % 1000) / 1000.0);
        b.sysmask.push_back(rng() % 2);
      }
    b.hit_off.push_back((int64_t)b.qlo.size());
    b.loc_off.push_back((int64_t)b.lstart.size());
    b.max_hits = std::max<int32_t>(b.max_hits, genes * hits_per_gene);
    b.max_loci = std::max<int32_t>(b.max_loci, genes);
  }
  return b;
}

static wf_batch view(Batch& b) {
  wf_batch v{};
  v.n_contigs = (int32_t)b.hit_off.size() - 1;
  v.n_systems = 1;
  v.n_hits = (int64_t)b.qlo.size();
  v.n_loci = (int64_t)b.lstart.size();
  v.max_hits = b.max_hits;
  v.max_loci = b.max_loci;
  v.hit_off = b.hit_off.data(); v.hit_qlo = b.qlo.data(); v.hit_qhi = b.qhi.data();
  v.hit_taxon = b.taxon.data(); v.hit_strand = b.hstrand.data(); v.hit_score = b.score.data();
  v.hit_scov = b.scov.data(); v.hit_sysmask = b.sysmask.data(); v.loc_off = b.loc_off.data();
  v.loc_start = b.lstart.data(); v.loc_end = b.lend.data(); v.loc_strand = b.lstrand.data();
  return v;
}

struct Out {
  std::vector<int8_t> call, dir;
  std::vector<double> crit, rank;
  std::vector<int32_t> c1, c2, nm1, nm2, meld, annot, status;
  std::vector<int16_t> iters;
  std::vector<uint8_t> syn;
  std::vector<int64_t> pairs, need;
  wf_result r{};
  explicit Out(const wf_batch& v) {
    const size_t n = (size_t)v.n_contigs;
    call.resize(n); dir.resize(n); crit.resize(n); rank.resize(n); c1.resize(n); c2.resize(n);
    nm1.resize(n); nm2.resize(n); meld.resize(2 * (size_t)v.n_hits + 2 * n);
    annot.resize((size_t)v.n_loci * v.n_systems + 1); status.resize(n); iters.resize(n);
    syn.resize((size_t)v.n_loci + 1); pairs.resize(n); need.resize(n);
    r = wf_result{call.data(), crit.data(), rank.data(), c1.data(), c2.data(), dir.data(),
                  iters.data(), syn.data(), nm1.data(), nm2.data(), meld.data(), annot.data(),
                  pairs.data(), status.data(), need.data()};
  }
};

int main() {
  int ndev = 0;
  CHECK(wf_device_count(&ndev) == WF_OK && ndev > 0);
  CHECK(wf_abi_version() == WF_ABI_VERSION);
  CHECK(wf_init(0, nullptr) == WF_E_BADINPUT);
  wf_ctx* bad = nullptr;
  CHECK(wf_init(ndev + 5, &bad) == WF_E_BADINPUT && bad == nullptr);

  wf_ctx* ctx = nullptr;
  CHECK(wf_init(0, &ctx) == WF_OK);
  CHECK(wf_set_mode(ctx, 1) == WF_E_BADINPUT);
  CHECK(wf_set_mode(ctx, WF_MODE_STAGED) == WF_OK);
  CHECK(wf_set_mode(ctx, WF_MODE_WAVES) == WF_OK);
  CHECK(wf_set_mode(ctx, WF_MODE_LEVEL0) == WF_OK);
  CHECK(wf_set_lds_bytes(ctx, 10) == WF_E_BADINPUT);

  std::vector<int32_t> parent, depth, sib;
  std::vector<int64_t> leaves;
  make_taxonomy(parent, depth, sib, leaves);
  wf_params p{0.5, 0.8, 0.05, 0.1, 0.75, 0.1, 1, 2, 0, 0, 1, 2, -1, -1, 0, 1, 0};

  Batch b0 = make_batch(50, 6, 8, 1);
  wf_batch v0 = view(b0);
  Out o0(v0);
  CHECK(wf_score(ctx, &v0, &p, &o0.r) == WF_E_STATE);          // taxonomy first
  wf_taxonomy t{(int32_t)parent.size(), parent.data(), depth.data(), sib.data(), leaves.data(), 0, 1};
  wf_taxonomy tbad = t;
  std::vector<int32_t> pbad = parent;
  pbad[5] = 99;
  tbad.parent = pbad.data();
  CHECK(wf_set_taxonomy(ctx, &tbad) == WF_E_BADINPUT);
  CHECK(wf_set_taxonomy(ctx, &t) == WF_OK);
  CHECK(wf_score(ctx, nullptr, &p, &o0.r) == WF_E_BADINPUT);
  wf_params pbadenum = p;
  pbadenum.weak_loci = 7;
  CHECK(wf_score(ctx, &v0, &pbadenum, &o0.r) == WF_E_BADINPUT);
  wf_batch vbad = v0;
  vbad.max_hits = 1;                                             // understated
  CHECK(wf_score(ctx, &vbad, &p, &o0.r) == WF_E_BADINPUT);

  // real runs: grow, shrink, grow again (scratch reallocation on the context stream)
  unsigned long long check = 0;
  for (int round = 0; round < 3; ++round)
    for (int n : {50, 3000, 10, 6000}) {
      Batch b = make_batch(n, 4 + round * 3, 6 + round * 4, 100 + n + round);
      wf_batch v = view(b);
      Out o(v);
      CHECK(wf_score(ctx, &v, &p, &o.r) == WF_OK);
      for (int c = 0; c < v.n_contigs; ++c) {
        CHECK(o.status[c] == 0 && o.call[c] >= 0 && o.call[c] <= 2);
        check += (unsigned long long)o.call[c] * 31 + (unsigned long long)(o.c1[c] + 7);
      }
    }
  // a second context on the same device, interleaved
  wf_ctx* ctx2 = nullptr;
  CHECK(wf_init(0, &ctx2) == WF_OK && wf_set_taxonomy(ctx2, &t) == WF_OK);
  {
    Batch b = make_batch(2000, 8, 10, 7);
    wf_batch v = view(b);
    Out a(v), c(v);
    CHECK(wf_score(ctx, &v, &p, &a.r) == WF_OK);
    CHECK(wf_score(ctx2, &v, &p, &c.r) == WF_OK);
    for (int i = 0; i < v.n_contigs; ++i) CHECK(a.call[i] == c.call[i] && a.crit[i] == c.crit[i]);
  }
  wf_free(ctx2);
  CHECK(wf_timing_enable(ctx, 1) == WF_OK);
  CHECK(wf_score(ctx, &v0, &p, &o0.r) == WF_OK);
  wf_timing tm{};
  CHECK(wf_timing_read(ctx, &tm) == WF_OK && tm.passes == 1 && tm.pass_ms > 0.0);
  CHECK(tm.phase_spans[WF_PHASE_WAVES] >= 1 && tm.phase_ms[WF_PHASE_WAVES] > 0.0);
  CHECK(wf_timing_enable(ctx, 0) == WF_OK);
  // options: validation, the attachment limit (WF_E_TOOBIG, nothing scored), the
  // segment-table decision forced for every staged contig (same records)
  CHECK(wf_set_option(ctx, WF_OPT_ATT_LIMIT, 0) == WF_E_BADINPUT);
  CHECK(wf_set_option(ctx, WF_OPT_SPARSE_BIG, 4) == WF_E_BADINPUT);
  CHECK(wf_set_option(ctx, 77, 1) == WF_E_BADINPUT);
  {
    Batch b = make_batch(1500, 7, 9, 11);
    wf_batch v = view(b);
    Out a(v), c(v);
    CHECK(wf_set_mode(ctx, WF_MODE_STAGED) == WF_OK);
    CHECK(wf_score(ctx, &v, &p, &a.r) == WF_OK);
    CHECK(wf_set_option(ctx, WF_OPT_ATT_LIMIT, 5) == WF_OK);
    CHECK(wf_score(ctx, &v, &p, &c.r) == WF_E_TOOBIG);
    CHECK(wf_set_option(ctx, WF_OPT_ATT_LIMIT, (int64_t(1) << 31) - 1) == WF_OK);
    CHECK(wf_set_option(ctx, WF_OPT_SPARSE_BIG, 2) == WF_OK);
    CHECK(wf_score(ctx, &v, &p, &c.r) == WF_OK);
    for (int i = 0; i < v.n_contigs; ++i)
      CHECK(a.call[i] == c.call[i] && a.crit[i] == c.crit[i] && a.rank[i] == c.rank[i] && a.c1[i] == c.c1[i]);
    CHECK(wf_set_option(ctx, WF_OPT_SPARSE_BIG, 1) == WF_OK);
    CHECK(wf_set_mode(ctx, WF_MODE_LEVEL0) == WF_OK);
  }

  // genecaller
  {
    std::vector<int64_t> off = {0, 3, 3, 5};
    std::vector<int32_t> lo = {1, 50, 900, 10, 15}, hi = {300, 400, 1200, 500, 480};
    std::vector<int8_t> st = {0, 1, 0, 0, 1};
    std::vector<double> sc = {0.9, 0.9, 0.9, 0.5, 0.95};
    wf_gc_batch gb{3, 0, 5, off.data(), lo.data(), hi.data(), st.data(), sc.data()};
    wf_gc_params gp{0.1, 0.75, 200.0, 0, 0};
    std::vector<int32_t> ng(3), gs(5), ge(5);
    std::vector<int8_t> gst(5);
    wf_gc_result gr{ng.data(), gs.data(), ge.data(), gst.data()};
    CHECK(wf_genecall(ctx, &gb, &gp, &gr) == WF_OK);
    CHECK(ng[0] == 2 && ng[1] == 0 && ng[2] == 1);
  }
  // junctions
  {
    std::vector<int64_t> clen = {1000, 500}, loff = {0, 3, 3}, ls = {10, 300, 700}, le = {250, 600, 990};
    std::vector<int32_t> pc = {0, 0, 0, 1};
    std::vector<int64_t> a1 = {100, 200, 950, 1}, b1 = {199, 299, 1049, 100}, a2 = {220, 500, 1, 400},
                         b2 = {319, 599, 100, 499};
    wf_jn_batch jb{2, 0, 4, 3, clen.data(), loff.data(), ls.data(), le.data(), pc.data(),
                   a1.data(), b1.data(), a2.data(), b2.data()};
    wf_jn_params jp{25};
    std::vector<int32_t> jh(3), lh(3);
    std::vector<double> g1(3), g2(3), gj(3), ra(3);
    std::vector<int64_t> cov(1500), pf(4);
    std::vector<uint64_t> pm(4);
    wf_jn_result jr{jh.data(), g1.data(), g2.data(), gj.data(), ra.data(), lh.data(), cov.data(),
                    pf.data(), pm.data()};
    CHECK(wf_junctions(ctx, &jb, &jp, &jr) == WF_OK);
    CHECK(jh[0] == 1 && jh[1] == 0 && lh[0] == 3);
    CHECK(cov[0] == 1 && cov[99] == 2 && cov[1000 + 0] == 1);
    std::vector<int64_t> ls_bad = {300, 10, 700};
    jb.loc_start = ls_bad.data();
    CHECK(wf_junctions(ctx, &jb, &jp, &jr) == WF_E_BADINPUT);     // loci must be start-sorted
  }
  wf_free(ctx);
  std::printf("api_driver ok check=%llu\n", check);
  // Every check above has run and every context is freed: leak-check now (the HIP/HSA
  // runtimes' own allocations are still reachable from their globals, so only memory this
  // code lost is reported; tests/sanitize/lsan.supp names the runtime libraries in case),
  // then leave without the runtimes' static destructors: under ASan they free runtime
  // memory after the sanitizer's device-allocator hooks are gone, and ASan aborts in its
  // own CHECK (sanitizer_allocator_device.h, dev_runtime_unloaded_) -- a teardown-order
  // artefact, not a finding in this code.
  std::fflush(stdout);
  if (__lsan_do_recoverable_leak_check() != 0) {
    std::printf("api_driver: leaks reported\n");
    std::fflush(stdout);
    std::_Exit(23);
  }
  std::printf("api_driver leak check ok\n");
  std::fflush(stdout);
  std::_Exit(0);
}
