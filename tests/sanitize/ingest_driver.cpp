// Sanitizer driver for the native ingest (libwaafle_ingest's source, built with
// -fsanitize=address,undefined by tests/test_sanitize.py).  Parses the given inputs with
// several thread counts and prints a checksum of every array of the view, so the test can
// also compare the instrumented build against the production library's Python view.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "waafle_ingest.h"

static uint64_t mix(uint64_t h, const void* p, size_t n) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s fasta blastout gff min_gene_length [threads...]\n", argv[0]);
    return 2;
  }
  const double mgl = std::atof(argv[4]);
  int rc_all = 0;
  for (int t = 5; t <= argc; ++t) {
    const int threads = t < argc ? std::atoi(argv[t]) : 0;
    wf_ingest* ing = wf_ingest_new();
    const int rc = wf_ingest_parse(ing, argv[1], argv[2], argv[3], mgl, threads);
    if (rc != WF_INGEST_OK) {
      std::printf("threads=%d rc=%d %s\n", threads, rc, wf_ingest_last_error(ing));
      wf_ingest_free(ing);
      rc_all = rc < 0 ? 1 : rc_all;
      continue;
    }
    wf_ingest_view v;
    wf_ingest_get_view(ing, &v);
    uint64_t h = 1469598103934665603ull;
    const int64_t N = v.n_contigs, H = v.n_hits, L = v.n_loci;
    h = mix(h, v.contig_length, N * 8);
    h = mix(h, v.hit_off, (N + 1) * 8);
    h = mix(h, v.hit_qlo, H * 4);
    h = mix(h, v.hit_qhi, H * 4);
    h = mix(h, v.hit_taxon, H * 4);
    h = mix(h, v.hit_strand, H);
    h = mix(h, v.hit_score, H * 8);
    h = mix(h, v.hit_scov, H * 8);
    h = mix(h, v.hit_sysmask, H * 4);
    h = mix(h, v.hit_row, H * 8);
    h = mix(h, v.loc_off, (N + 1) * 8);
    h = mix(h, v.loc_start, L * 4);
    h = mix(h, v.loc_end, L * 4);
    h = mix(h, v.loc_strand, L);
    h = mix(h, v.contig_blob, v.contig_off[N]);
    h = mix(h, v.taxa_blob, v.taxa_off[v.n_taxa]);
    std::printf("threads=%d contigs=%lld hits=%lld loci=%lld taxa=%d hash=%016llx\n", threads,
                (long long)N, (long long)H, (long long)L, v.n_taxa, (unsigned long long)h);
    wf_ingest_free(ing);
  }
  return rc_all;
}
