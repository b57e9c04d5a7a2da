// Internal definitions shared by the HIP kernels (wf_staged.hip, wf_genecall.hip) and the
// C-ABI implementation (wf_api.cpp).  Not part of the public interface.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace wf {

constexpr int kBlock = 256;             // 4 waves of 64 lanes per contig workgroup
constexpr int kWaves = kBlock / 64;
constexpr int kLeafMax = 128;           // numpy pairwise-sum leaf size (PW_BLOCKSIZE)
constexpr int kNpyBuf = 8192;           // numpy reduction buffer (NPY_BUFSIZE)
// wf_batch.hit_key (include/waafle_hip.h): taxon | scov >= min_scov << 24 | strand '-' << 25 |
// systems 0-5 << 26 (k_pack_keys packs it when the caller passes none)
constexpr uint32_t kKeyTaxon = (1u << 24) - 1u, kKeyScov = 1u << 24, kKeyMinus = 1u << 25;
constexpr int kKeySys = 26;
constexpr int kLeafSlots = 160;         // >= leaves of one 8192-element buffer
constexpr int kMaxIter = 100;           // orgscorer.py:580
constexpr int kLin = 16;                // lineage row: ancestors at depths 0..15 (64 B)
constexpr int kAnnSlots = 256;          // (locus, system) annotation slots in LDS

// Parameters with the derived thresholds precomputed on the host
// (orgscorer.py:338-346, :515-516, :720-721).
struct DevParams {
  double k1, k2, kmin, k_amb, range, min_overlap, min_scov, amb_frac, sister_thr, annot_ref;
  int dis1;        // 0 report-best, 1 meld
  int dis2;        // 0 report-best, 1 jump, 2 meld
  int jump;        // number of initial raises
  int allow_lca, clade_genes, clade_leaves, weak, stranded, sister_on;
};

struct KArgs {
  // batch
  int n_contigs, n_sys;
  const int64_t* hit_off; const int32_t* qlo; const int32_t* qhi; const int32_t* taxon;
  const int8_t* hstrand; const double* score; const double* scov; const uint32_t* sysmask;
  const int64_t* loc_off; const int32_t* lstart; const int32_t* lend; const int8_t* lstrand;
  const uint32_t* hkey;          // wf_batch.hit_key (caller's, or packed by k_pack_keys)
  // taxonomy
  const int32_t* parent; const int32_t* depth; const int32_t* sibp; const int64_t* leaves;
  const int32_t* lin;            // [names * kLin] ancestor at each depth (-1 below the name);
                                 // null when the taxonomy is kLin or more levels deep
  int32_t root, unknown;
  DevParams p;
  // results
  int8_t* call; double* crit; double* rank; int32_t* c1; int32_t* c2; int8_t* dir;
  int16_t* iters; uint8_t* syn; int32_t* nm1; int32_t* nm2; int32_t* meld; int32_t* annot;
  int64_t* pair_evals; int32_t* status; int64_t* need;
  int64_t* ppot;                 // wf_result.ppot_sum (optional): bits 0-39 the sum, 40-47 the
                                 // highest iteration counted (a level counted once, whichever
                                 // form decides it)
  // HBM decision slots for contigs whose state outgrows the LDS arena (k_decide_big)
  char* big_ws; int64_t slot_bytes;
};

// Staged pipeline state (wf_staged.hip): flat kernels over all hits / attachments /
// segments, a device radix sort per roll-up level, one decision workgroup per contig.
struct SArgs {
  KArgs k;                       // batch, taxonomy, params, results (k.big_ws: tier-3 slots)
  int n_hits_i;                  // hits in the batch (int range checked on the host)
  int key_lb, key_tb;            // key = crank << (tb + lb) | clade << lb | locus
  const int64_t* catt_off;       // [n_contigs + 1] exclusive scan of attachments per contig
  int32_t *att_lo, *att_hi, *att_loc, *att_clade, *att_hit;
  double* att_sc;
  // current level
  uint64_t* keys;  int32_t* vals;             // sorted (key, attachment) pairs
  int32_t* flags;  int32_t* seg_id;           // segment starts / inclusive scan
  int32_t* seg_start; int32_t* seg_crank; double* seg_mean;
  const int32_t* act;  const int64_t* act_base;   // active contigs of this level
  int32_t* act_next; int64_t* act_base_next;      // raised contigs (next level)
  unsigned long long* counters;  // [0] next active << 40 | next attachments, [2] big count
  int32_t* big_list;             // contigs whose decision state needs an HBM slot
  int32_t* big2_list;            // ... of those, the ones k_big_sparse declines (counters[1])
  char* sp_ws;                   // k_big_sparse: HBM scratch, kSpSlot bytes per wave
  int32_t* two_list;             // (rank, contig) pairs that need explain_two (counters[5])
  int32_t* one_list;             // (rank, contig) pairs for the dense explain_one workgroup
                                 // (counters[6]); null: every active contig goes there
  int32_t* seg_nleaf;            // [segments + 1] numpy leaves per segment
  int32_t* leaf_off;             // [segments + 1] exclusive scan of seg_nleaf
  int32_t* leaf_seg;             // [leaves] segment of each leaf
  int4* seg_rec;                 // [segments] (first sorted attachment, count, locus length, leaves)
  int32_t* wave_list;            // segments for k_seg_wave (counters[7])
  int2* seg_cg;                  // [segments] (clade, locus)
  int32_t* crank_first;          // [active + 1] first segment of each active contig
  int32_t* seg_cnt;              // [active + 1] segments per active contig (per-contig sort)
  int32_t* seg_len;              // [segments] locus length (k_seg_build; null on the radix path)
  int2* satt_lohi;               // [attachments] site range, in sorted (segment) order
  double* satt_sc;               // [attachments] score, in sorted order
  double* leaf_val;              // [leaves] exact leaf sums
  uint64_t* annot_best;          // [n_loci * n_sys] best annotation score bits
  const int32_t* lut_off;        // [kNpyBuf + 2] numpy leaf table offsets by length
  const int4* lut;               // (start, length, parent adds) per leaf
  int64_t dec_lds_bytes;         // LDS arena of the decision workgroup
  int sort_cap;                  // per-contig LDS sort capacity: a power of 2 <= 4,096 (bitonic), a
                                 // multiple of 512 above (the LDS radix sort), 0: device radix sort
  int force_big;                 // WF_OPT_SPARSE_BIG 2: k_one hands every contig over
  int route_sparse;              // WF_OPT_SPARSE_BIG 2, 3: every k_decide contig to k_big_sparse
  int sparse_on;                 // WF_OPT_SPARSE_BIG != 0: k_big_sparse runs
  const unsigned long long* in_counts;   // this level's counts on the device (null: the
                                         // kernel arguments are exact)
  // Level-0 segment tables the first wave form hands to k_dump_sparse: contigs it leaves at
  // explain_two (or at an unproven --weak-loci assign-unknown row), every mean evaluated
  int64_t dump_cap;              // entries dump_cg / dump_mean hold (0: no hand-over)
  int2* dump_cg;                 // [dump_cap] (clade, locus), in (clade, locus) order per contig
  double* dump_mean;             // [dump_cap] segment means
  int32_t* dump_first;           // [n_contigs + 1] first entry of each slot
  int32_t* dump_list;            // [2 n_contigs] (form, contig); contig -1: did not fit; form 1:
                                 // compact (explain_two's inputs only, sp_two), 0: the whole table
  uint64_t* dump_um;             // [n_contigs] compact slots: unmasked loci | r__Root present << 63
  unsigned long long* dump_ctr;  // slots << 40 | entries
  int32_t* seed_pend;            // k_dump_sparse: pend of the contigs it decides (0), raises
                                 // (2: staged level-1 seed) or declines (1: staged level 0)
  // Roll-up levels by the first wave form (wave levels): level L re-attaches its contigs'
  // hits with clade anc[taxon] = parent^(jump + L)(taxon), decides explain_one and
  // explain_two in the wave, and appends the contigs it raises to roll_next (count in
  // *roll_next_n); contigs that leave the wave forms count in *fail_ctr (pend 1)
  int32_t* anc;                  // [n_tax] ancestor of each name at this level (null: level 0)
  int n_tax;
  int wave_two;                  // explain_two in the first form (else every such contig
                                 // goes to k_dump_sparse with its segment table)
  int32_t* roll_next;            // contigs raised at this level (null: no wave levels)
  unsigned long long* roll_next_n;
  unsigned long long* fail_ctr;
  unsigned long long* dump_ctr_next;   // k_dump_sparse zeroes the next level's table counter
  unsigned long long* wq;        // k_wave over a list: its contigs handed out one at a time by this
                                 // counter (zeroed per pass), else in static XCD order (null)
};

// waafle_genecaller (wf_genecall.hip): one contig group per wave
struct GcArgs {
  int n_groups, cap;                       // cap: intervals held in LDS per group (power of 2)
  const int64_t* hit_off; const int32_t* qlo; const int32_t* qhi; const int8_t* strand;
  const double* scov;
  double min_overlap, min_scov, min_gene_length;
  int32_t* n_genes; int32_t* gene_start; int32_t* gene_stop; int8_t* gene_strand;
  int32_t* status;                         // per group: 0, or -4 when it exceeds cap
};
hipError_t launch_genecall(const GcArgs& a, int cus, hipStream_t s);

// waafle_junctions (wf_junctions.hip): read-pair coverage and junction support
struct JnArgs {
  int n_contigs;
  int loc_forward;                         // every locus has start <= end and min_sites > 0
                                           // (early exit past the pair's right end ok)
  int64_t n_pairs, n_loci, n_sites;        // n_sites = sum of (contig length + 1)
  int64_t min_sites;                       // --min-overlap-sites
  const int64_t* site_off;                 // [n_contigs + 1]
  const int64_t* loc_off;                  // [n_contigs + 1] loci sorted by start per contig
  const int32_t* loc_contig;               // [n_loci]
  const int64_t* loc_start; const int64_t* loc_end;
  const int32_t* pair_contig;              // [n_pairs]
  const int64_t* m1_start; const int64_t* m1_end; const int64_t* m2_start; const int64_t* m2_end;
  int32_t* diff;                           // [n_sites] scratch
  int64_t* coverage;                       // [n_sites] per-site coverage (sentinels 0)
  int64_t* prefix;                         // [n_sites] inclusive prefix of coverage
  int32_t* junction_hits;                  // [n_loci] pairs supporting (j, j+1)
  int32_t* locus_hits;                     // [n_loci] pairs hitting locus j, or null
  int64_t* pair_first;                     // [n_pairs] first hit locus (-1: none), or null
  uint64_t* pair_mask;                     // [n_pairs] hit loci first .. first + 63
  unsigned* overflow;                      // pairs with a hit 64+ loci after their first
  double* cov1; double* cov2; double* covj; double* ratio;   // [n_loci] per junction j
};
int junctions_run(const JnArgs& a, void* tmp, size_t tmp_bytes, hipStream_t s, std::string* err);
size_t junctions_tmp_bytes(int64_t n_sites);

// --write-details: per roll-up level, the evaluated (active) contigs and the segment
// records of the level, copied to the host (wf_staged.hip details_level)
struct DetailsLevel {
  int level = 0;
  std::vector<int32_t> act;                  // active contigs (level 0: every contig)
  std::vector<int32_t> seg_start;            // [segments + 1] first sorted attachment
  std::vector<int32_t> seg_crank;            // active rank of each segment's contig
  std::vector<int32_t> seg_cg;               // (clade, locus) pairs
  std::vector<double> seg_mean;              // gene score
  std::vector<int32_t> span_cnt;             // runs (-1: all-zero site array)
  std::vector<int32_t> spans;                // (first, last) 1-based pairs at 2 * seg_start
};
struct DetailsSink {
  std::vector<DetailsLevel> levels;
};

struct StagedState;
// Level-0 triage (wf_triage.hip): pend[c] = 0 for the contigs it finished (explain_one from
// the full clades), kPendTriage for the rest, which the first wave form then runs (list).
constexpr int kPendTriage = 9;
hipError_t pack_keys(const KArgs& k, int64_t n_hits, uint32_t* key, int cus, hipStream_t s);
hipError_t finish_ppot(const KArgs& k, hipStream_t s);   // strips the iteration tags of K.ppot
hipError_t launch_triage(const SArgs& sa, int64_t* ccnt, int64_t* cleaves, int32_t* pend, int max_hits, int cus,
                         hipStream_t s);
// the first wave form over `list` (length *n_dev, on the device) at level 0
hipError_t launch_fast_list(const SArgs& sa, int64_t* ccnt, int64_t* cleaves, int32_t* pend, const int32_t* list,
                            const int64_t* n_dev, int max_hits, int cus, hipStream_t s);
// Per-contig wave kernels (wf_fast.hip): pend[c] = 0 finished there, 1 handed to the
// staged path with its attachment and leaf counts in ccnt / cleaves.  launch_fast: every
// contig, explain_one at level 0; launch_full: the contigs of `list` (length *n_dev, on
// the device), explain_two and the roll-up levels.
hipError_t launch_fast(const SArgs& sa, int64_t* ccnt, int64_t* cleaves, int32_t* pend, int max_hits, int cus,
                       hipStream_t s);
hipError_t launch_full(const SArgs& sa, int64_t* ccnt, int64_t* cleaves, int32_t* pend, const int32_t* list,
                       const int64_t* n_dev, int max_hits, int cus, bool rollup, hipStream_t s);
// roll-up level `level` (>= 1) of the first wave form over `list` (length *n_dev)
hipError_t launch_level(const SArgs& sa, int64_t* ccnt, int64_t* cleaves, int32_t* pend, const int32_t* list,
                        const int64_t* n_dev, int level, int max_hits, int cus, hipStream_t s);
StagedState* staged_create(int device);
void staged_destroy(StagedState* st);
void staged_set_lds(StagedState* st, int64_t bytes);
// context options (include/waafle_hip.h wf_option): the segment-table decision for contigs
// that outgrow the LDS arena, the attachments one call accepts (more: WF_E_TOOBIG), explain_two
// and the roll-up levels in the first wave form, the hand-over buffer's size (0: default)
void staged_set_options(StagedState* st, int sparse_big, int64_t att_limit, int64_t dump_cap,
                        int triage);
// per-phase timing (wf_phase): HIP events around each phase of each level, read back at the
// end of every staged_score call into the accumulators (reset by staged_timing(st, on))
void staged_timing(StagedState* st, bool on);
void staged_timing_read(const StagedState* st, double* ms, int64_t* spans, int n);
// wave kernels (wf_fast.hip) first; rollup: they also carry the roll-up levels
void staged_set_level0(StagedState* st, bool on, bool rollup);
// Runs the staged path for one batch on stream `s` (synchronises on it); 0 or -1/-2/-7
// with the message in *err (-1 bad input, -2 HIP failure, -7 WF_E_TOOBIG).
int staged_score(StagedState* st, const KArgs& k, int n_tax, int max_loci, int max_hits, int64_t n_hits,
                 int64_t n_loci, hipStream_t s, std::string* err, DetailsSink* det = nullptr);

}  // namespace wf
