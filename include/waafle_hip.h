/*
 * waafle_hip.h -- C-ABI of libwaafle_hip.so, the MI355X (gfx950) implementation of the
 * waafle_orgscorer contig-scoring hot path.
 *
 * The reference (menickname/waafle v0.1.0, pure Python + numpy) has no FFI; its
 * in-process seam is the per-contig loop of `waafle/waafle_orgscorer.py:943-960`
 * (attach_hits -> update_gene_scores -> [jump_taxonomy] -> evaluate_contig).  One
 * wf_score() call replaces that loop for a whole batch of contigs.  The host side
 * (Python, ctypes) parses the four input files, interns taxa, packs the flat arrays
 * below and renders the three TSVs from the result records.
 *
 * Conventions: plain pointers + sizes, no ownership transfer (every buffer is owned by
 * the caller and only borrowed for the duration of the call), 0 = success and a
 * negative WF_E_* code otherwise with the message in wf_last_error(ctx), no exceptions
 * and no exit() inside the library.  One wf_ctx per device; distinct contexts may be
 * used from different host threads concurrently; a context is not re-entrant.
 */
#ifndef WAAFLE_HIP_H
#define WAAFLE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WF_ABI_VERSION 6   /* 4: WF_OPT_SPARSE_BIG 0/1 retired, WF_PHASE_ROLLUP, WF_OPT_WAVE_TWO / _DUMP_CAP;
                                 5: WF_OPT_TRIAGE, WF_PHASE_TRIAGE;
                                 6: wf_batch.hit_key (packed hit record), wf_pack_hit_keys;
                                    WF_OPT_WAVE_TWO 0 (the round-3 hand-over flow) retired */

enum wf_status {
  WF_OK = 0,
  WF_E_BADINPUT = -1,  /* malformed arguments (sizes, null pointers, limits) */
  WF_E_HIP = -2,       /* a HIP runtime call failed */
  WF_E_RUNAWAY = -3,   /* > 100 roll-up iterations: orgscorer.py:580-581 */
  WF_E_NOMEM = -4,     /* per-contig workspace too small (see wf_result.need_bytes) */
  WF_E_STATE = -5,     /* call order (e.g. wf_score before wf_set_taxonomy) */
  WF_E_EMPTYMASK = -6, /* every locus masked at a roll-up level (np.min of empty) */
  WF_E_TOOBIG = -7     /* the hit-locus attachments the staged kernels would hold in HBM
                          (the contigs the wave forms hand them; every contig in
                          WF_MODE_STAGED) exceed one call's limit (WF_OPT_ATT_LIMIT, at
                          most 2^31 - 1): score the batch in parts */
};

enum wf_call { WF_CALL_UNCLASSIFIED = 0, WF_CALL_NO_LGT = 1, WF_CALL_LGT = 2 };

/* Execution form of wf_score (the results are identical).
 * WF_MODE_LEVEL0 (default): per-contig wave kernels carry level 0 in LDS (explain_one in
 *   the wave; explain_two from the segment table it hands over, k_dump_sparse), and every
 *   roll-up level is one more launch of the same wave form over the contigs the level before
 *   raised.  Only contigs that exceed a wave's LDS slice (attachments,
 *   loci, leaf tables) or the hand-over tables continue in the second wave form and then
 *   the staged kernels.
 * WF_MODE_WAVES: the second (FULL) wave form carries explain_two and the roll-up levels in
 *   its LDS slice.
 * WF_MODE_STAGED: every contig through the staged kernels (one kernel per phase over all
 *   contigs: attachments, per-contig sort, segment means, decisions; one pass per level).
 * The ABI-1 WF_MODE_FUSED form (1) stays retired; wf_set_mode rejects it. */
enum wf_mode { WF_MODE_STAGED = 0, WF_MODE_LEVEL0 = 2, WF_MODE_WAVES = 3 };

/* Context options (wf_set_option); every one leaves the results unchanged.
 * WF_OPT_SPARSE_BIG: the decision form of the staged kernels for contigs of <= 63 loci.
 *   3 (default): explain_one by one wave per contig (k_one), and every contig it leaves
 *   open (explain_two, more segments than its LDS holds, --weak-loci assign-unknown) takes
 *   the decision straight from the segment table, one wave per contig (k_big_sparse);
 *   2: every staged decision in the segment-table form (a test setting: it exercises that
 *   form on every input).  The dense matrix decision remains for > 63 loci and for a table
 *   the segment-table form declines (its class or pair tables outgrown).  The values 0 and 1
 *   (dense decisions for <= 63 loci) are retired: WF_E_BADINPUT.
 * WF_OPT_ATT_LIMIT: hit-locus attachments the staged kernels accept in one wf_score call
 *   (default and maximum 2^31 - 1; more -> WF_E_TOOBIG and the call's records are not
 *   valid: score the batch in parts).  The wave forms hold a contig's attachments in LDS.
 * WF_OPT_WAVE_TWO (WF_MODE_LEVEL0): 1, the only value since ABI 6: the first wave form also
 *   decides explain_two (up to 64 potential clades, <= 63 loci) and carries the roll-up
 *   levels, one pass per level over the contigs still open; the rest goes to the
 *   segment-table decision (k_dump_sparse).  0 (every explain_two contig there and the
 *   roll-up levels in the staged kernels: the round-3 flow) is retired: WF_E_BADINPUT.
 * WF_OPT_DUMP_CAP: segment-table entries of the wave form's hand-over buffer (default
 *   max(32 * contigs, 65536)); contigs past it go to the staged kernels (a test setting).
 * WF_OPT_TRIAGE (WF_MODE_LEVEL0 / _WAVES): 1 (default) a level-0 triage kernel first decides
 *   the contigs explain_one settles from the clades present on every locus (one-run gene
 *   scores), without the wave form's sort and segment table; the wave form runs the rest.
 *   0: the wave form runs every contig (a test setting: it exercises that path on every
 *   input). */
enum wf_option { WF_OPT_SPARSE_BIG = 1, WF_OPT_ATT_LIMIT = 2, WF_OPT_WAVE_TWO = 3, WF_OPT_DUMP_CAP = 4,
                 WF_OPT_TRIAGE = 5 };

typedef struct wf_ctx wf_ctx;

/* Interned taxonomy.  Ids are the ranks of all names (taxonomy file names, hit taxa,
 * "r__Root", "Unknown") in Python code-point order, so `clade1 < clade2`
 * (orgscorer.py:608) is an integer compare.  Replaces utils.py:374-447. */
typedef struct wf_taxonomy {
  int32_t n;                  /* number of names */
  const int32_t* parent;      /* [n] Taxonomy.get_parent (utils.py:386-387) */
  const int32_t* depth;       /* [n] len(Taxonomy.get_lineage) - 1 (utils.py:392-399) */
  const int32_t* sib_parent;  /* [n] parent the name is listed under as a child in the
                                 taxonomy file (children map, utils.py:382), or -1 */
  const int64_t* leaf_count;  /* [n] Taxonomy.get_leaf_count (utils.py:436-447) */
  int32_t root;               /* id of "r__Root" (utils.py:368) */
  int32_t unknown;            /* id of "Unknown" (utils.py:367) */
} wf_taxonomy;

/* orgscorer.py:135-303 + genecaller.py:81-101 (enums in the choice order shown). */
typedef struct wf_params {
  double k1;                  /* -k1 / --one-clade-threshold */
  double k2;                  /* -k2 / --two-clade-threshold */
  double range;               /* --range */
  double min_overlap;         /* --min-overlap */
  double min_scov;            /* --min-scov */
  double ambiguous_fraction;  /* --ambiguous-fraction */
  int32_t disambiguate_one;   /* 0 report-best, 1 meld */
  int32_t disambiguate_two;   /* 0 report-best, 1 jump, 2 meld */
  int32_t jump_taxonomy;      /* 0 = off (None) */
  int32_t allow_lca;          /* --allow-lca */
  int32_t ambiguous_threshold;/* 0 off, 1 lenient, 2 strict */
  int32_t sister_penalty;     /* 0 off, 1 lenient, 2 strict */
  int32_t clade_genes;        /* -1 = off (None) */
  int32_t clade_leaves;       /* -1 = off (None) */
  int32_t weak_loci;          /* 0 ignore, 1 penalize, 2 assign-unknown */
  int32_t annotation_threshold; /* 0 off, 1 lenient, 2 strict */
  int32_t stranded;           /* --stranded */
} wf_params;

/* A batch of contigs in CSR form.  Contig c owns hits [hit_off[c], hit_off[c+1]) in
 * blastout file order (utils.py:255-270) and loci [loc_off[c], loc_off[c+1]) -- the
 * loci that passed --min-gene-length, in GFF order (orgscorer.py:348-352). */
typedef struct wf_batch {
  int32_t n_contigs;
  int32_t n_systems;          /* annotation systems (<= 32); bit s of hit_sysmask */
  int64_t n_hits;
  int64_t n_loci;
  int32_t max_hits;           /* max hits of one contig (workspace sizing) */
  int32_t max_loci;           /* max loci of one contig */
  int32_t device_resident;    /* 1: all pointers (batch and result) are device memory
                                 and wf_score only enqueues on the context stream;
                                 0: host memory, wf_score copies and synchronises */
  int32_t _pad;
  const int64_t* hit_off;     /* [n_contigs+1] */
  const int32_t* hit_qlo;     /* [n_hits] min(qstart, qend)  (utils.py:173-174) */
  const int32_t* hit_qhi;     /* [n_hits] max(qstart, qend) */
  const int32_t* hit_taxon;   /* [n_hits] taxon id = sseqid.split("|")[1] (utils.py:234-235) */
  const int8_t*  hit_strand;  /* [n_hits] 0 '+', 1 '-' (sstrand, utils.py:214) */
  const double*  hit_score;   /* [n_hits] waafle_score (utils.py:229) */
  const double*  hit_scov;    /* [n_hits] scov_modified (utils.py:227) */
  const uint32_t* hit_sysmask;/* [n_hits] annotation systems present (utils.py:237-241) */
  const int64_t* loc_off;     /* [n_contigs+1] */
  const int32_t* loc_start;   /* [n_loci] GFF start */
  const int32_t* loc_end;     /* [n_loci] GFF end */
  const int8_t*  loc_strand;  /* [n_loci] 0 '+', 1 '-', 2 anything else */
  /* Optional (NULL: the library packs it on the device, one extra pass over the hits): the
     hit's filter fields packed in one word, wf_pack_hit_keys' layout -- bits 0-23 hit_taxon,
     bit 24 hit_scov >= params.min_scov (the attach_hits filter, orgscorer.py:363-364: it
     must be packed with the min_scov of the wf_score call it is passed to), bit 25
     hit_strand '-', bits 26-31 hit_sysmask & 63 (systems 0-5).  The level-0 triage, the
     kernel of most contigs, then reads 20 bytes per hit (qlo, qhi, key, score) instead of
     32.  The other arrays stay required (the other kernels read them). */
  const uint32_t* hit_key;    /* [n_hits] */
} wf_batch;

/* Per-contig results (caller-allocated, same residency as the batch). */
typedef struct wf_result {
  int8_t*  call;              /* [n] wf_call: routing of orgscorer.py:838-890 */
  double*  crit;              /* [n] min (max) score of the reported option */
  double*  rank;              /* [n] avg (max) score of the reported option */
  int32_t* clade1;            /* [n] reported clade / clade_A (after melding) */
  int32_t* clade2;            /* [n] clade_B (lgt only) */
  int8_t*  direction;         /* [n] 0 "A?B", 1 "B>A" */
  int16_t* iterations;        /* [n] roll-up iterations performed (1 = none) */
  uint8_t* synteny;           /* [n_loci] synteny characters, CSR by loc_off */
  int32_t* n_meld1;           /* [n] melded clades for clade1 (tails), 0 = none */
  int32_t* n_meld2;           /* [n] melded clades for clade2 */
  int32_t* meld;              /* [2*n_hits + 2*n]; contig c writes its meld1 ids then its
                                 meld2 ids from 2*hit_off[c] + 2*c */
  int32_t* annot_hit;         /* [n_loci * n_systems] batch hit index whose annotation
                                 the locus keeps (orgscorer.py:384-392), or -1 */
  int64_t* pair_evals;        /* [n] sum of P_pot*(P_pot-1)/2 over explain_two calls */
  int32_t* status;            /* [n] 0 or a WF_E_* code for this contig */
  int64_t* need_bytes;        /* [n] workspace bytes asked for when status == WF_E_NOMEM */
  int64_t* ppot_sum;          /* [n] optional (NULL: not reported): sum of P_pot over the
                                 explain_two calls that evaluate pairs (P_pot >= 2), one per
                                 roll-up level -- the per-call sizes behind pair_evals, for
                                 SURVEY 8(d)'s B_k2 = sum P_pot * G * 8 (ABI 6) */
} wf_result;

/* Pass timing accumulated while enabled: HIP events recorded on the context stream
 * around every kernel of each wf_score pass. */
enum wf_phase {
  WF_PHASE_WAVES = 0,         /* wave kernels: level 0, explain_one / explain_two in LDS */
  WF_PHASE_ATTACH = 1,        /* staged: attachment counts, offsets, attachments */
  WF_PHASE_SEGMENTS = 2,      /* staged, per level: sort, segments, exact segment means */
  WF_PHASE_DECIDE = 3,        /* staged, per level: k_one + k_decide (LDS arena) */
  WF_PHASE_BIG = 4,           /* staged, per level: k_big_sparse + k_decide_big */
  WF_PHASE_HANDOVER = 5,      /* level 0 of the contigs the wave kernels hand over with
                                 their segment tables (k_dump_sparse) */
  WF_PHASE_ROLLUP = 6,        /* roll-up levels 1, 2, ... in the first wave form (with their
                                 hand-overs), WF_OPT_WAVE_TWO 1 */
  WF_PHASE_TRIAGE = 7,        /* the level-0 triage kernel and the list of contigs it hands
                                 on (WF_OPT_TRIAGE 1); WF_PHASE_WAVES is then the first wave
                                 form's launch over that list */
  WF_N_PHASES = 8
};
typedef struct wf_timing {
  double pass_ms;             /* sum over timed passes */
  int64_t passes;             /* number of wf_score calls timed */
  double phase_ms[WF_N_PHASES];       /* per wf_phase, summed over timed passes */
  int64_t phase_spans[WF_N_PHASES];   /* timed spans (one per phase and level) */
} wf_timing;

/* ---- waafle_genecaller (waafle_genecaller.py:107-233) -------------------------------
 * Gene calls from one blastout: per contig group (a run of consecutive rows with the same
 * qseqid, utils.py:255-270), hits with scov_modified >= min_scov become intervals, the
 * connected components of overlapping intervals (calc_overlap >= min_overlap) are merged
 * (min start, max stop, strand of the longest member, ties to '-'), and merged genes of
 * length >= min_gene_length are returned in component order.  Replaces the per-contig
 * hits2ints / overlap_intervals / merge_inodes calls of the reference's main loop. */
typedef struct wf_gc_batch {
  int32_t n_groups;           /* contig groups, blastout order */
  int32_t device_resident;    /* 1: device pointers (enqueue only); 0: host arrays */
  int64_t n_hits;
  const int64_t* hit_off;     /* [n_groups + 1] hit range of each group */
  const int32_t* hit_qlo;     /* [n_hits] qstart / qend, either order */
  const int32_t* hit_qhi;
  const int8_t* hit_strand;   /* 0 '+', 1 '-' (sstrand "minus", utils.py:214) */
  const double* hit_scov;     /* scov_modified (utils.py:227) */
} wf_gc_batch;

typedef struct wf_gc_params {
  double min_overlap;         /* --min-overlap, default 0.1 */
  double min_scov;            /* --min-scov, default 0.75 */
  double min_gene_length;     /* --min-gene-length, default 200 */
  int32_t stranded;           /* accepted, no effect: dead upstream (genecaller.py:212-215) */
  int32_t _pad;
} wf_gc_params;

typedef struct wf_gc_result { /* same residency as the batch */
  int32_t* n_genes;           /* [n_groups] */
  int32_t* gene_start;        /* [n_hits]: group g's genes at [hit_off[g], hit_off[g] + n_genes[g]) */
  int32_t* gene_stop;
  int8_t*  gene_strand;       /* 0 '+', 1 '-' */
} wf_gc_result;

int wf_genecall(wf_ctx* ctx, const wf_gc_batch* batch, const wf_gc_params* params, wf_gc_result* out);

/* ---- waafle_junctions (waafle_junctions.py:252-316, 414-451) ---------------------------
 * Read-pair support of gene-gene junctions.  For every concordant pair (two consecutive
 * aligned SAM records with the same QNAME and RNAME, concordant_hits :252-275) the pair's
 * span [min(coords) - 1, max(coords) - 1] adds 1 to the contig's per-site coverage
 * (:432-436), and every locus overlapping either mate by >= min_overlap_sites sites
 * (find_hit_loci :277-286) is hit.  For each pair of start-adjacent loci (j, j+1) of a
 * contig (evaluate_contig :292-316): junction_hits = pairs hitting both, coverage_gene1/2 =
 * mean coverage over each locus, coverage_junction = mean over [end(j) - 1, start(j+1))
 * (0 when the loci touch or overlap), ratio = junction / (mean of the two genes + 1e-6).
 * Slices follow Python's rules on the contig's coverage array; an empty slice gives NaN
 * (np.mean of nothing).  Replaces the SAM loop of the reference's main() and its
 * evaluate_contig calls. */
typedef struct wf_jn_batch {
  int32_t n_contigs;
  int32_t device_resident;    /* 1: device pointers (enqueue only); 0: host arrays */
  int64_t n_pairs;
  int64_t n_loci;
  const int64_t* contig_length; /* [n_contigs] FASTA lengths (read_contig_lengths) */
  const int64_t* loc_off;     /* [n_contigs + 1] loci of each contig, sorted by start (stable) */
  const int64_t* loc_start;   /* [n_loci] GFF start */
  const int64_t* loc_end;     /* [n_loci] GFF end */
  const int32_t* pair_contig; /* [n_pairs] contig of both mates */
  const int64_t* m1_start;    /* [n_pairs] mate 1: POS, POS + cigar_length - 1 (utils.py:524-539) */
  const int64_t* m1_end;
  const int64_t* m2_start;    /* mate 2 */
  const int64_t* m2_end;
} wf_jn_batch;

typedef struct wf_jn_params {
  int64_t min_overlap_sites;  /* --min-overlap-sites, default 25 */
} wf_jn_params;

typedef struct wf_jn_result {   /* same residency as the batch */
  int32_t* junction_hits;     /* [n_loci] at j: junction (j, j+1) of j's contig */
  double* coverage_gene1;     /* [n_loci] */
  double* coverage_gene2;
  double* coverage_junction;
  double* ratio;
  int32_t* locus_hits;        /* [n_loci] pairs hitting locus j, or NULL */
  int64_t* coverage;          /* [sum(contig_length)] per-site coverage, contig-major, or NULL */
  int64_t* pair_first;        /* [n_pairs] first hit locus of each pair (-1: none), or NULL */
  uint64_t* pair_mask;        /* [n_pairs] bit i: locus pair_first + i hit (the pair's code
                                 set, :277-286; WF_E_NOMEM if hits span more than 64 loci) */
} wf_jn_result;

int wf_junctions(wf_ctx* ctx, const wf_jn_batch* batch, const wf_jn_params* params, wf_jn_result* out);

/* ---- --write-details (orgscorer.py:766-812, 931-937) --------------------------------
 * With details on, the next wf_score (staged mode) also records, for every roll-up level,
 * the contigs it evaluated and each (contig, clade, locus) segment of that level: its gene
 * score (Contig.update_gene_scores :394-406, the exact numpy mean) and its gene spans
 * (make_gene_spans_field :770-789: first and last 1-based site of every nonzero run longer
 * than one site).  The caller renders the reference's rows from them (clades per contig
 * and level, 'Unknown' = 1 - max for --weak-loci assign-unknown).  Replaces the
 * write_details(details, contig, iteration) calls of evaluate_contig (:566-583).
 * Arrays stay valid until the next wf_score or wf_free.  Synchronous; a diagnostic path. */
typedef struct wf_details {
  int64_t n_evals;            /* evaluated (contig, level) pairs, level-major */
  const int32_t* eval_contig;
  const int32_t* eval_level;
  int64_t n_segs;             /* segment records, level-major */
  const int32_t* seg_level;
  const int32_t* seg_contig;
  const int32_t* seg_clade;   /* taxonomy id at that level */
  const int32_t* seg_locus;   /* index among the contig's kept loci */
  const double* seg_mean;     /* gene score */
  const int32_t* seg_nspan;   /* runs listed; -1: the site array is all zero (upstream raises) */
  const int64_t* span_off;    /* [n_segs + 1] first run of each segment */
  const int32_t* spans;       /* [2 * span_off[n_segs]] (first, last) 1-based site pairs */
} wf_details;

int wf_details_enable(wf_ctx* ctx, int on);
int wf_details_read(wf_ctx* ctx, wf_details* out);

int wf_abi_version(void);
int wf_device_count(int* count);
int wf_init(int device, wf_ctx** out);
void wf_free(wf_ctx* ctx);
const char* wf_last_error(const wf_ctx* ctx);
int wf_set_stream(wf_ctx* ctx, void* hip_stream);     /* NULL = the context's own stream */
int wf_set_lds_bytes(wf_ctx* ctx, int64_t bytes);     /* decision arena per workgroup (LDS) */
int wf_set_mode(wf_ctx* ctx, int mode);               /* WF_MODE_LEVEL0 (default), _WAVES or _STAGED */
int wf_set_option(wf_ctx* ctx, int option, int64_t value);   /* wf_option */
int wf_set_taxonomy(wf_ctx* ctx, const wf_taxonomy* tax);
int wf_score(wf_ctx* ctx, const wf_batch* batch, const wf_params* params, wf_result* out);
/* wf_batch.hit_key from the separate arrays (host memory, any thread, no context):
   out[i] = taxon[i] | (scov[i] >= min_scov) << 24 | (strand[i] == 1) << 25
            | (sysmask[i] & 63) << 26.
   WF_E_BADINPUT for a taxon id outside [0, 2^24) or a strand other than 0 / 1. */
int wf_pack_hit_keys(int64_t n_hits, const int32_t* taxon, const int8_t* strand, const double* scov,
                     const uint32_t* sysmask, double min_scov, uint32_t* out);
int wf_synchronize(wf_ctx* ctx);
int wf_timing_enable(wf_ctx* ctx, int on);             /* also resets the counters */
int wf_timing_read(wf_ctx* ctx, wf_timing* out);       /* synchronises first */

#ifdef __cplusplus
}
#endif
#endif /* WAAFLE_HIP_H */
