/*
 * waafle_ingest.h -- C-ABI of libwaafle_ingest.so: native, multi-threaded parsing of the
 * waafle_orgscorer inputs (FASTA, 15-column BLAST tabular, GFF) straight into the flat
 * CSR arrays that wf_score() takes (include/waafle_hip.h).  SURVEY.md §8(f) row 1.
 *
 * Replaces, for well-formed input, the reference readers
 *   read_contig_lengths      waafle/utils.py:109-120
 *   Hit / iter_contig_hits   waafle/utils.py:207-241, 255-270  (+ derived scov / score)
 *   Locus / iter_contig_loci waafle/utils.py:300-322, 341-355
 * and the contig bookkeeping of waafle/waafle_orgscorer.py:348-357, 908-946.
 *
 * Contract: the parser accepts the plain spelling of every field (ASCII, tab separated,
 * '\n' line ends, no csv-quoted field, decimal integers, decimal / exponent floats).  Anything
 * else -- including every input the reference rejects -- returns WF_INGEST_FALLBACK with a
 * description in wf_ingest_last_error(); the caller then runs the reference-equivalent
 * Python reader, which either accepts the unusual spelling or raises the reference's
 * error.  Results are therefore identical to the Python reader by construction.
 *
 * Memory: every array is owned by the wf_ingest object and valid until wf_ingest_free().
 * A wf_ingest object is not thread-safe; distinct objects are independent.
 */
#ifndef WAAFLE_INGEST_H
#define WAAFLE_INGEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WF_INGEST_ABI_VERSION 3

enum wf_ingest_status {
  WF_INGEST_OK = 0,
  WF_INGEST_FALLBACK = 1,   /* input needs the Python reader (unusual spelling or an error) */
  WF_INGEST_E_IO = -1,      /* a file could not be opened or mapped */
  WF_INGEST_E_STATE = -2    /* call order / null arguments */
};

typedef struct wf_ingest wf_ingest;

/* Parsed inputs.  Strings are packed as blob + offsets ([count + 1] int64 offsets). */
typedef struct wf_ingest_view {
  int32_t n_contigs;            /* FASTA records (output contigs, FASTA order) */
  int32_t n_taxa;               /* distinct hit taxa (sseqid field 1) */
  int32_t n_systems;            /* distinct annotation systems, sorted (bit order) */
  int32_t n_warn_gff;           /* GFF contig groups not in the FASTA (in file order) */
  int32_t n_warn_blast;         /* BLAST contig groups not in the FASTA (in file order) */
  int32_t _pad;
  int64_t n_hits;               /* hits of FASTA contigs */
  int64_t n_loci;               /* loci kept by --min-gene-length */
  int64_t n_values;             /* annotation value texts (a text may repeat) */
  /* contigs */
  const char* contig_blob; const int64_t* contig_off;  /* names */
  const int64_t* contig_length;                        /* [n_contigs] summed line lengths */
  /* hits: CSR by FASTA contig, file order within a contig */
  const int64_t* hit_off;       /* [n_contigs + 1] */
  const int32_t* hit_qlo;       /* min(qstart, qend) */
  const int32_t* hit_qhi;       /* max(qstart, qend) */
  const int32_t* hit_taxon;     /* index into the taxa list below */
  const int8_t*  hit_strand;    /* 1 iff sstrand == "minus" (utils.py:214) */
  const double*  hit_score;     /* waafle_score (utils.py:229) */
  const double*  hit_scov;      /* scov_modified (utils.py:227) */
  const uint32_t* hit_sysmask;  /* bit s = system s annotated */
  const int64_t* hit_row;       /* blastout row of each hit */
  const int32_t* hit_value;     /* [n_hits * n_systems] value id (index into values), -1 */
  const char* taxa_blob; const int64_t* taxa_off;      /* [n_taxa] */
  const char* system_blob; const int64_t* system_off;  /* [n_systems] sorted */
  const char* value_blob; const int64_t* value_off;    /* [n_values] */
  const int32_t* value_system;  /* [n_values] system of each value (-1: unused system) */
  /* loci: CSR by FASTA contig, GFF order, length filter applied */
  const int64_t* loc_off;       /* [n_contigs + 1] */
  const int32_t* loc_start;
  const int32_t* loc_end;
  const int8_t*  loc_strand;    /* 0 '+', 1 '-', 2 other */
  const char* loc_strand_blob; const int64_t* loc_strand_off;   /* raw strand strings */
  /* warnings (orgscorer.py:944-946 and the GFF equivalent) */
  const char* warn_gff_blob; const int64_t* warn_gff_off;
  const char* warn_blast_blob; const int64_t* warn_blast_off;
  /* per contig: the LOCI output field, the kept loci's codes "start:end:strand" joined by
     '|' (orgscorer.py:795-800), [n_contigs + 1] offsets */
  const char* loci_blob; const int64_t* loci_off;
  /* a blastout not grouped by contig (ABI 3): per hit, its run of the contig's consecutive
     rows (0, 1, ...; hits stay in file order within a contig), or NULL when every contig's
     hits are one run.  The reference evaluates such a contig once per run
     (waafle_orgscorer.py:941-960); waafle_amd/regroup.py does the same over wf_score */
  const int32_t* hit_group;
} wf_ingest_view;

int wf_ingest_abi_version(void);
wf_ingest* wf_ingest_new(void);
void wf_ingest_free(wf_ingest* ing);
const char* wf_ingest_last_error(const wf_ingest* ing);
/* Parse the three files; threads <= 0 picks the hardware concurrency (capped at 64). */
int wf_ingest_parse(wf_ingest* ing, const char* fasta_path, const char* blastout_path,
                    const char* gff_path, double min_gene_length, int threads);
int wf_ingest_get_view(const wf_ingest* ing, wf_ingest_view* out);

#ifdef __cplusplus
}
#endif
#endif /* WAAFLE_INGEST_H */
