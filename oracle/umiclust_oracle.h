/*
 * umiclust_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * A C restatement of the arithmetic behind the reference's hot path:
 *   `vsearch --cluster_fast <fa> --strand both --id X --clusters <dir>/cluster --consout ...
 *    --clusterout_id --clusterout_sort [--gapopen 0E/40I --mismatch -40 --match 10]`
 * as driven by /root/reference/ont_tcr_consensus/vsearch_umi_cluster.py:21-54 (round 1) and
 * :71-97 (round 2).  The arithmetic itself lives in the third-party program vsearch
 * (torognes/vsearch, pinned `vsearch>=2.29.0` at pyproject.toml:39 and `>=2.29.1` at
 * ont_tcr_consensus.yml:12), which is NOT vendored in the reference and not present in
 * this image.  This file restates vsearch 2.29's published algorithm (cluster.cc,
 * searchcore.cc, align_simd.cc, msa.cc, mask.cc, unique.cc, minheap.cc) as summarised in
 * SURVEY.md Appendix A.  PARITY UNPINNED: no vsearch binary, source or golden output exists
 * offline, and the reference ships no tests/fixtures for this path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library -- as the checker, never as the product path.
 */
#ifndef UMICLUST_ORACLE_H
#define UMICLUST_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* gap-penalty slots: a "query gap" consumes target residues (CIGAR 'I', horizontal move),
 * a "target gap" consumes query residues (CIGAR 'D', vertical move). */
enum { ORC_QL = 0, ORC_TL = 1, ORC_QI = 2, ORC_TI = 3, ORC_QR = 4, ORC_TR = 5 };

typedef struct orc_params {
  double id;             /* --id */
  double weak_id;        /* vsearch default 10.0 clipped to id (cluster.cc) */
  int32_t minseqlength;  /* --minseqlength */
  int32_t maxseqlength;  /* --maxseqlength */
  int32_t wordlength;    /* 8 */
  int32_t minwordmatches;/* 12 for k=8 */
  int32_t maxaccepts;    /* 1 */
  int32_t maxrejects;    /* 32 */
  int32_t match;         /* --match */
  int32_t mismatch;      /* --mismatch (negative) */
  int32_t gap_open[6];   /* ORC_QL..ORC_TR, positive penalties */
  int32_t gap_ext[6];
  int32_t strand_both;   /* --strand both */
  int32_t qmask_dust;    /* --qmask dust (default) */
  int32_t clusterout_sort;
  int32_t clusterout_id;
  int32_t fasta_width;   /* 80 */
  int32_t policy_boundary_open; /* O3b: E(i,0)/F(0,j) opened from the boundary H (1) or -inf (0) */
  int32_t threads;       /* --threads (vsearch_umi_cluster.py:33-34; >= 25 in the pipeline, utils.py:56-63) */
  int32_t policy_threads;/* O4 [L]: 0 = the sequential definition (cluster_core_serial, --threads 1);
                            1 = cluster_core_parallel restated: rounds of `threads` queries searched
                            against the index frozen at the round's start, then, in order, each query
                            re-checked against the round's new centroids (inserted into its hit list by
                            k-mer count and re-walked one alignment at a time) */
                         /* policy_threads = 1 with the environment's ORC_WORKERS = n: the round's searches run
                            on n OpenMP worker threads (results unchanged) */
} orc_params;

/* presets: 1 = round 1 (vsearch_umi_cluster.py:44-50: --gapopen 0E/40I --mismatch -40
 * --match 10), 2 = vsearch defaults (round 2, :71-97). */
void orc_params_preset(orc_params *p, int preset, double id, int minlen, int maxlen);

/* global alignment of q vs t (vsearch search16 + backtrack16 semantics).
 * Writes stats; cigar (vsearch run-length form, NUL-terminated) if cigar != NULL
 * (buffer >= 2*(qlen+tlen)+1). Returns the alignment score. */
int orc_align(const orc_params *p, const char *q, int qlen, const char *t, int tlen,
              int *columns, int *matches, int *mismatches, int *gaps,
              int *trim_left, int *trim_right, int *internal_len, double *id2, char *cigar);

/* DUST soft-mask (mask.cc): upper-cases seq then lower-cases masked intervals, in place. */
void orc_dust(char *seq, int len);

/* unique k-mers (unique.cc) of seq, skipping k-mers that touch a lower-case residue when
 * mask != 0. Codes written in first-seen order; returns the count. */
int orc_unique_kmers(const char *seq, int len, int k, int mask, uint32_t *out);

/* full clustering of n sequences (already in memory, in input order).
 * out_cluster[i]  : output cluster number of input record i (-1: length-filtered out)
 * out_strand[i]   : 0 = plus, 1 = minus (centroids: 0)
 * out_centroid[i] : 1 if record i is a centroid
 * out_sorted[k]   : input index of the k-th sequence after the length sort
 * cons_buf/cons_off: consensus of output cluster c is cons_buf[cons_off[c] .. cons_off[c+1])
 *                  (cons_buf capacity cons_cap; cons_off needs n+1 entries)
 * stats[0..7]     : {kept, clusters, alignments, cells, kmer_postings, candidates, dust_masked_seqs, 0}
 * masked_out (optional, n*maxlen): DUST-masked sequences of kept records (input order)
 * Returns number of clusters, or <0 on error. */
int64_t orc_cluster(const orc_params *p, int32_t n, const char *const *seqs, const int32_t *lens,
                    int32_t *out_cluster, uint8_t *out_strand, uint8_t *out_centroid,
                    int32_t *out_sorted, char *cons_buf, int64_t cons_cap, int64_t *cons_off,
                    int64_t *stats);

/* vsearch-like CLI run: read FASTA, cluster, write <clusters_prefix><N> files and consout.
 * Any output path may be NULL. Returns number of clusters or <0 on error. */
int64_t orc_run_fasta(const orc_params *p, const char *in_fasta, const char *clusters_prefix,
                      const char *consout, int64_t *stats);

#ifdef __cplusplus
}
#endif
#endif
