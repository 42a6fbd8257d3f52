/*
 * umiclust.h -- C ABI of the MI355X-native UMI clustering hot path.
 *
 * Drop-in for the `vsearch --cluster_fast ... --consout ... --clusters ...` subprocess that
 * the reference runs per region bin:
 *   - round 1: /root/reference/ont_tcr_consensus/vsearch_umi_cluster.py:8-56  (vsearch_cluster)
 *   - round 2: /root/reference/ont_tcr_consensus/vsearch_umi_cluster.py:59-99 (vsearch_cluster_consensus)
 * The reference's boundary is `subprocess.run(argv)` (vsearch_umi_cluster.py:21,71) with files
 * as the only data exchange; `umiclust_run_argv` accepts that exact argv, `umiclust_run_fasta`
 * the decoded parameters, and the session API (`umiclust_load` / `umiclust_cluster` /
 * `umiclust_fetch`) the in-memory form used by the benchmark (inputs resident in HBM).
 *
 * Conventions: plain C types only; every function returns 0 (or a count) on success and a
 * negative UMICLUST_E* code on failure, never throws across the ABI; one umiclust_ctx per
 * (process, GPU); a context is not thread-safe, distinct contexts are.
 */
#ifndef UMICLUST_H
#define UMICLUST_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UMICLUST_ABI_VERSION 9

/* error codes (negative returns) */
#define UMICLUST_OK 0
#define UMICLUST_EINVAL (-22)   /* bad argument / parameters / argv */
#define UMICLUST_EIO (-5)       /* file read/write failure */
#define UMICLUST_ENOMEM (-12)   /* host or device allocation failed */
#define UMICLUST_EDEVICE (-19)  /* no HIP device / HIP runtime error */
#define UMICLUST_ESTATE (-77)   /* call out of order (e.g. cluster before load) */
#define UMICLUST_ERANGE (-34)   /* a sequence exceeds the supported length (UMICLUST_MAX_LEN) */

#define UMICLUST_MAX_LEN 112    /* longest sequence the kernels are compiled for */

/* gap slots (vsearch --gapopen/--gapext letters): Q = gap in the query (CIGAR I, consumes the
 * target), T = gap in the target (CIGAR D, consumes the query); L/I/R = left end, interior,
 * right end. */
enum { UMICLUST_QL = 0, UMICLUST_TL = 1, UMICLUST_QI = 2, UMICLUST_TI = 3, UMICLUST_QR = 4,
       UMICLUST_TR = 5 };

typedef struct umiclust_params {
  double id;              /* --id */
  double weak_id;         /* vsearch --weak_id (fraction); only classifies rejects */
  int32_t minseqlength;   /* --minseqlength */
  int32_t maxseqlength;   /* --maxseqlength */
  int32_t wordlength;     /* --wordlength (8; the kernels require 8) */
  int32_t minwordmatches; /* --minwordmatches (12 for wordlength 8) */
  int32_t maxaccepts;     /* --maxaccepts (1) */
  int32_t maxrejects;     /* --maxrejects (32) */
  int32_t match;          /* --match */
  int32_t mismatch;       /* --mismatch */
  int32_t gap_open[6];    /* --gapopen, indexed by UMICLUST_QL..UMICLUST_TR */
  int32_t gap_ext[6];     /* --gapext */
  int32_t strand_both;    /* --strand both */
  int32_t qmask_dust;     /* --qmask dust (vsearch default) */
  int32_t clusterout_sort;/* --clusterout_sort */
  int32_t clusterout_id;  /* --clusterout_id */
  int32_t fasta_width;    /* --fasta_width (80) */
  int32_t policy_boundary_open; /* E(i,0)/F(0,j) opened from the DP
                                   boundary (1, default) or -inf (0) */
  int32_t threads;        /* --threads n (vsearch_umi_cluster.py:33-34,83-84; n >= 25 in the pipeline,
                             utils.py:56-63).  Only read under policy_threads = 1. */
  int32_t policy_threads; /* SURVEY Appendix C O4 [L]: 0 (default) = the sequential definition (vsearch
                             --threads 1, cluster_core_serial); 1 = vsearch's multithreaded cluster_fast
                             restated (cluster_core_parallel): rounds of `threads` queries, each searched
                             against the index frozen at the round's start, then re-checked in order against
                             the round's new centroids (inserted into its hit list by k-mer count and
                             re-walked one alignment at a time).  umiclust_params_from_argv sets 1 whenever
                             the argv's --threads is > 1 (the reference's --threads 25: since round 5, ABI 8),
                             unless the environment has UMICLUST_O4=sequential. */
} umiclust_params;

/* presets */
#define UMICLUST_PRESET_ROUND1 1          /* --gapopen 0E/40I --mismatch -40 --match 10 */
#define UMICLUST_PRESET_VSEARCH_DEFAULT 2 /* --match 2 --mismatch -4 --gapopen 20I/2E */

typedef struct umiclust_stats {
  int64_t n_input;        /* records read */
  int64_t n_kept;         /* records within [minseqlength, maxseqlength] */
  int64_t n_clusters;
  int64_t n_alignments;   /* alignments vsearch's procedure performs (GCUPS numerator set) */
  int64_t cells;          /* sum of Lq*Lt over those alignments */
  int64_t cells_computed; /* cells the GPU computed (incl. speculative work) */
  int64_t kmer_postings;  /* prefilter postings touched */
  int64_t n_blocks;       /* greedy blocks */
  double t_total_s;       /* wall time of umiclust_cluster */
  double t_prefilter_s;   /* kernel time, prefilter (HIP events) */
  double t_align_s;       /* kernel time, alignment */
  double t_consensus_s;   /* kernel time, traceback + consensus */
  double t_host_s;        /* host greedy resolve */
  int64_t n_deferred;     /* queries resolved by the host's exact merged walk (in-block peers) */
  int64_t pairs_round_b;  /* alignments issued for deferred queries */
  int64_t pairs_peer;     /* speculative in-block peer alignments */
  double t_index_s;       /* kernel time, index tile rebuilds */
  double t_sync_s;        /* host wall time blocked on device->host result copies */
  double t_host_pass1_s;  /* host first in-order pass of every block */
  int64_t n_merged_walks; /* (query, strand) walks the host re-ran with in-block centroids */
  double t_merged_s;      /* host time inside those merged walks */
  double t_read_s;        /* file path: FASTA read + parse (umiclust_run_fasta*) */
  double t_write_s;       /* file path: cluster<N> / consout (+ in-process parse) writing */
  double t_run_s;         /* file path: the whole call, read to files written */
  int64_t n_reruns;       /* block pieces re-run alone after an in-window peer list overflowed */
  int64_t n_overlap_passes; /* overlap hash-table passes (1 + re-seeds after 64-bit hash collisions) */
  int64_t n_lazy_passes;  /* passes whose in-window peers were aligned on demand (round B) only */
  double t_count_s;       /* kernel time, the prefilter's counting kernel alone (k_pf_count, HIP events) */
  int64_t n_count_launches; /* its launches (one per pass over one counter segment) */
  int64_t kmer_postings_deferred; /* postings of the lists the counting kernel deferred (frequent k-mers whose
                                     matches it adds per surviving target instead; x 8 chunks, incl. padding;
                                     0 since round 5: the deferral was removed) */
  int64_t counter_cells;  /* ABI 8: sum over the counting launches of query-strands x centroids indexed (the C of
                             SURVEY 8d's prefilter bytes, postings x 4 B + C x 2 B counter traffic) */
  int64_t n_regrows;      /* ABI 9: times a block size halved by a peer-list overflow doubled again (after `regrow`
                             clean, shallow blocks; UMICLUST_REGROW) */
} umiclust_stats;

typedef struct umiclust_ctx umiclust_ctx;

/* ---- versioning / parameters ---- */
int32_t umiclust_abi_version(void);
/* fill p with a preset (UMICLUST_PRESET_*) and the given identity / length window */
int32_t umiclust_params_init(umiclust_params *p, int32_t preset, double identity,
                             int32_t minseqlength, int32_t maxseqlength);
/* parse a vsearch argv (argv[0] may be "vsearch"); fills p and the path outputs (each
 * buffer of pathcap bytes, may be NULL).  Unknown options -> UMICLUST_EINVAL. */
int32_t umiclust_params_from_argv(umiclust_params *p, int32_t argc, const char *const *argv,
                                  char *in_fasta, char *clusters_prefix, char *consout,
                                  char *log_path, int32_t pathcap);

/* ---- context ---- */
/* device_id >= 0 selects a HIP device; there is no CPU backend (a missing device returns NULL
 * and sets *err = UMICLUST_EDEVICE). */
umiclust_ctx *umiclust_create(int32_t device_id, int32_t *err);
void umiclust_destroy(umiclust_ctx *ctx);
/* ABI 7: the context's main (counting) stream at the device's greatest stream priority (level 1) or a plain
 * stream (level 0, the default); its alignment stream is prioritised at both levels.  Level -1 (background):
 * every stream plain, the alignment stream included.  Lets a caller running several bins at once on one GPU
 * (BinRunner lanes; tcr_consensus.py:231-245 runs one vsearch per bin) put the bins that set the makespan ahead
 * of the others.  Synchronises the context first.  Results do not depend on it. */
int32_t umiclust_set_priority(umiclust_ctx *ctx, int32_t level);
/* Waits for the host work a file-path call (umiclust_run_fasta / _run_argv / _run_fasta_parse) leaves running after
 * it returns: the release of its input (unmapping a multi-GB FASTA, ~0.11 s for config 2's 3.5 GB) and of the fused
 * path's smolecule_clusters.fa mapping (RAM-backed outputs; the file's contents are in place before the call returns),
 * done on a thread of the context once every output is written.  The context's next file-path call and umiclust_destroy wait
 * for it too.  Returns UMICLUST_OK.  (Round 6; an added function, the struct layouts are unchanged.) */
int32_t umiclust_wait_host(umiclust_ctx *ctx);
/* human-readable message for the last error on this context */
const char *umiclust_last_error(const umiclust_ctx *ctx);

/* ---- whole-file drop-in (vsearch CLI semantics) ---- */
/* Reads in_fasta, clusters, writes <clusters_prefix><N> per cluster, the consout FASTA and a
 * text log.  Any output path may be NULL. Returns number of clusters (>=0) or an error. */
int64_t umiclust_run_fasta(umiclust_ctx *ctx, const umiclust_params *p, const char *in_fasta,
                           const char *clusters_prefix, const char *consout, const char *log_path,
                           umiclust_stats *stats);
/* same, from the exact vsearch argv the reference builds (vsearch_umi_cluster.py:22-53). */
int64_t umiclust_run_argv(umiclust_ctx *ctx, int32_t argc, const char *const *argv,
                          umiclust_stats *stats);

/* ---- in-process consumer ---- */
/* Parameters of the reference's parse_umi_clusters / polish_cluster
 * (/root/reference/ont_tcr_consensus/parse_umi_clusters.py:10-21, :143-151). */
typedef struct umiclust_parse_params {
  int32_t min_reads_per_cluster;  /* min_reads_per_cluster (20) */
  int32_t max_reads_per_cluster;  /* max_reads_per_cluster (60) */
  int32_t balance_strands;        /* balance_strands (0) */
  int32_t max_clusters;           /* max_clusters; 0 = no limit (the reference's None); any other value
                                     stops once n_written > max_clusters, as Python's truthiness does */
} umiclust_parse_params;

typedef struct umiclust_parse_result {
  int64_t n_clusters;     /* consout records */
  int64_t n_written;      /* clusters written to clusters_fa/ */
  int64_t reads_found;    /* the reference's running total as it computes it (last cluster's count x 2) */
  int64_t reads_written;  /* likewise */
  int32_t empty_region;   /* 1: n_written == 0 or reads_found == 0 -- the caller appends the region to
                             regions_wo_clusters_txt (parse_umi_clusters.py:222-231) and no log is written */
  int32_t pad;
} umiclust_parse_result;

/* Replaces the vsearch_cluster -> parse_umi_clusters task pair (tcr_consensus.py:237-265 round 1,
 * :419-444 round 2; consumer parse_umi_clusters.py:10-242).
 * umiclust_run_fasta followed by parse_umi_clusters' outputs straight from the in-memory clusters:
 * <work_dir>/clusters_fa/cluster<N>.fasta, <work_dir>/smolecule_clusters.fa,
 * <work_dir>/vsearch_cluster_stats.tsv and <work_dir>/parse_cluster.log, byte-identical to running
 * the reference's parse_umi_clusters on the files umiclust_run_fasta writes (work_dir = the consout's
 * directory; clusterout_sort and clusterout_id must be set).  clusters_prefix may be NULL: the
 * per-cluster vsearch files, which the consumer only re-reads, are then not written at all.
 * <work_dir>/clusters_fa must not exist (UMICLUST_EEXIST).  A record header without the 7
 * `;`-separated fields or a strand other than + / - is UMICLUST_EFORMAT (the reference raises). */
#define UMICLUST_EEXIST (-17)   /* output directory already exists */
#define UMICLUST_EFORMAT (-74)  /* a record header does not follow the extract_umis format */
int64_t umiclust_run_fasta_parse(umiclust_ctx *ctx, const umiclust_params *p, const char *in_fasta,
                                 const char *clusters_prefix, const char *consout, const char *log_path,
                                 const umiclust_parse_params *pp, const char *work_dir,
                                 umiclust_parse_result *result, umiclust_stats *stats);

/* ---- session API (in-memory, inputs resident in HBM) ---- */
/* Stage n sequences (concatenated ASCII `seqs`, record i at [offsets[i], offsets[i+1])) into
 * device memory, then prepare them (umiclust_prepare).  = umiclust_stage + umiclust_prepare. */
int32_t umiclust_load(umiclust_ctx *ctx, const umiclust_params *p, const char *seqs,
                      const int64_t *offsets, int64_t n);
/* The two halves of umiclust_load (ABI 6).  umiclust_stage copies the raw records into HBM (bin_start as in
 * umiclust_load_bins; NULL = one bin) and keeps them resident.  umiclust_prepare does vsearch's load-time work on
 * the staged records (the length filter, DUST soft-masking and the stable length sort that
 * `vsearch --cluster_fast` runs before clustering; vsearch_umi_cluster.py:21-54 starts it): the length
 * filter and sort on the host, DUST, 4-bit codes and unique 8-mers on the device.  It may be called again with
 * other parameters (or the same, benchmarking: the headline times umiclust_prepare + umiclust_cluster). */
int32_t umiclust_stage(umiclust_ctx *ctx, const char *seqs, const int64_t *offsets, int64_t n,
                       const int64_t *bin_start, int32_t nbins);
int32_t umiclust_prepare(umiclust_ctx *ctx, const umiclust_params *p);
/* Run the hot path on the loaded sequences (prefilter, alignment, greedy, consensus).
 * Returns number of clusters. May be called repeatedly (benchmarking). */
int64_t umiclust_cluster(umiclust_ctx *ctx, umiclust_stats *stats);
/* Fetch results for the input records (input order):
 *   cluster[i]  output cluster number (clusterout_sort numbering), -1 if length-filtered
 *   strand[i]   0 '+', 1 '-' (orientation of record i relative to its centroid)
 *   centroid[i] 1 if record i is its cluster's centroid
 * and the consensus sequences: cluster c is cons[cons_off[c] .. cons_off[c+1]) (cons_off has
 * n_clusters+1 entries; cons capacity cons_cap bytes). Any pointer may be NULL. */
int64_t umiclust_fetch(umiclust_ctx *ctx, int32_t *cluster, uint8_t *strand, uint8_t *centroid,
                       char *cons, int64_t cons_cap, int64_t *cons_off);

/* ---- many region bins per load (BASELINE configs 3 and 4) ---- */
/* The reference runs one vsearch process per (library x region bin) (tcr_consensus.py:231-245 round 1,
 * :411-427 round 2).  A load may hold many such bins resident in HBM at once: bin b is input records
 * [bin_start[b], bin_start[b+1]) (bin_start has nbins+1 entries, bin_start[0] = 0, bin_start[nbins] = n).
 * Every bin is length-filtered, sorted and clustered on its own, exactly as its own vsearch run would
 * be; umiclust_load / umiclust_cluster / umiclust_fetch are the nbins = 1 case. */
int32_t umiclust_load_bins(umiclust_ctx *ctx, const umiclust_params *p, const char *seqs,
                           const int64_t *offsets, int64_t n, const int64_t *bin_start, int32_t nbins);
/* cluster one bin of the load; returns its number of clusters */
int64_t umiclust_cluster_bin(umiclust_ctx *ctx, int32_t bin, umiclust_stats *stats);
/* cluster the bins [first, first + nbins) of the load as one pack: the bins' queries in one greedy order (each bin
 * sorted on its own, the bins one after another), so small bins share the GPU passes of the bins around them.  Every
 * bin's result is exactly its own vsearch run's (tcr_consensus.py:231-245 runs one vsearch per bin); fetch each with
 * umiclust_fetch_bin.  Stats cover the whole pack; returns the pack's number of clusters.  Under the batched O4
 * policy every bin's rounds are counted from its own first sorted query. */
int64_t umiclust_cluster_pack(umiclust_ctx *ctx, int32_t first, int32_t nbins, umiclust_stats *stats);
/* umiclust_fetch for one clustered bin: arrays over the bin's input records (bin-local index) */
int64_t umiclust_fetch_bin(umiclust_ctx *ctx, int32_t bin, int32_t *cluster, uint8_t *strand,
                           uint8_t *centroid, char *cons, int64_t cons_cap, int64_t *cons_off);

/* ---- region-vs-region UMI overlap ---- */
/* Replaces the Python string scans of /root/reference/ont_tcr_consensus/extract_umis.py.
 * umiclust_overlap_counts: count_single_umi_overlaps (:270-290) for every UMI of set 1 at once:
 *   counts[i] = number of set-2 sequences byte-equal to set-1 sequence i.
 * umiclust_overlap_regions: count_overlapping_umis_between_2_regions (:293-342) for every region pair of
 *   count_overlapping_umis_between_all_regions (:345-369): region r = sequences [region_start[r],
 *   region_start[r+1]); for a < b, total[a * nregions + b] = the pair's summed count (the TSV value) and
 *   maxcount[a * nregions + b] = the largest count of one region-a UMI (> 1 = the warning).  Entries with
 *   a >= b are 0.  A GPU hash join: exact (byte comparison; a 64-bit hash collision re-runs with another
 *   seed). */
#define UMICLUST_OVERLAP_MAX_REGIONS 4096
int32_t umiclust_overlap_counts(umiclust_ctx *ctx, const char *seqs1, const int64_t *offsets1, int64_t n1,
                                const char *seqs2, const int64_t *offsets2, int64_t n2, int64_t *counts);
int32_t umiclust_overlap_regions(umiclust_ctx *ctx, const char *seqs, const int64_t *offsets, int64_t n,
                                 const int64_t *region_start, int32_t nregions, int64_t *total,
                                 int32_t *maxcount);

/* ---- UMI extraction ---- */
/* Replaces extract_umis (/root/reference/ont_tcr_consensus/extract_umis.py:189-267): per read, the first
 * adapter_length_5_end and the last adapter_length_3_end bases (:110-126) are searched for umi_fwd / umi_rev
 * as edlib does (:89-107: mode "HW", task "path", k = max_pattern_dist, the IUPAC additionalEqualities of
 * :26-87).  umiclust_extract_umis: out[i*6 + 0..2] = (edit distance or -1, start, end) of the 5' UMI in
 * its window, out[i*6 + 3..5] of the 3' UMI.  umiclust_extract_umis_file: FASTA or FASTQ in, the
 * <region>_detected_umis.fasta records of write_fasta (:154-186) out, in input order; returns the number
 * of reads with both UMIs (the reference's n_both_umi).  Patterns of 1..64 symbols.  A record name
 * without "strand=" is UMICLUST_EFORMAT ("Read strand not annotated!"). */
int32_t umiclust_extract_umis(umiclust_ctx *ctx, const char *seqs, const int64_t *offsets, int64_t n,
                              int32_t adapter_length_5_end, int32_t adapter_length_3_end,
                              int32_t max_pattern_dist, const char *umi_fwd, const char *umi_rev, int32_t *out);
int64_t umiclust_extract_umis_file(umiclust_ctx *ctx, const char *fastx_file, const char *out_fasta,
                                   int32_t adapter_length_5_end, int32_t adapter_length_3_end,
                                   int32_t max_pattern_dist, const char *umi_fwd, const char *umi_rev);

/* ---- region binning ---- */
/* Replaces the record loop of filter_and_split_reads_by_region_cluster
 * (/root/reference/ont_tcr_consensus/region_split.py:219-333): BAM in (BGZF inflated on the host threads,
 * records classified and FASTA records built on the device), every kept primary alignment appended to
 * <out_dir>/region_cluster<k>.fasta as `>{query_name};strand={+|-}` + its forward sequence, in BAM order.
 * Regions come from the reference FASTA (names, lengths) and the cluster JSON (region_clusters[r], -1 if the
 * region is not in it).  counts = {n_unmapped, n_primary_mapped, n_short, n_long} of the records the
 * reference's loop reaches; reads_per_cluster[k] (ncluster_cap entries); region_detected[r] = 1 if a kept
 * record aligned to region r.  Returns the number of cluster files appended to.  A record aligned to a
 * reference missing from the regions (or from the cluster JSON once it passes the filters) stops the loop
 * as the reference's KeyError does: the records before it are written and UMICLUST_EFORMAT is returned with
 * the name in missing_name. */
int64_t umiclust_region_split(umiclust_ctx *ctx, const char *bam_file, int32_t nregions,
                              const char *const *region_names, const int64_t *region_lengths,
                              const int32_t *region_clusters, double minimal_region_overlap,
                              int32_t max_softclip_5_end, int32_t max_softclip_3_end, const char *out_dir,
                              int64_t *counts, int64_t *reads_per_cluster, int32_t ncluster_cap,
                              uint8_t *region_detected, char *missing_name, int32_t missing_cap);

/* ---- kernel-level entry points (parity tests) ---- */
/* Align npairs (query, target) pairs with the production alignment kernel.  Sequences are
 * ASCII; q/t record k at [q_off[k], q_off[k+1]).  Outputs per pair: score, matches,
 * internal alignment length (columns minus the terminal gap runs, vsearch align_trim) and,
 * if cigar_ops != NULL, the alignment ops ('M','D','I', alignment order) at
 * cigar_ops[k*ops_stride ...] with their count in ops_len[k]. */
int32_t umiclust_align_pairs(umiclust_ctx *ctx, const umiclust_params *p, const char *q,
                             const int64_t *q_off, const char *t, const int64_t *t_off,
                             int64_t npairs, int32_t *score, int32_t *matches,
                             int32_t *internal_len, char *cigar_ops, int32_t ops_stride,
                             int32_t *ops_len);
/* DUST-mask and extract unique 8-mers of n sequences on the device (K1). masked receives the
 * case-masked sequences (same layout as seqs); kmers[i*kstride ...] the sorted unique k-mer
 * codes of strand s (0 '+', 1 '-') at kmers[(2*i+s)*kstride], counts in nk[2*i+s]. */
int32_t umiclust_prep(umiclust_ctx *ctx, const umiclust_params *p, const char *seqs,
                      const int64_t *offsets, int64_t n, char *masked, uint16_t *kmers,
                      int32_t kstride, int32_t *nk);

/* ---- measurement (bench.py; no reference counterpart) ---- */
/* Process-wide device timeline of the counting launches (kind 0) and the alignment chains
 * (kind 1) of every context: busy_s = the union of their HIP-event brackets since the last
 * reset, launches = the number of brackets.  reset != 0 clears it and records a new
 * reference event on device_id first.  Several contexts (lanes) on one device overlap their
 * brackets, so the union is the time the kernel held the device, and the sum is not. */
int32_t umiclust_timeline(int32_t device_id, int32_t kind, int32_t reset, double *busy_s,
                          int64_t *launches);

#ifdef __cplusplus
}
#endif
#endif
