// Internal declarations shared by the HIP kernels (kernels.hip) and the host driver
// (driver.cpp).  Not part of the C ABI (see include/umiclust.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "umiclust_consts.h"

namespace uc {

struct Scoring {
  int32_t match, mismatch;
  int32_t go[6], ge[6];  // QL TL QI TI QR TR
  int32_t boundary_open;
  int32_t wave_prio;  // alignment kernels: nonzero raises the waves' issue priority (s_setprio: round B, which the host
                      // waits for while the next pass's kernels share the SIMDs)
};

// One index tile: CSR over bins (part << 16 | k-mer); postings live in one arena shared by all tiles.
struct TileView {
  const uint32_t* off;     // [kBins + 1] tile-relative, each list a multiple of 8 postings
  uint64_t post_base;      // arena index of the tile's first posting
  int32_t n;               // sequences in the tile
  int32_t base;            // first centroid ordinal / first seqno (peer tiles)
  int32_t seg;             // counter segment (centroid tiles) / peer region 0|1 (peer tiles)
  int32_t len;             // peer tiles: the block's query length (one length per block)
};

struct DevSeqs {
  const uint32_t* codes;   // [(s*2+strand)*kCodeWords] 4-bit codes, sorted order
  const uint8_t* lens;     // [s]
  const uint16_t* kmers;   // [(s*2+strand)*kKmerStride]
  const uint8_t* nk;       // [s*2+strand]
};

// ---- kernel launchers (kernels.hip) ----
hipError_t launch_iota(int32_t* out, int32_t n, hipStream_t st);
hipError_t launch_prep(const char* ascii, const int64_t* offs, const int32_t* perm, int32_t n,
                       int dust, uint32_t* codes, uint8_t* lens, uint16_t* kmers, uint8_t* nk,
                       char* masked, uint32_t* ambig, hipStream_t st,
                       uint8_t* mchg = nullptr);
// XOR every k-mer of sequence s (both strands) with xmask[bin[s]] (packs: a bijection per bin)
hipError_t launch_kmer_xor(uint16_t* kmers, const uint8_t* nk, int32_t n, const int32_t* bin, const uint16_t* xmask,
                           hipStream_t st);
// index tile build over sequences c in [0, count) with seqno map[first + c] and ordinal
// x = xoff + c (centroid tiles: the centroid ordinal; peer tiles: c): count (hist[kBins], all zero
// on entry), scan (padded offsets off[kBins+1], fill cursors, padding postings written into post,
// hist re-zeroed), fill (posting = vbase + (x % seg_mod) / kParts)
constexpr int kScanPer = 1024;
constexpr int kScanBlocks = kBins / kScanPer;
hipError_t launch_index_count(const uint16_t* kmers, const uint8_t* nk, const int32_t* map, int32_t first,
                              int32_t count, int32_t xoff, uint32_t* hist, hipStream_t st);
hipError_t launch_index_scan(uint32_t* hist, uint32_t* partial, uint32_t* off, uint32_t* cursor, uint16_t* post,
                             hipStream_t st);
hipError_t launch_index_fill(const uint16_t* kmers, const uint8_t* nk, const int32_t* map, int32_t first,
                             int32_t count, int32_t xoff, int32_t vbase, int32_t seg_mod, uint32_t* cursor,
                             uint16_t* post, hipStream_t st);
// bank-aware posting order within every list of a tile (after the fill; kernels.hip k_list_arrange)
hipError_t launch_index_arrange(const uint32_t* off, uint16_t* post, hipStream_t st);
// the host-to-device half of an index append in one dispatch: n centroid seqnos / lengths, ns seq -> ordinal entries
// and nb bin-start ordinals, each read from pinned host memory and written to its device array
hipError_t launch_append_stage(const int32_t* hc, const uint8_t* hl, int32_t n, int32_t* dc, uint8_t* dl,
                               const int32_t* hs, int32_t* ds, int32_t ns, const int32_t* hb, int32_t* db, int32_t nb,
                               hipStream_t st);
// prefilter: for query-strands qs in [0, nqs): query seqno = q0 + qs/2 (or qs if !both), strand.
// postings-touched partial sums: slots counters[16 + 32 s], s < kPostSpread (separate L2 lines)
constexpr int kPostSpread = 32;
constexpr int kPartCand = 64;  // candidates a (query-strand, part) passes to the merge
// pass counters: [0..15] stats and pair counts, the postings partial sums, the overflowed-unit count
constexpr int kUnitsSlot = 16 + kPostSpread * 32;
// per-length pair counters of the three walk rounds (SegTab), kSegLens each
constexpr int kSegLens = 32;  // query lengths one greedy block may span
constexpr int kSegSlot = kUnitsSlot + 32;
constexpr int kCountersLen = kSegSlot + 3 * kSegLens;
constexpr int kPfWinBase = 128;   // k_pf_count: windows whose base list and start mask are tabulated (the rest: search)
// centroid tile views passed in the kernel arguments (a pass reads them by scalar loads either way; in the arguments
// they need no host-to-device copy, a blit dispatch between every two counting launches)
constexpr int kArgTiles = 32;
struct PrefilterArgs {
  DevSeqs seqs;
  const uint16_t* arena;   // postings of every tile
  const TileView* tiles;   // device array, centroid tiles in segment order (used when ntiles > kArgTiles)
  int32_t ntiles;
  TileView tv[kArgTiles];  // the same views when ntiles <= kArgTiles
  int32_t nseg;            // counter segments holding centroids (0 if none)
  int32_t seg_tile[kMaxSegs + 1];  // tiles of segment s: [seg_tile[s], seg_tile[s+1])
  uint64_t seg_base[kMaxSegs];     // lowest arena index a pass of segment s reads (peers: last pass)
  int32_t ncent;           // centroid ordinals [0, ncent) are indexed
  const int32_t* cent_seqno;  // centroid ordinal -> sorted seqno
  // centroids of length >= L, for L = 0..kMaxLen: lengths never increase with the ordinal (queries
  // are length-sorted, centroids appended in query order), so ordinal o has the largest L with
  // cnt_ge[L] > o
  int32_t cnt_ge[kMaxLen + 1];
  int32_t q0, nq;          // block of queries (sorted seqnos)
  int32_t both;            // strands per query (1 or 2)
  int32_t minwordmatches;
  // peer tiles: mini indexes over the + strand k-mers of the previous block and of this block
  // (base = first seqno, n = 0 if absent); together they cover the peer window [peer_base, q0+nq),
  // and a query sees the window entries before it
  TileView peer[kPeerTiles];  // oldest first, the block's own tile last (absent ones: n = 0)
  int32_t peer_base;
  int32_t nlist_cap;       // list-table capacity of the lean counting kernel (>= k-mers x tiles)
  int32_t pf1_lds;         // the lean counting kernel runs one-wave units when its LDS is at most this (bytes)
  // per-(query-strand, part) outputs, merged by launch_prefilter's last kernel: candidates (count >= the
  // threshold) as count << 24 | ordinal, unsorted, at most kPartCand (255 in pncand: overflow, re-run by
  // the full kernel, which writes its exact part top-41 in the same form)
  uint32_t* pcand;           // [nqs*kParts*kPartCand]
  uint8_t* pncand;           // [nqs*kParts]
  uint32_t* units;           // [nqs*kParts] overflowed (query-strand, part) units, *nunits of them
  uint32_t* nunits;  // (the merge resets *nunits to 0)
  // split passes (the counting of a block runs before the block two ahead of it is resolved): peer tile
  // flag_tile (>= 0) is that unresolved block; its hits become flagged candidates count << 24 | 1 << 23 |
  // (seqno - cand_base), kept by the merge if seq2ord[seqno] >= 0 (a centroid by then).  Stored peer ids
  // are relative to cand_base; the merge writes them relative to peer_base (id - peer_shift), and the full
  // kernel stores its own (peer_base-relative) ids + peer_id_add.
  int32_t flag_tile;
  int32_t cand_base;
  int32_t peer_shift;
  int32_t peer_id_add;
  const int32_t* seq2ord;  // [seqno] centroid ordinal or -1 (absolute seqnos)
  uint16_t* ppeer_id;        // [nqs*kParts*kPeerCap]
  uint8_t* ppeer_count;      // [nqs*kParts*kPeerCap]
  uint8_t* pnpeer;           // [nqs*kParts] (255 = overflow)
  uint32_t* ppost;           // [nqs*kParts] postings touched (stats; one atomic per merge workgroup)
  // outputs
  uint32_t* top_seqno;     // [nqs*kTopHits]
  uint8_t* top_count;      // [nqs*kTopHits]
  uint8_t* ntop;           // [nqs]
  uint16_t* peer_id;       // [nqs*kPeerCap] window-local (seqno - peer_base)
  uint8_t* peer_count;     // [nqs*kPeerCap]
  uint8_t* npeer;          // [nqs] (255 = overflow)
  uint32_t* postings_touched;  // counters[0]; the merge adds into kPostSpread slots 128 B apart after
                               // counters[16], which k_pack sums into the host copy of counters[0]
  unsigned long long* prof;    // [9] optional phase clocks of sampled workgroups (see k_prefilter), then their count
  // Packs (umiclust_cluster_pack: several bins in one greedy order, their k-mers XOR-scrambled per bin so other
  // bins' postings are sparse noise): query q of load bin qbin[q] takes centroid candidates only from ordinals >=
  // bin_ord0[bin] (INT32_MAX until the bin's first centroid is indexed) and peers / flagged hits only from
  // seqnos >= bin_seq0[bin]; k_pf_full keys centroids by cent_len (lengths are not monotone in the ordinal across
  // bins).  qbin == nullptr: one bin.
  const int32_t* qbin;
  const int32_t* bin_seq0;
  const int32_t* bin_ord0;
  const uint8_t* cent_len;
};
// two kernels: the per-part counting/selection (grid nqs*kParts) and the per-query-strand merge
// mode 0: the whole prefilter (lean counting + the full kernel over its overflowed units, or the full
// kernel alone for multi-segment bins, then the merge); mode 1: only the lean counting (a split pass's
// first half); mode 2: the full kernel over the units mode 1 left + the merge (its second half)
hipError_t launch_prefilter(const PrefilterArgs& a, hipStream_t st, int mode = 0);

// alignment of pairs whose queries all have length qlen; pq = (query seqno << 1) | strand, pt = target seqno (plus strand)
// out[outidx ? outidx[k] : k] = matches | internal << 8 | (score & 0xffff) << 16.
// If dev_npairs != NULL only pairs k < *dev_npairs run (npairs is the launch bound).  Launches of at most
// band_max pairs (one-hot codes) spread each pair over a lane group (k_align_band) instead of one lane.
hipError_t launch_align(const DevSeqs& s, int32_t qlen, bool ambig, const uint32_t* pq, const uint32_t* pt, int32_t npairs,
                        const uint32_t* dev_npairs, const uint32_t* outidx, const Scoring& sc,
                        uint32_t* out, hipStream_t st, int32_t band_max = 0);

struct WalkState {
  unsigned long long lastkey;  // key of the last walked candidate
  uint32_t best_t;             // best accepted target seqno
  uint32_t cells;              // sum of qlen*tlen over walked candidates
  uint16_t best_rank;          // id rank of the best accepted hit
  uint8_t w;                   // candidates walked (aligned)
  uint8_t done;
  uint8_t acc;                 // an accepted hit exists
  uint8_t e;                   // candidates emitted for alignment so far (results exist for [0, e))
  uint8_t pad[2];
};
// round -1 initialises and emits batch 0 -- or, speculatively, every candidate up to kWalk when the best
// candidate's k-mer count is below spec_thr (junk-like lists walk to the end);
// round r >= 0 evaluates every batch whose results exist and, if the walk goes on, emits all of its
// remaining candidates (up to kWalk): a pass has two dependent alignment launches, not five.
// Speculation changes which alignments are computed, never the walk: batches are evaluated in order.
// A block may hold several query lengths (the aligner is compiled per length): the walk and the peer pairs append
// their pairs to per-length segments, segment i = query length lmax - i at pair index base[i] (its capacity is the
// block's query-strands of that length x the pairs one can emit), counted in seg_cnt[i]; one alignment launch per
// segment.  Blocks span at most kSegLens lengths.
struct SegTab {
  int32_t lmax;
  int32_t nseg;
  uint32_t base[kSegLens];
};
hipError_t launch_walk(int32_t round, int32_t q0, int32_t nqs, int32_t both, int32_t spec_thr,
                       const uint32_t* top_seqno, const uint8_t* top_count, const uint8_t* ntop,
                       const uint8_t* lens, const uint32_t* res, const uint8_t* acc_tab,
                       const uint16_t* rank_tab, WalkState* ws, uint32_t* pq, uint32_t* pt,
                       uint32_t* outidx, const SegTab& sg, uint32_t* seg_cnt, unsigned long long* cells,
                       hipStream_t st);
// cells accumulates qlen x tlen of the pairs emitted (the cells the device computes for them)
hipError_t launch_peer_pairs(int32_t q0, int32_t w0, int32_t nqs, int32_t both, const uint8_t* lens,
                             const WalkState* ws, const uint16_t* peer_id, const uint8_t* peer_count,
                             const uint8_t* npeer, uint32_t* pq, uint32_t* pt, uint32_t* outidx, const SegTab& sg,
                             uint32_t* seg_cnt, unsigned long long* cells, uint32_t* nstat, uint32_t out0,
                             unsigned long long* aligned, int32_t emit, const WalkState* ws_prev,
                             const uint8_t* npeer_prev, int32_t q0_prev, int32_t nq_prev, hipStream_t st);
hipError_t launch_pack(int32_t nqs, int32_t w0, const uint8_t* lens, const WalkState* ws, const uint8_t* ntop,
                       const uint32_t* top_seqno, const uint8_t* top_count, const uint32_t* res,
                       const uint8_t* npeer, const uint16_t* peer_id, const uint8_t* peer_count,
                       const uint32_t* peer_res, const unsigned long long* aligned, uint32_t* reccount, HostQs* hq,
                       uint32_t* rec, uint32_t* counters, uint32_t* hcounters, uint32_t* hreccount, hipStream_t st);
// traceback (one wave per pair, any query length): ops[k*kOpsStride...] ('M','D','I' in alignment order,
// right-aligned in the slot), nops[k], out[k] as launch_align's
// maxl: the longest query or target length among the pairs (sizes the kernel's LDS)
// maxl: the launch's longest sequence; maxq: its longest query (0: maxl) -- every pair's query must fit it
hipError_t launch_traceback(const DevSeqs& s, const uint32_t* pq, const uint32_t* pt, int32_t npairs,
                            const Scoring& sc, uint8_t* ops, uint16_t* nops, uint32_t* out, hipStream_t st,
                            int32_t maxl, int32_t maxq = 0);
// consensus: cluster c members member_seqno[cstart[c] .. cstart[c+1]) (centroid first),
// member_ops index per member (-1 for centroid), member strand.
hipError_t launch_consensus(const DevSeqs& s, const int32_t* cstart, int32_t nclusters,
                            const int32_t* member_seqno, const int32_t* member_opsidx,
                            const uint8_t* member_strand, const uint8_t* ops,
                            const uint16_t* nops, char* cons, uint16_t* conslen,
                            int32_t* overflow, hipStream_t st);

// ---- region-vs-region UMI overlap (overlap.hip) ----
struct OvBuffers {
  uint64_t* hash;                 // [n]
  int32_t* region;                // [n]
  unsigned long long* keys;       // [m] slot hash (~0 = empty)
  unsigned long long* rep;        // [m] lowest member index
  int64_t* slot;                  // [n]
  uint32_t* cnt;                  // [m]
  uint32_t* start;                // [m + 1]
  uint32_t* cursor;               // [m]
  uint32_t* bsum;                 // [m / 1024 + 1]
  uint32_t* members;              // [n]
  uint32_t* collision;            // [1]
  uint32_t* big;                  // [n / (kOvSmallBucket + 1) + 1] slots whose buckets k_ov_pairs hands on
  uint32_t* nbig;                 // [1]
};
constexpr int kOvSmallBucket = 32;  // larger buckets (a UMI in many regions): one workgroup each, region histogram
// one hash-table pass over n sequences of nreg regions (region r = [rstart[r], rstart[r+1])), table of
// mask + 1 slots; csr also buckets the members by slot.  Synchronous; *collided != 0 means two different
// sequences shared a 64-bit hash (re-run with another seed).
hipError_t launch_overlap_table(const char* seqs, const int64_t* offs, int64_t n, const int64_t* rstart, int32_t nreg,
                                uint64_t seed, uint64_t hmask, uint64_t mask, const OvBuffers& B, bool csr,
                                uint32_t* collided, hipStream_t st);
// total[a * nreg + b] += c_a(s) c_b(s), maxc[a * nreg + b] = max c_b(s) over sequences s held by a and b (a < b)
hipError_t launch_overlap_pairs(const OvBuffers& B, uint64_t mask, int32_t nreg, unsigned long long* total,
                                uint32_t* maxc, hipStream_t st);
// two sets (region 0 = the first n1 sequences, region 1 = the rest): counts[i] = equal sequences in set 2
hipError_t launch_overlap_two(const OvBuffers& B, uint64_t mask, int64_t n, int64_t n1, int64_t* counts,
                              hipStream_t st);

// ---- UMI extraction (extract.hip) ----
struct ExtractPatterns {
  uint64_t peq[2][256];   // [fwd | rev pattern][byte]: bit i = pattern[i] equals the byte
  uint64_t peqr[2][256];  // same for the reversed pattern
  int32_t m[2];           // pattern lengths (1..64)
  int32_t pad[2];
};
// out[(i * 2 + w) * 3 ...] = (edit distance or -1, start, end) of edlib HW locations[0] in window w of read i
hipError_t launch_extract(const char* seqs, const int64_t* offs, int64_t n, int32_t a5, int32_t a3, int32_t k,
                          const ExtractPatterns* P, int32_t* out, hipStream_t st);
// the same on host-gathered windows (read i's at win[i * S ...], 5' window first, 3' at a5; lengths wlen[2i + w])
constexpr int kExMaxSlot = 252;  // S <= this: 128 slots fit the LDS staging of k_extract_win
hipError_t launch_extract_win(const char* win, const uint8_t* wlen, int64_t n, int32_t S, int32_t a5, int32_t k,
                              const ExtractPatterns* P, int32_t* out, hipStream_t st);

// ---- region binning of BAM records (regionsplit.hip) ----
enum : int8_t { kBamUnmapped = 0, kBamSecondary = 1, kBamShort = 2, kBamLong = 3, kBamKept = 4, kBamNoRegion = 5,
                kBamNoCluster = 6 };
// raw: uncompressed BAM, roff[r]: offset of record r's block_size field; ref_len / ref_cluster per BAM reference
// (-1: not in the reference FASTA / not in the cluster dict)
hipError_t launch_bam_classify(const uint8_t* raw, const int64_t* roff, int64_t n, int32_t nref, const int64_t* ref_len,
                               const int32_t* ref_cluster, double minov, int32_t s5, int32_t s3, int8_t* cls,
                               int32_t* cluster, int64_t* outlen, hipStream_t st);
hipError_t launch_bam_emit(const uint8_t* raw, const int64_t* roff, int64_t n, const int8_t* cls, const int64_t* pos,
                           char* out, hipStream_t st);

}  // namespace uc
