// Internal declarations shared by the HIP kernels (kernels.hip) and the host driver
// (driver.cpp).  Not part of the C ABI (see include/umiclust.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace uc {

constexpr int kMaxLen = 72;          // longest supported UMI (UMICLUST_MAX_LEN)
constexpr int kMinTplLen = 32;       // shortest query length with a compiled aligner
constexpr int kCodeWords = kMaxLen / 8;  // 4-bit codes, 8 residues per u32
constexpr int kMaxKmers = kMaxLen - 8 + 1;  // unique 8-mers per strand <= 65
constexpr int kKmerStride = 68;     // u16 slots per (sequence, strand) k-mer list
constexpr int kTile = 65536;        // centroids per index tile (u16 local ids)
constexpr int kTopHits = 41;        // maxaccepts + maxrejects + MAXDELAYED (searchcore.cc)
constexpr int kBatch = 8;           // MAXDELAYED: alignment batch of search_onequery
constexpr int kWalk = 32;           // maxaccepts + maxrejects - 1: most candidates ever aligned
constexpr int kPeerCap = 64;        // in-block peer candidates kept per query-strand
constexpr int kCandCap = 2048;      // LDS candidate buffer of the prefilter
constexpr int kOpsStride = 2 * kMaxLen;  // alignment ops per member (<= qlen + tlen)
constexpr int kConsCap = 2 * kMaxLen;    // consensus bytes reserved per cluster
constexpr int kMsaCols = 2048;      // LDS profile columns of the consensus kernel

struct Scoring {
  int32_t match, mismatch;
  int32_t go[6], ge[6];  // QL TL QI TI QR TR
  int32_t boundary_open;
};

// One index tile: CSR over 4^8 k-mers of up to kTile centroids, u16 local ids.
struct TileView {
  const uint32_t* off;     // [65537]
  const uint16_t* post;    // postings
  int32_t n;               // centroids in tile
  int32_t base;            // centroid ordinal of local id 0
};

struct DevSeqs {
  const uint32_t* codes;   // [(s*2+strand)*kCodeWords] 4-bit codes, sorted order
  const uint8_t* lens;     // [s]
  const uint16_t* kmers;   // [(s*2+strand)*kKmerStride]
  const uint8_t* nk;       // [s*2+strand]
};

// ---- kernel launchers (kernels.hip) ----
hipError_t launch_prep(const char* ascii, const int64_t* offs, const int32_t* perm, int32_t n,
                       int dust, uint32_t* codes, uint8_t* lens, uint16_t* kmers, uint8_t* nk,
                       char* masked, uint32_t* ambig, hipStream_t st);
hipError_t launch_index_count(const uint16_t* kmers, const uint8_t* nk, const int32_t* cent_seqno,
                              int32_t first, int32_t count, uint32_t* hist, hipStream_t st);
// hist_to_off: [65536] histogram followed by [65537] offsets
hipError_t launch_index_scan(uint32_t* hist_to_off, hipStream_t st);
hipError_t launch_index_fill(const uint16_t* kmers, const uint8_t* nk, const int32_t* cent_seqno,
                             int32_t first, int32_t count, const uint32_t* off, uint32_t* cursor,
                             uint16_t* post, hipStream_t st);
// prefilter: for query-strands qs in [0, nqs): query seqno = q0 + qs/2 (or qs if !both), strand.
struct PrefilterArgs {
  DevSeqs seqs;
  const TileView* tiles;   // device array
  int32_t ntiles;
  const int32_t* cent_seqno;  // centroid ordinal -> sorted seqno
  int32_t q0, nq;          // block of queries (sorted seqnos)
  int32_t both;            // strands per query (1 or 2)
  int32_t minwordmatches;
  // peer tiles: mini indexes over the + strand k-mers of the previous block and of this block
  // (base = first seqno, local id c = seqno - base; n = 0 if absent); together they cover the peer
  // window [peer_base, q0+nq), and a query sees the window entries before it
  TileView peer[2];
  int32_t peer_base;
  // outputs
  uint32_t* top_seqno;     // [nqs*kTopHits]
  uint8_t* top_count;      // [nqs*kTopHits]
  uint8_t* ntop;           // [nqs]
  uint16_t* peer_id;       // [nqs*kPeerCap] window-local (seqno - peer_base)
  uint8_t* peer_count;     // [nqs*kPeerCap]
  uint8_t* npeer;          // [nqs] (255 = overflow)
  uint32_t* postings_touched;  // [1] atomic counter (stats)
};
hipError_t launch_prefilter(const PrefilterArgs& a, hipStream_t st);

// alignment of pairs whose queries all have length qlen; pq = (query seqno << 1) | strand, pt = target seqno (plus strand)
// out[outidx ? outidx[k] : k] = matches | internal << 8 | (score & 0xffff) << 16.
// If dev_npairs != NULL only pairs k < *dev_npairs run (npairs is the launch bound).
hipError_t launch_align(const DevSeqs& s, int32_t qlen, bool ambig, const uint32_t* pq, const uint32_t* pt, int32_t npairs,
                        const uint32_t* dev_npairs, const uint32_t* outidx, const Scoring& sc,
                        uint32_t* out, hipStream_t st);

constexpr int kTabL = 2 * kMaxLen + 1;  // internal alignment length 0..144
constexpr int kTabM = kMaxLen + 1;      // matches 0..72
struct WalkState {
  unsigned long long lastkey;  // key of the last walked candidate
  uint32_t best_t;             // best accepted target seqno
  uint32_t cells;              // sum of qlen*tlen over walked candidates
  uint16_t best_rank;          // id rank of the best accepted hit
  uint8_t w;                   // candidates walked (aligned)
  uint8_t done;
  uint8_t acc;                 // an accepted hit exists
  uint8_t pad[3];
};
// round -1 initialises and emits batch 0; round r >= 0 evaluates batch r, emits batch r+1.
hipError_t launch_walk(int32_t round, int32_t q0, int32_t nqs, int32_t both,
                       const uint32_t* top_seqno, const uint8_t* top_count, const uint8_t* ntop,
                       const uint8_t* lens, const uint32_t* res, const uint8_t* acc_tab,
                       const uint16_t* rank_tab, WalkState* ws, uint32_t* pq, uint32_t* pt,
                       uint32_t* outidx, uint32_t* npairs, hipStream_t st);
hipError_t launch_peer_pairs(int32_t q0, int32_t w0, int32_t nqs, int32_t both, const uint16_t* peer_id,
                             const uint8_t* npeer, uint32_t* pq, uint32_t* pt, uint32_t* outidx,
                             uint32_t* npairs, hipStream_t st);
// traceback: ops[k*kOpsStride...] ('M','D','I' in alignment order), nops[k]
hipError_t launch_traceback(const DevSeqs& s, int32_t qlen, const uint32_t* pq, const uint32_t* pt,
                            int32_t npairs, const Scoring& sc, uint32_t* dirbuf, uint8_t* ops,
                            uint16_t* nops, uint32_t* out, hipStream_t st);
// consensus: cluster c members member_seqno[cstart[c] .. cstart[c+1]) (centroid first),
// member_ops index per member (-1 for centroid), member strand.
hipError_t launch_consensus(const DevSeqs& s, const int32_t* cstart, int32_t nclusters,
                            const int32_t* member_seqno, const int32_t* member_opsidx,
                            const uint8_t* member_strand, const uint8_t* ops,
                            const uint16_t* nops, char* cons, uint16_t* conslen,
                            int32_t* overflow, hipStream_t st);

}  // namespace uc
