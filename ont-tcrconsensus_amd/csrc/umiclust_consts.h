// Constants and host-visible layouts shared by the HIP kernels, the host driver and the host-only resolve core
// (resolve.cpp, built without HIP for the ThreadSanitizer harness).  Not part of the C ABI (include/umiclust.h).
#pragma once
#include <stdint.h>

namespace uc {

constexpr int kMaxLen = 112;         // longest supported UMI (UMICLUST_MAX_LEN; config 5 needs 110)
constexpr int kMinTplLen = 32;       // shortest query length with a compiled aligner
constexpr int kCodeWords = kMaxLen / 8;  // 4-bit codes, 8 residues per u32
constexpr int kMaxKmers = kMaxLen - 8 + 1;  // unique 8-mers per strand <= 105
constexpr int kKmerStride = (kMaxKmers + 3) & ~3;  // u16 slots per (sequence, strand) k-mer list
constexpr int kMaskWords = (kMaxLen + 31) / 32;    // DUST mask bits per sequence
static_assert(kMaxKmers <= 128, "k-mer slots are lanes l and l + 64");
static_assert(kMaxLen % 8 == 0 && kMaxLen <= 120, "summaries and keys hold lengths in 7 bits");
constexpr int kTile = 65536;        // centroids per sealed index tile
// Index layout.  Every posting list is split into kParts parts by the ordinal of its sequence
// (centroid ordinal, or seqno for the per-block peer tiles): part = x % kParts.  The prefilter runs
// one workgroup per (query-strand, part) and the launch maps part p to XCD p (workgroups are dealt
// to the 8 XCDs round-robin), so each XCD's L2 holds only its part of the index.  CSR bins are
// part-major (bin = part << 16 | k-mer) and every list is padded to a multiple of 8 postings
// (16-byte chunks; padding postings hit spare counters), so the counting loop needs no bounds.
// A posting IS its LDS counter index:
//   [r*kPeerRegion, (r+1)*kPeerRegion)  peer tile of a block in region r = block % depth (r < kPeerTiles)
//                                       (x - base) / kParts
//   [kDummy, kDummy + 64)         padding postings
//   [kTrash, kTrash + 256)        spare (lanes past the end of the posting stream add 0 instead)
//   [kCentBase, ...)              centroids: kCentBase + (ordinal % kSegCentroids) / kParts
// Centroids beyond kSegCentroids live in further counter segments, processed one after another.
constexpr int kParts = 8;
constexpr int kPartShift = 3;
constexpr int kBins = kParts << 16;
constexpr int kMaxBlock = 8192;                     // queries per greedy block
constexpr int kPeerRegion = kMaxBlock / kParts;     // counter slots per part of a peer tile
constexpr int kPeerTiles = 3;                       // blocks in a prefilter's peer window, at most
constexpr int kDummy = kPeerTiles * kPeerRegion;
constexpr int kTrash = kDummy + 64;
constexpr int kCentBase = kTrash + 256;
constexpr int kSegCentroids = 7 * kTile;            // counter indexes stay below 65536
constexpr int kMaxSegs = 16;
constexpr int kTopHits = 41;        // maxaccepts + maxrejects + MAXDELAYED (searchcore.cc)
constexpr int kBatch = 8;           // MAXDELAYED: alignment batch of search_onequery
constexpr int kWalk = 32;           // maxaccepts + maxrejects - 1: most candidates ever aligned
constexpr int kPeerCap = 128;       // in-window peer candidates kept per query-strand (a multiple of 64; <= 254:
                                    // u8 counts, 255 = overflow)
static_assert(kPeerCap % 64 == 0 && kPeerCap <= 254, "peer cap");
constexpr int kOpsStride = 2 * kMaxLen;  // alignment ops per member (<= qlen + tlen)
constexpr int kConsCap = 2 * kMaxLen;    // consensus bytes reserved per cluster
constexpr int kMsaCols = 2048;      // LDS profile columns of the consensus kernel

constexpr int kTabL = 2 * kMaxLen + 1;  // internal alignment length 0..2*kMaxLen
constexpr int kTabM = kMaxLen + 1;      // matches 0..kMaxLen
// per query-strand outcome of the device walk, as the host reads it (pinned host memory)
constexpr int kInlineRel = 6;  // relevant peers listed in HostQs itself
struct HostQs {
  uint32_t best_t;      // best accepted target seqno
  uint32_t cells;       // sum of qlen*tlen over walked candidates
  uint32_t rec;         // word offset of the record (relevant peers), 0xffffffff if none
  uint16_t best_rank;   // id rank of the best accepted hit
  uint8_t w;            // candidates walked
  uint8_t flags;        // bit 0: an accepted hit exists; bit 1: peer list overflow
  uint16_t nrel;        // relevant peers
  uint8_t e;            // walk candidates with an alignment result (record res[0, e))
  uint8_t npeer;        // peers counted in the window (<= kPeerCap; 255: overflow) -- the block-size feedback
  uint16_t rel[kInlineRel];  // the first kInlineRel of them (window ids), so the host reads the
                             // record only when one turns out to be a centroid (or nrel is larger)
};
static_assert(sizeof(HostQs) == 32, "HostQs layout");
constexpr int kRecWords = 1 + 2 * kWalk + kWalk / 4 + 2 * kPeerCap;  // largest record

}  // namespace uc
