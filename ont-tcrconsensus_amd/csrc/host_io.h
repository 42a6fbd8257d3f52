// host_io.h -- the HIP-free host side of the drop-in boundary: FASTA/FASTQ input, the vsearch output
// writers (--consout, --clusters), the in-process parse_umi_clusters, the vsearch argv
// grammar, BGZF inflation (f4) and the detected-UMI writer (f1).  Compiled by g++ (no HIP), so the CPU
// suite builds it with ASan/UBSan (tests/test_sanitizers_cpu.py, tools/host_asan_main.cpp).  Not part of the
// C ABI except umiclust_params_init / umiclust_params_from_argv, which it defines.
#pragma once
#include <stdint.h>

#include <string>
#include <memory>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/umiclust.h"

namespace uc {
namespace io {

// A failure of an I/O-side step: an UMICLUST_E* code and a message (driver.cpp turns it into the context's
// error; nothing is thrown across the C ABI).
struct IoError {
  int code;
  std::string msg;
};

// CPUs this process may use: its affinity mask, bounded by the cgroup CPU quota (cpu.max) when one is set
int host_cpus();
// writer / parser threads of one call: UMICLUST_IO_THREADS, else the process's CPUs shared among the device contexts
// alive (set_live_contexts; a bin-set runner's lanes write concurrently), at most 16
int io_threads();
void set_live_contexts(int n);

// run f(t) for t in [0, T) on T threads (the caller's thread runs t = 0)
template <typename F>
void parallel_for(int T, F&& f) {
  std::vector<std::thread> th;
  for (int t = 1; t < T; t++) th.emplace_back([&f, t] { f(t); });
  f(0);
  for (auto& x : th) x.join();
}

// std::allocator without value-initialisation on resize (large arrays filled in parallel right after)
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <class U>
  NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept {
    ::new ((void*)p) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new ((void*)p) U(std::forward<A>(a)...);
  }
};
template <class T>
using RawVec = std::vector<T, NoInitAlloc<T>>;

// The input FASTA (or FASTQ), memory-mapped; labels point into the mapping, sequences are copied out.
struct Fasta {
  const char* data = nullptr;     // file contents (mapping)
  size_t size = 0;
  void* map = nullptr;
  RawVec<int64_t> hdr_off;   // label start (after '>' / '@')
  RawVec<int32_t> hdr_len;   // label length (truncated at whitespace)
  RawVec<char> seq;          // concatenated sequences
  RawVec<int64_t> seq_off;   // n+1
  Fasta() = default;
  Fasta(const Fasta&) = delete;
  Fasta& operator=(const Fasta&) = delete;
  ~Fasta();
  void release();  // unmap the file and free the arrays
};
// vsearch's FASTA reader: labels truncated at the first whitespace, sequence lines keep letters only, lines
// before the first '>' ignored; parsed by io_threads() threads over slices of the mapping
bool read_fasta(const char* path, Fasta& f);
// pysam.FastxFile's FASTQ records: '@' name, sequence lines up to '+', as many quality characters
bool read_fastq(const char* path, Fasta& f);

// clusters in output order: cluster k = sorted seqnos omemb[ostart[k] .. ostart[k+1]) (centroid first), input
// record of sorted seqno s = perm[s]
struct ClusterView {
  int32_t K = 0;
  const int32_t* ostart = nullptr;
  const int32_t* omemb = nullptr;
  const int32_t* perm = nullptr;
};

// clusters [0, K) split over T threads by member count
std::vector<int32_t> cluster_slices(const int32_t* ostart, int32_t K, int T);

// --consout: >centroid=<label>;seqs=<m>[;clusterid=<k>] + the consensus of cluster k, wrapped at width
void write_consout(const char* path, const Fasta& f, const ClusterView& cv, const char* cons, const int64_t* cons_off,
                   bool clusterout_id, int width);
// --clusters: <prefix><k> per cluster, the members' labels and masked sequences (masked[s * stride], length
// hlen[s]) in cluster order; masked == nullptr: every sequence prints as its input bytes (no sequence changed);
// mrow != nullptr: sorted seqno s prints masked row mrow[s], or its input bytes where mrow[s] < 0
void write_cluster_files(const char* prefix, const Fasta& f, const ClusterView& cv, const char* masked, int stride,
                         const uint8_t* hlen, int width, const int32_t* mrow = nullptr);
// a small text file (the log)
void write_text(const char* path, const std::string& text);
// whole-buffer write / create-write-close (false on an I/O error)
bool write_all(int fd, const char* p, size_t n);
bool write_file(const std::string& path, const std::string& data);

// parse_umi_clusters / polish_cluster (/root/reference/ont_tcr_consensus/parse_umi_clusters.py:10-242) on the
// in-memory clusters: <work_dir>/clusters_fa/cluster<k>.fasta, smolecule_clusters.fa, vsearch_cluster_stats.tsv,
// parse_cluster.log; byte-identical to the reference run on the vsearch files
// The per-record header fields parse_clusters needs (cols[0], the strand, cols[6] and its seq= read), computed
// ahead -- the fused drop-in runs it on a few threads while the GPU clusters.  ok = 0: the header does not have 7
// fields or a valid strand= field (parse_clusters re-derives the reference's error from the header).
struct RecFields {
  uint32_t id_n = 0, last_off = 0, last_n = 0, read_n = 0;
  int32_t read_off = -1;  // -1: cols[6] has no seq=
  uint8_t ok = 0, strand = 0;
};
void precompute_fields(const Fasta& f, std::vector<RecFields>& out, int threads);
// unmap: when given, the smolecule file's shared mapping (RAM-backed outputs) is handed over instead of unmapped, for
// the caller to release once the call has returned (its contents are in the page cache already)
void parse_clusters(const Fasta& f, const ClusterView& cv, const umiclust_parse_params* pp, const char* work_dir,
                    umiclust_parse_result* pr, const RecFields* pre = nullptr,
                    std::vector<std::pair<void*, size_t>>* unmap = nullptr);

// write_fasta of extract_umis (/root/reference/ont_tcr_consensus/extract_umis.py:154-186) for records [0, ngood):
// res[i*6 ..] = (dist, start, end) of the 5' and 3' UMI in their windows; returns the reads with both UMIs
int64_t write_detected_umis(const char* path, const Fasta& f, const int32_t* res, int64_t ngood, int32_t a3);

// BGZF (SAM/BAM specification §4.1) inflated on the host threads
bool inflate_bgzf(const char* path, std::vector<uint8_t>& raw);

// the reference's string helpers
struct Sv {
  const char* p;
  size_t n;
  std::string str() const { return std::string(p, n); }
  bool operator==(const char* s) const;
};
bool split1(Sv s, const char* sep, Sv& out);  // Python s.split(sep)[1]
std::string pjoin(const std::string& a, const std::string& b);  // os.path.join(a, b), b relative

}  // namespace io
}  // namespace uc
