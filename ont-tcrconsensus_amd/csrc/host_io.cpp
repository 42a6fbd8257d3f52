// host_io.cpp -- the HIP-free host side of the drop-in boundary (see host_io.h).  Built by g++; the CPU
// suite builds it again with ASan/UBSan and drives it from tools/host_asan_main.cpp.
#include "host_io.h"

#include <fcntl.h>
#include <sys/uio.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/statfs.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace uc {
namespace io {

int host_cpus() {
  static const int n = [] {
    int cpus = (int)std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) cpus = CPU_COUNT(&set);
    // cgroup v2 quota "max 100000" or "<quota> <period>" (the GPU box: 1600000 100000 = 16 CPUs of 256 visible)
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long per = 0;
      if (fscanf(f, "%31s %ld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0) {
        const long quota = atol(q);
        if (quota > 0) cpus = std::min<int>(cpus, (int)((quota + per - 1) / per));
      }
      fclose(f);
    }
    return std::max(1, cpus);
  }();
  return n;
}

static std::atomic<int> g_io_ctx{1};
void set_live_contexts(int n) { g_io_ctx.store(std::max(1, n)); }

// 16 threads per call with 8 lanes writing at once oversubscribed the box's 16-CPU quota: config 4's file
// boundary at quarter scale, round 2 0.29 -> 0.63 M UMIs/s with 4 threads per lane (profiles/r05/io_threads_ab)
int io_threads() {
  static const int env = [] {
    const char* e = getenv("UMICLUST_IO_THREADS");
    return e ? std::max(1, std::min(atoi(e), 16)) : 0;
  }();
  if (env) return env;
  return std::max(1, std::min(16, host_cpus() / g_io_ctx.load()));
}

Fasta::~Fasta() { release(); }

void Fasta::release() {
  if (map) munmap(map, size);
  map = nullptr;
  data = nullptr;
  size = 0;
  RawVec<int64_t>().swap(hdr_off);
  RawVec<int32_t>().swap(hdr_len);
  RawVec<char>().swap(seq);
  RawVec<int64_t>().swap(seq_off);
}

struct FastaPart {
  std::vector<int64_t> hdr_off;
  std::vector<int32_t> hdr_len;
  std::vector<char> seq;
  std::vector<int64_t> seq_off;
};

// records starting in [a, b) (a is a record start or 0): headers are truncated at the first whitespace
// (vsearch without --notrunclabels); sequence lines keep letters only; lines before the first '>' are
// ignored
void parse_fasta_range(const char* d, size_t a, size_t b, FastaPart& P) {
  size_t i = a;
  bool in = false;
  P.seq_off.push_back(0);
  while (i < b) {
    const char* nl = (const char*)memchr(d + i, '\n', b - i);
    const size_t e = nl ? (size_t)(nl - d) : b;
    if (d[i] == '>') {
      if (in) P.seq_off.push_back((int64_t)P.seq.size());
      const size_t j = i + 1;
      size_t k = j;
      while (k < e && d[k] != '\r' && d[k] != ' ' && d[k] != '\t') k++;
      P.hdr_off.push_back((int64_t)j);
      P.hdr_len.push_back((int32_t)(k - j));
      in = true;
    } else if (in) {
      for (size_t k = i; k < e; k++) {
        const char ch = d[k];
        if ((ch >= 'A' && ch <= 'Z') || (ch >= 'a' && ch <= 'z')) P.seq.push_back(ch);
      }
    }
    i = e + 1;
  }
  if (in) P.seq_off.push_back((int64_t)P.seq.size());
}

bool read_fasta(const char* path, Fasta& f) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) return false;
  struct stat sb;
  if (fstat(fd, &sb) != 0) {
    close(fd);
    return false;
  }
  f.size = (size_t)sb.st_size;
  if (f.size > 0) {
    // no MAP_POPULATE: the parse threads fault their own slices in, in parallel (one thread populating 3.5 GB of a
    // config-2 FASTA took 0.14-0.21 s of a 0.34-0.38 s read; without it 0.21 s: tools/read_probe.cpp)
    f.map = mmap(nullptr, f.size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (f.map == MAP_FAILED) {
      f.map = nullptr;
      close(fd);
      return false;
    }
    f.data = (const char*)f.map;
  }
  close(fd);
  const char* d = f.data;
  const size_t N = f.size;
  const int T = N < (1u << 20) ? 1 : io_threads();
  // slice starts: the first record start at or after t*N/T
  std::vector<size_t> cut(T + 1, N);
  cut[0] = 0;
  for (int t = 1; t < T; t++) {
    size_t p = std::max(cut[t - 1], N / T * t);
    while (p < N && !(d[p] == '>' && d[p - 1] == '\n')) {
      const char* q = (const char*)memchr(d + p, '>', N - p);
      if (!q) { p = N; break; }
      p = (size_t)(q - d);
      if (d[p - 1] != '\n') p++;
    }
    cut[t] = p;
  }
  std::vector<FastaPart> parts(T);
  const auto tr0 = std::chrono::steady_clock::now();
  parallel_for(T, [&](int t) { parse_fasta_range(d, cut[t], cut[t + 1], parts[t]); });
  const auto tr1 = std::chrono::steady_clock::now();
  // the slices' arrays laid end to end, each slice copied by its own thread (one thread copying a config-2 FASTA's
  // 2M records and 180 MB of sequence took ~30 ms)
  std::vector<size_t> rb(T + 1, 0), so(T + 1, 0);
  for (int t = 0; t < T; t++) {
    if (parts[t].seq_off.size() != parts[t].hdr_off.size() + 1) return false;
    rb[t + 1] = rb[t] + parts[t].hdr_off.size();
    so[t + 1] = so[t] + parts[t].seq.size();
  }
  const size_t nrec = rb[T];
  f.hdr_off.resize(nrec);
  f.hdr_len.resize(nrec);
  f.seq.resize(so[T]);
  f.seq_off.resize(nrec + 1);
  f.seq_off[0] = 0;
  parallel_for(T, [&](int t) {
    const FastaPart& P = parts[t];
    const size_t n = P.hdr_off.size();
    if (n) {
      memcpy(f.hdr_off.data() + rb[t], P.hdr_off.data(), n * sizeof(int64_t));
      memcpy(f.hdr_len.data() + rb[t], P.hdr_len.data(), n * sizeof(int32_t));
    }
    if (!P.seq.empty()) memcpy(f.seq.data() + so[t], P.seq.data(), P.seq.size());
    for (size_t r = 1; r < P.seq_off.size(); r++) f.seq_off[rb[t] + r] = (int64_t)so[t] + P.seq_off[r];
  });
  if (getenv("UMICLUST_DEBUG")) {
    const auto tr2 = std::chrono::steady_clock::now();
    fprintf(stderr, "umiclust: read_fasta: %d threads, parse %.3f s, merge %.3f s\n", T,
            std::chrono::duration<double>(tr1 - tr0).count(), std::chrono::duration<double>(tr2 - tr1).count());
  }
  return true;
}

void put_wrapped(std::string& out, const char* s, int64_t len, int width) {
  if (width <= 0) {
    out.append(s, (size_t)len);
    out.push_back('\n');
    return;
  }
  if (len == 0) out.push_back('\n');
  for (int64_t i = 0; i < len; i += width) {
    out.append(s + i, (size_t)std::min<int64_t>(width, len - i));
    out.push_back('\n');
  }
}

bool write_all(int fd, const char* p, size_t n) {
  while (n > 0) {
    const ssize_t w = write(fd, p, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

bool write_file(const std::string& path, const std::string& data) {
  const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0666);
  if (fd < 0) return false;
  bool ok = write_all(fd, data.data(), data.size());
  ok = (close(fd) == 0) && ok;
  return ok;
}

// The directory of `path` is RAM-backed (tmpfs / ramfs).  There buffered writes into one file serialise on its inode
// lock (a config-2 fused drop-in streamed its 2.9 GB smolecule_clusters.fa at ~3 GB/s whatever the thread count),
// while stores into a shared mapping of it run in parallel; on the GPU box's disk-backed overlay the mapping was 5x
// slower than pwrite (profiles/r03/e2e_probes.json), so only RAM-backed outputs are mapped.
bool ram_backed(const std::string& path) {
  std::string dir = path;
  const size_t sl = dir.find_last_of('/');
  dir = sl == std::string::npos ? "." : (sl == 0 ? "/" : dir.substr(0, sl));
  struct statfs sf;
  if (statfs(dir.c_str(), &sf) != 0) return false;
  return (unsigned long)sf.f_type == 0x01021994ul /* TMPFS_MAGIC */ || (unsigned long)sf.f_type == 0x858458f6ul /* RAMFS */;
}

// fd's first n bytes mapped for writing (the file already extended to n); nullptr if that fails
char* map_for_write(int fd, size_t n) {
  if (n == 0) return nullptr;
  void* m = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  return m == MAP_FAILED ? nullptr : (char*)m;
}

// a file made of parts written side by side: each part at its offset (pwrite, or stores into a shared mapping on a
// RAM-backed filesystem), on one thread per part
bool write_parts(const std::string& path, const std::vector<std::string>& parts) {
  const int fd = open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0666);
  if (fd < 0) return false;
  const int T = (int)parts.size();
  std::vector<off_t> at(T + 1, 0);
  for (int t = 0; t < T; t++) at[t + 1] = at[t] + (off_t)parts[t].size();
  bool ok = at[T] == 0 || ftruncate(fd, at[T]) == 0;
  std::vector<char> good(T, 1);
  char* map = ok && at[T] > 0 && ram_backed(path) ? map_for_write(fd, (size_t)at[T]) : nullptr;
  if (map) {
    parallel_for(T, [&](int t) {
      if (!parts[t].empty()) memcpy(map + at[t], parts[t].data(), parts[t].size());
    });
    ok = munmap(map, (size_t)at[T]) == 0 && ok;
    ok = (close(fd) == 0) && ok;
    return ok;
  }
  if (ok)
    parallel_for(T, [&](int t) {
      const char* p = parts[t].data();
      size_t n = parts[t].size();
      off_t o = at[t];
      while (n > 0) {
        const ssize_t w = pwrite(fd, p, n, o);
        if (w < 0) {
          if (errno == EINTR) continue;
          good[t] = 0;
          return;
        }
        p += w;
        n -= (size_t)w;
        o += w;
      }
    });
  for (int t = 0; t < T; t++) ok = ok && good[t];
  ok = (close(fd) == 0) && ok;
  return ok;
}

// clusters [0, K) split over T threads by member count
std::vector<int32_t> cluster_slices(const int32_t* ostart, int32_t K, int T) {
  std::vector<int32_t> cut(T + 1, K);
  cut[0] = 0;
  const int64_t tot = ostart[K];
  int32_t k = 0;
  for (int t = 1; t < T; t++) {
    const int64_t want = tot * t / T;
    while (k < K && ostart[k] < want) k++;
    cut[t] = std::max(k, cut[t - 1]);
  }
  return cut;
}


// FASTQ records (pysam.FastxFile): '@' header (name up to whitespace), sequence lines up to the '+' line, then
// as many quality characters as sequence ones
bool read_fastq(const char* path, Fasta& f) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) return false;
  struct stat sb;
  if (fstat(fd, &sb) != 0) {
    close(fd);
    return false;
  }
  f.size = (size_t)sb.st_size;
  if (f.size > 0) {
    // no MAP_POPULATE: the parse threads fault their own slices in, in parallel (one thread populating 3.5 GB of a
    // config-2 FASTA took 0.14-0.21 s of a 0.34-0.38 s read; without it 0.21 s: tools/read_probe.cpp)
    f.map = mmap(nullptr, f.size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (f.map == MAP_FAILED) {
      f.map = nullptr;
      close(fd);
      return false;
    }
    f.data = (const char*)f.map;
  }
  close(fd);
  const char* d = f.data;
  const size_t N = f.size;
  size_t i = 0;
  f.seq_off.push_back(0);
  auto line_end = [&](size_t x) {
    const char* nl = (const char*)memchr(d + x, '\n', N - x);
    return nl ? (size_t)(nl - d) : N;
  };
  while (i < N) {
    if (d[i] == '\n' || d[i] == '\r') { i++; continue; }
    if (d[i] != '@') return false;
    const size_t e = line_end(i);
    size_t k = i + 1;
    while (k < e && d[k] != '\r' && d[k] != ' ' && d[k] != '\t') k++;
    f.hdr_off.push_back((int64_t)(i + 1));
    f.hdr_len.push_back((int32_t)(k - i - 1));
    i = e + 1;
    size_t nseq = 0;
    while (i < N && d[i] != '+') {
      const size_t le = line_end(i);
      for (size_t x = i; x < le; x++)
        if (d[x] != '\r') {
          f.seq.push_back(d[x]);
          nseq++;
        }
      i = le + 1;
    }
    if (i >= N) return false;
    i = line_end(i) + 1;  // the '+' line
    size_t nq = 0;
    while (i < N && nq < nseq) {
      const size_t le = line_end(i);
      for (size_t x = i; x < le; x++) nq += d[x] != '\r';
      i = le + 1;
    }
    f.seq_off.push_back((int64_t)f.seq.size());
  }
  return true;
}

// the reverse_complement of extract_umis.py:10-12: str.translate("ACTG" -> "TGAC"), reversed
void revcomp_ref(const char* s, size_t n, std::string& out) {
  for (size_t x = n; x-- > 0;) {
    const char ch = s[x];
    out.push_back(ch == 'A' ? 'T' : ch == 'C' ? 'G' : ch == 'T' ? 'A' : ch == 'G' ? 'C' : ch);
  }
}

// BGZF (SAM/BAM specification §4.1): gzip members with a BC extra field holding BSIZE; every block is
// inflated independently, so the blocks are split over the host threads
bool inflate_bgzf(const char* path, std::vector<uint8_t>& raw) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) return false;
  struct stat sb;
  if (fstat(fd, &sb) != 0) {
    close(fd);
    return false;
  }
  const size_t N = (size_t)sb.st_size;
  void* map = N ? mmap(nullptr, N, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0) : nullptr;
  close(fd);
  if (N && map == MAP_FAILED) return false;
  const uint8_t* d = (const uint8_t*)map;
  std::vector<size_t> boff, bsz;
  std::vector<uint32_t> isz;
  size_t o = 0;
  bool ok = true;
  while (o + 18 <= N) {
    if (d[o] != 31 || d[o + 1] != 139 || d[o + 2] != 8 || !(d[o + 3] & 4)) { ok = false; break; }
    const size_t xlen = (size_t)d[o + 10] | ((size_t)d[o + 11] << 8);
    size_t bs = 0;
    for (size_t x = o + 12; x + 4 <= o + 12 + xlen;) {
      const size_t sl = (size_t)d[x + 2] | ((size_t)d[x + 3] << 8);
      if (d[x] == 66 && d[x + 1] == 67 && sl == 2) bs = ((size_t)d[x + 4] | ((size_t)d[x + 5] << 8)) + 1;
      x += 4 + sl;
    }
    if (!bs || o + bs > N) { ok = false; break; }
    boff.push_back(o);
    bsz.push_back(bs);
    isz.push_back((uint32_t)d[o + bs - 4] | ((uint32_t)d[o + bs - 3] << 8) | ((uint32_t)d[o + bs - 2] << 16) |
                  ((uint32_t)d[o + bs - 1] << 24));
    o += bs;
  }
  if (ok && o != N) ok = false;
  std::vector<size_t> uo(boff.size() + 1, 0);
  for (size_t b = 0; b < boff.size(); b++) uo[b + 1] = uo[b] + isz[b];
  if (ok) {
    raw.resize(uo.back());
    const int T = std::max(1, std::min<int>(io_threads(), (int)boff.size()));
    std::vector<int> bad(T, 0);
    parallel_for(T, [&](int t) {
      for (size_t b = (size_t)t; b < boff.size(); b += (size_t)T) {
        if (!isz[b]) continue;
        const size_t xlen = (size_t)d[boff[b] + 10] | ((size_t)d[boff[b] + 11] << 8);
        z_stream zs{};
        if (inflateInit2(&zs, -15) != Z_OK) { bad[t] = 1; return; }
        zs.next_in = const_cast<Bytef*>(d + boff[b] + 12 + xlen);
        zs.avail_in = (uInt)(bsz[b] - 12 - xlen - 8);
        zs.next_out = raw.data() + uo[b];
        zs.avail_out = isz[b];
        const int rc = inflate(&zs, Z_FINISH);
        inflateEnd(&zs);
        if (rc != Z_STREAM_END || zs.avail_out != 0) { bad[t] = 1; return; }
      }
    });
    for (int v : bad) ok = ok && !v;
  }
  if (map) munmap(map, N);
  return ok;
}


// ---------------------------------------------------------------- the reference's string helpers
bool Sv::operator==(const char* s) const { return n == strlen(s) && !memcmp(p, s, n); }

std::string pjoin(const std::string& a, const std::string& b) {
  if (a.empty()) return b;
  return a.back() == '/' ? a + b : a + "/" + b;
}

// Python `s.split(sep)[1]`: the text between the first and the second occurrence of sep
bool split1(Sv s, const char* sep, Sv& out) {
  const size_t m = strlen(sep);
  const char* e = s.p + s.n;
  if (m == 0) return false;
  // memchr for the separator's first character, then compare (vectorised; a read of ~1.5 kb never holds the 's' of
  // "seq=", so the second search is one memchr pass over it)
  auto find = [&](const char* from) -> const char* {
    while (from + m <= e) {
      const char* q = (const char*)memchr(from, sep[0], (size_t)(e - from) - (m - 1));
      if (!q) return nullptr;
      if (!memcmp(q, sep, m)) return q;
      from = q + 1;
    }
    return nullptr;
  };
  const char* a = find(s.p);
  if (!a) return false;
  a += m;
  const char* b = find(a);
  out = Sv{a, (size_t)((b ? b : e) - a)};
  return true;
}

static void split_fields(Sv name, std::vector<Sv>& f) {  // name.split(";")
  f.clear();
  const char* p = name.p;
  const char* const e = name.p + name.n;
  for (;;) {  // memchr: the headers are ~1.6 KB, nearly all of it the last field's read
    const char* q = (const char*)memchr(p, ';', (size_t)(e - p));
    if (!q) {
      f.push_back(Sv{p, (size_t)(e - p)});
      return;
    }
    f.push_back(Sv{p, (size_t)(q - p)});
    p = q + 1;
  }
}

// ---------------------------------------------------------------- vsearch writers (--consout, --clusters)
void write_text(const char* path, const std::string& text) {
  if (!write_file(path, text)) throw IoError{UMICLUST_EIO, std::string("cannot write ") + path};
}

void write_consout(const char* path, const Fasta& f, const ClusterView& cv, const char* cons, const int64_t* cons_off,
                   bool clusterout_id, int width) {
  const int32_t K = cv.K;
  const int T = K < 256 ? 1 : io_threads();
  const std::vector<int32_t> cut = cluster_slices(cv.ostart, K, T);
  std::vector<std::string> part(T);
  parallel_for(T, [&](int t) {
    std::string& out = part[t];
    out.reserve((size_t)(cut[t + 1] - cut[t]) * 256);
    for (int32_t k = cut[t]; k < cut[t + 1]; k++) {
      const int32_t ci = cv.perm[cv.omemb[cv.ostart[k]]];
      out += ">centroid=";
      out.append(f.data + f.hdr_off[ci], (size_t)f.hdr_len[ci]);
      out += ";seqs=" + std::to_string(cv.ostart[k + 1] - cv.ostart[k]);
      if (clusterout_id) out += ";clusterid=" + std::to_string(k);
      out.push_back('\n');
      put_wrapped(out, cons + cons_off[k], cons_off[k + 1] - cons_off[k], width);
    }
  });
  if (!write_parts(path, part)) throw IoError{UMICLUST_EIO, std::string("cannot write ") + path};
}

// writev of every segment (IOV_MAX at a time, partial writes resumed)
static bool writev_all(int fd, std::vector<iovec>& iov) {
  size_t at = 0;
  while (at < iov.size()) {
    const int n = (int)std::min<size_t>(iov.size() - at, 1024);
    const ssize_t w = writev(fd, iov.data() + at, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    size_t left = (size_t)w;
    while (at < iov.size() && left >= iov[at].iov_len) left -= iov[at++].iov_len;
    if (left) {
      iov[at].iov_base = (char*)iov[at].iov_base + left;
      iov[at].iov_len -= left;
    }
  }
  return true;
}

void write_cluster_files(const char* prefix, const Fasta& f, const ClusterView& cv, const char* masked, int stride,
                         const uint8_t* hlen, int width, const int32_t* mrow) {
  const int32_t K = cv.K;
  const int T = K < 256 ? 1 : io_threads();
  const std::vector<int32_t> cut = cluster_slices(cv.ostart, K, T);
  std::vector<int32_t> bad(T, -1);
  parallel_for(T, [&](int t) {
    // A member whose input record is byte for byte what it prints (">label\n" + its sequence on one line, unmasked,
    // within the line width) is written straight from the input mapping; the others are formatted into `out`.
    // Segments: (pointer, length) with pointer null = an offset into `out` (resolved once it stops growing).
    std::string fn, out;
    std::vector<std::pair<const char*, size_t>> seg;
    std::vector<iovec> iov;
    for (int32_t k = cut[t]; k < cut[t + 1]; k++) {
      out.clear();
      seg.clear();
      for (int32_t x = cv.ostart[k]; x < cv.ostart[k + 1]; x++) {
        const int32_t s = cv.omemb[x];
        const int32_t i = cv.perm[s];
        const int64_t row = !masked ? -1 : mrow ? mrow[s] : s;
        const int64_t L = f.seq_off[i + 1] - f.seq_off[i];
        const char* h = f.data + f.hdr_off[i];
        const size_t hl = (size_t)f.hdr_len[i];
        if (row < 0 && (width <= 0 || L <= width) && f.hdr_off[i] > 0 && h[-1] == '>' &&
            (size_t)f.hdr_off[i] + hl + 2 + (size_t)L <= f.size && h[hl] == '\n' && h[hl + 1 + L] == '\n' &&
            memcmp(h + hl + 1, f.seq.data() + f.seq_off[i], (size_t)L) == 0) {
          seg.push_back({h - 1, hl + (size_t)L + 3});
          continue;
        }
        const size_t o0 = out.size();
        out.push_back('>');
        out.append(h, hl);
        out.push_back('\n');
        if (row >= 0) put_wrapped(out, masked + (size_t)row * stride, hlen[s], width);
        else put_wrapped(out, f.seq.data() + f.seq_off[i], L, width);
        seg.push_back({nullptr, o0});
      }
      iov.clear();
      for (size_t j = 0; j < seg.size(); j++) {
        if (seg[j].first) {
          iov.push_back({(void*)seg[j].first, seg[j].second});
        } else {  // this formatted record runs to the next formatted one's start (or out's end)
          size_t e = out.size();
          for (size_t u = j + 1; u < seg.size(); u++)
            if (!seg[u].first) {
              e = seg[u].second;
              break;
            }
          iov.push_back({(void*)(out.data() + seg[j].second), e - seg[j].second});
        }
      }
      fn = prefix;
      fn += std::to_string(k);
      const int fd = open(fn.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0666);
      bool ok = fd >= 0;
      if (ok) {
        ok = writev_all(fd, iov);
        ok = close(fd) == 0 && ok;
      }
      if (!ok) {
        bad[t] = k;
        return;
      }
    }
  });
  for (int t = 0; t < T; t++)
    if (bad[t] >= 0) throw IoError{UMICLUST_EIO, std::string("cannot write ") + prefix + std::to_string(bad[t])};
}

// ---------------------------------------------------------------- in-process parse (§8f f2)
// parse_umi_clusters over the in-memory clusters (parse_umi_clusters.py:10-242).  Clusters are independent
// except for the loop's early exit (`max_clusters`) and its first error, so the work runs in three phases:
// every cluster's counts, caps and first error on io_threads() threads; in cluster order, the exit and the
// first error; then the cluster files and the per-cluster text of the kept range on the threads, concatenated
// in order.  On an error the outputs are what the reference leaves behind when it raises: the files and the
// stats / smolecule lines of the clusters before the failing one (its `with` blocks flush them), plus the
// records a missing `seq=` field interrupts in the middle of a cluster (:104-116), and no log.
void precompute_fields(const Fasta& f, std::vector<RecFields>& out, int threads) {
  const int64_t n = (int64_t)f.hdr_off.size();
  out.assign((size_t)n, RecFields{});
  const int T = std::max(1, std::min<int>(threads, (int)(n / 4096 + 1)));
  parallel_for(T, [&](int t) {
    std::vector<Sv> fields;
    for (int64_t i = n * t / T; i < n * (t + 1) / T; i++) {
      const char* h = f.data + f.hdr_off[i];
      split_fields(Sv{h, (size_t)f.hdr_len[i]}, fields);
      if (fields.size() != 7) continue;
      Sv strand;
      if (!split1(fields[1], "strand=", strand)) continue;
      RecFields& r = out[(size_t)i];
      if (strand == "+") r.strand = 0;
      else if (strand == "-") r.strand = 1;
      else continue;
      r.id_n = (uint32_t)fields[0].n;
      r.last_off = (uint32_t)(fields[6].p - h);
      r.last_n = (uint32_t)fields[6].n;
      Sv read;
      if (split1(fields[6], "seq=", read)) {
        r.read_off = (int32_t)(read.p - h);
        r.read_n = (uint32_t)read.n;
      }
      r.ok = 1;
    }
  });
}

void parse_clusters(const Fasta& f, const ClusterView& cv, const umiclust_parse_params* pp, const char* work_dir_c,
                    umiclust_parse_result* pr, const RecFields* pre, std::vector<std::pair<void*, size_t>>* unmap) {
  const int64_t min_reads = pp->min_reads_per_cluster, max_reads = pp->max_reads_per_cluster;
  const std::string work_dir = work_dir_c ? work_dir_c : "";
  const std::string fa_dir = pjoin(work_dir, "clusters_fa");  // :167
  struct stat sb;
  if (stat(fa_dir.c_str(), &sb) == 0)
    throw IoError{UMICLUST_EEXIST, fa_dir + " should not exist yet but does exist!"};  // :174-177
  if (mkdir(fa_dir.c_str(), 0777) != 0) throw IoError{UMICLUST_EIO, "cannot create " + fa_dir};
  const int32_t K = cv.K;
  struct PClus {
    int64_t n_fwd = 0, n_rev = 0, found = 0, max_fwd = 0, max_rev = 0, w_fwd = 0, w_rev = 0, w_all = 0;
    int written = 0, err = 0;
    int64_t noseq_at = -1;  // the first entry to write without a seq= field (an IndexError mid-cluster)
    int64_t smol_bytes = 0; // this cluster's smolecule_clusters.fa records (">{k}\n{read}\n" per entry written)
    std::string msg;
  };
  struct Scratch {
    std::vector<Sv> fields;
    struct Kept {
      Sv id, last;  // cols[0] and cols[6] of the record's header
      int32_t rec;
    };
    std::vector<Kept> kept[2];  // insertion-ordered dict read id -> record (:61-65)
  };
  // an entry written: its read id (`cols[0]`) and read (`cols[6].split("seq=")[1]`), kept from the analysis so the
  // write phase never splits a header again
  struct Ent {
    const char* rid;
    const char* read;
    uint32_t rid_n, read_n;
  };
  auto entry = [&](const PClus& r, const Scratch& sc, int64_t y) -> const Scratch::Kept& {
    return y < r.w_fwd ? sc.kept[0][y] : sc.kept[1][y - r.w_fwd];
  };
  // one cluster's counts (and the entries it writes, appended to ents); false on the first error
  auto analyze = [&](int32_t k, PClus& r, Scratch& sc, std::vector<Ent>& ents) -> bool {
    sc.kept[0].clear();
    sc.kept[1].clear();
    int64_t seen[2] = {0, 0};
    for (int32_t x = cv.ostart[k]; x < cv.ostart[k + 1]; x++) {  // cluster<N> file order (:36)
      const int32_t i = cv.perm[cv.omemb[x]];
      const Sv name{f.data + f.hdr_off[i], (size_t)f.hdr_len[i]};
      Sv id, last;
      int st = 0;
      if (pre && pre[i].ok) {  // fields computed ahead (precompute_fields)
        id = Sv{name.p, pre[i].id_n};
        last = Sv{name.p + pre[i].last_off, pre[i].last_n};
        st = pre[i].strand;
      } else {
        split_fields(name, sc.fields);
        if (sc.fields.size() != 7) {  // :38-47
          r.err = UMICLUST_EFORMAT;
          r.msg = "cluster " + std::to_string(k) + ": header has " + std::to_string(sc.fields.size()) +
                  " cols while it should contain 7: " + name.str();
          return false;
        }
        Sv strand;
        if (!split1(sc.fields[1], "strand=", strand)) {
          r.err = UMICLUST_EFORMAT;
          r.msg = "no strand= field: " + name.str();
          return false;
        }
        if (strand == "+") st = 0;
        else if (strand == "-") st = 1;
        else {
          r.found++;
          r.err = UMICLUST_EFORMAT;
          r.msg = "Strand annotation is " + strand.str() + " but only - or + are allowed!";
          return false;
        }
        id = sc.fields[0];
        last = sc.fields[6];
      }
      r.found++;
      if (seen[st] < max_reads) {  // kept[strand][id] = rec: a repeated id keeps its first position
        std::vector<Scratch::Kept>& kv = sc.kept[st];
        size_t pos = kv.size();
        for (size_t y = 0; y < kv.size(); y++)
          if (kv[y].id.n == id.n && !memcmp(kv[y].id.p, id.p, id.n)) {
            pos = y;
            break;
          }
        if (pos == kv.size()) {
          kv.push_back(Scratch::Kept{id, last, i});
        } else {
          kv[pos].last = last;  // a repeated id: the later record (its id is the same)
          kv[pos].rec = i;
        }
      }
      seen[st]++;
    }
    // strand caps (:66-87)
    r.n_fwd = seen[0];
    r.n_rev = seen[1];
    int64_t min_fwd, min_rev;
    if (pp->balance_strands) {
      min_fwd = min_rev = min_reads / 2;
      const int64_t capped = std::min(std::min(r.n_fwd * 2, r.n_rev * 2), max_reads);
      r.max_fwd = r.max_rev = capped / 2;
    } else if (r.n_fwd > r.n_rev) {
      min_fwd = min_rev = 0;
      r.max_rev = std::min(r.n_rev, max_reads / 2);
      r.max_fwd = std::min(max_reads - r.max_rev, r.n_fwd);
    } else {
      min_fwd = min_rev = 0;
      r.max_fwd = std::min(r.n_fwd, max_reads / 2);
      r.max_rev = std::min(max_reads - r.max_fwd, r.n_rev);
    }
    const int64_t n_reads = r.max_fwd + r.max_rev;
    if (n_reads > max_reads) {  // :89-92
      r.err = UMICLUST_EINVAL;
      r.msg = "n_reads is higher than max_reads_per_cluster";
      return false;
    }
    if (r.n_fwd >= min_fwd && r.n_rev >= min_rev && n_reads >= min_reads) {  // :95-120
      r.w_fwd = std::min<int64_t>((int64_t)sc.kept[0].size(), r.max_fwd);
      r.w_rev = std::min<int64_t>((int64_t)sc.kept[1].size(), r.max_rev);
      r.w_all = std::min<int64_t>(r.w_fwd + r.w_rev, max_reads);
      r.written = 1;
      const int64_t head = 3 + (int64_t)std::to_string(k).size();  // '>' k '\n' ... '\n'
      for (int64_t y = 0; y < r.w_all; y++) {  // `cols[6].split("seq=")[1]` of every entry written (:106)
        const Scratch::Kept& ke = entry(r, sc, y);
        const int32_t i = ke.rec;
        Sv read;
        bool has_read;
        if (pre && pre[i].ok) {
          has_read = pre[i].read_off >= 0;
          read = Sv{f.data + f.hdr_off[i] + (has_read ? pre[i].read_off : 0), pre[i].read_n};
        } else {
          has_read = split1(ke.last, "seq=", read);
        }
        if (!has_read) {
          r.err = UMICLUST_EFORMAT;
          r.noseq_at = y;  // the entries before it are written (and kept in ents)
          r.msg = "IndexError: no seq= field in " + Sv{f.data + f.hdr_off[i], (size_t)f.hdr_len[i]}.str();
          return false;
        }
        ents.push_back(Ent{ke.id.p, read.p, (uint32_t)ke.id.n, (uint32_t)read.n});
        r.smol_bytes += head + (int64_t)read.n;
      }
    }
    return true;
  };
  static const bool debug = getenv("UMICLUST_DEBUG") != nullptr;
  auto clk = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double tp0 = clk();
  const int T = K < 256 ? 1 : io_threads();
  const std::vector<int32_t> cut = cluster_slices(cv.ostart, K, T);
  std::vector<PClus> res((size_t)K);
  std::vector<std::vector<Ent>> ents_t((size_t)T);
  std::vector<int64_t> ent_beg((size_t)K + 1, 0);  // cluster k's entries: ents_t[thread of k][ent_beg[k] ..)
  std::vector<int32_t> ent_thr((size_t)K, 0);
  parallel_for(T, [&](int t) {
    Scratch sc;
    std::vector<Ent>& ents = ents_t[(size_t)t];
    for (int32_t k = cut[t]; k < cut[t + 1]; k++) {
      ent_beg[k] = (int64_t)ents.size();
      ent_thr[k] = t;
      analyze(k, res[k], sc, ents);
    }
  });
  const double tp1 = clk();
  // the reference's loop in order: its first error, its early exit
  int64_t n_written = 0, reads_found = 0, reads_written = 0;
  int32_t kend = K, kerr = -1;
  for (int32_t k = 0; k < K; k++) {
    if (res[k].err) {
      kerr = k;
      kend = k;
      break;
    }
    n_written += res[k].written;
    // the reference's quirk (:206, :219-221): the totals are overwritten by this cluster's counts, then doubled
    reads_found = 2 * res[k].found;
    reads_written = 2 * res[k].w_all;
    // `if max_clusters and n_written > max_clusters` (:222-223): any non-zero value applies, as in Python
    if (pp->max_clusters != 0 && n_written > pp->max_clusters) {
      kend = k + 1;
      break;
    }
  }
  // a missing seq= field interrupts cluster kerr after its first noseq_at entries: written like the others (its
  // smol_bytes and entries stop before the failing one)
  const bool partial = kerr >= 0 && res[kerr].noseq_at >= 0;
  const int32_t kwrite = partial ? kerr + 1 : kend;
  // smolecule_clusters.fa: every read written once more (GBs at production depth).  Its records are laid out
  // by cluster in advance (offsets from the counts above); each writing thread streams its clusters' records to
  // their offsets in chunks of kSmolChunk bytes while it creates its cluster files, so the one file's writes (which
  // serialise on its inode) overlap the other threads' file creation.  (A shared mapping of the file was measured
  // 5x slower than pwrite on the GPU box's filesystem: 2.2 vs 10.4 GB/s, profiles/r03/e2e_probes.json.)
  constexpr size_t kSmolChunk = 8u << 20;
  std::vector<int64_t> smol_off((size_t)kwrite + 1, 0);
  for (int32_t k = 0; k < kwrite; k++) smol_off[k + 1] = smol_off[k] + res[k].smol_bytes;
  const std::string smol_path = pjoin(work_dir, "smolecule_clusters.fa");
  const int smol_fd = open(smol_path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0666);
  if (smol_fd < 0) throw IoError{UMICLUST_EIO, "cannot write smolecule_clusters.fa"};
  // RAM-backed work_dir: the records go straight into a shared mapping of the file (no inode lock; see ram_backed)
  const size_t smol_total = (size_t)smol_off[kwrite];
  char* smol_map = nullptr;
  if (smol_total > 0 && ram_backed(smol_path) && ftruncate(smol_fd, (off_t)smol_total) == 0)
    smol_map = map_for_write(smol_fd, smol_total);
  // cluster files and the text of clusters [0, kwrite), on the threads
  const std::vector<int32_t> wcut = cluster_slices(cv.ostart, kwrite, T);
  std::vector<std::string> log_p(T), stats_p(T);
  std::vector<size_t> stats_beg((size_t)kwrite + 1, 0);  // a cluster's line starts here in its thread's part
  std::vector<int32_t> bad(T, -1);
  std::vector<uint8_t> wrote((size_t)kwrite, 0), smol_bad(T, 0);
  parallel_for(T, [&](int t) {
    std::string smol, &log = log_p[t], &stats_out = stats_p[t];
    std::vector<iovec> iov;
    smol.reserve(kSmolChunk + (1u << 16));
    // this thread's records, contiguous in the file from its first cluster's offset (also on an early return:
    // the clusters before a failing one keep their records, as the reference's buffered file does)
    struct Flush {
      std::string& s;
      int fd;
      off_t at;
      uint8_t& bad;
      char* map;
      void run() {
        if (map) {
          memcpy(map + at, s.data(), s.size());
          at += (off_t)s.size();
          s.clear();
          return;
        }
        size_t o = 0;
        while (o < s.size()) {
          const ssize_t w = pwrite(fd, s.data() + o, s.size() - o, at + (off_t)o);
          if (w < 0) {
            if (errno == EINTR) continue;
            bad = 1;
            break;
          }
          o += (size_t)w;
        }
        at += (off_t)s.size();
        s.clear();
      }
      ~Flush() { run(); }
    } flush{smol, smol_fd, (off_t)smol_off[wcut[t]], smol_bad[t], smol_map};
    std::string fname;
    for (int32_t k = wcut[t]; k < wcut[t + 1]; k++) {
      stats_beg[k] = stats_out.size();
      const PClus& r = res[k];
      const int64_t nw = (partial && k == kerr) ? r.noseq_at : r.w_all;
      const std::string kstr = std::to_string(k);
      fname = "cluster" + kstr + ".fasta";
      const std::string out_fasta = pjoin(fa_dir, fname);  // :34
      log += "Cluster: " + out_fasta + " has " + std::to_string(r.n_fwd) + "/" + std::to_string(r.max_fwd) +
             " fwd and " + std::to_string(r.n_rev) + "/" + std::to_string(r.max_rev) + " rev reads\n";
      if (r.written) {
        // the cluster file's records are gathered from the input mapping (writev: no formatting copy of the reads);
        // the smolecule records go straight into the file's mapping when there is one
        static const char kGt = '>', kNl = '\n';
        iov.clear();
        const Ent* e = ents_t[(size_t)ent_thr[k]].data() + ent_beg[k];
        for (int64_t y = 0; y < nw; y++) {
          iov.push_back({(void*)&kGt, 1});
          iov.push_back({(void*)e[y].rid, e[y].rid_n});
          iov.push_back({(void*)&kNl, 1});
          iov.push_back({(void*)e[y].read, e[y].read_n});
          iov.push_back({(void*)&kNl, 1});
          if (smol_map) {
            char* d = smol_map + flush.at;
            *d++ = '>';
            memcpy(d, kstr.data(), kstr.size());
            d += kstr.size();
            *d++ = '\n';
            memcpy(d, e[y].read, e[y].read_n);
            d += e[y].read_n;
            *d++ = '\n';
            flush.at = (off_t)(d - smol_map);
          } else {
            smol.push_back('>');
            smol += kstr;
            smol.push_back('\n');
            smol.append(e[y].read, e[y].read_n);
            smol.push_back('\n');
          }
        }
        const int fd = open(out_fasta.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0666);
        bool ok = fd >= 0;
        if (ok) {
          ok = writev_all(fd, iov);
          ok = close(fd) == 0 && ok;
        }
        if (!ok) {
          if (bad[t] < 0) bad[t] = k;
          return;
        }
        wrote[k] = 1;
        if (smol.size() >= kSmolChunk) flush.run();
      } else {
        log += "Cluster " + kstr + " skipped\n";
      }
      if (partial && k == kerr) break;  // the exception: no log or stats line for it
      log += "Cluster: " + out_fasta + " has " + std::to_string(r.w_all) + " reads written: " + std::to_string(r.w_fwd) +
             " fwd - " + std::to_string(r.w_rev) + " rev\n";
      stats_out += "cluster" + kstr + "\t" + std::to_string(r.n_fwd) + "\t" + std::to_string(r.n_rev) +
                   "\t" + std::to_string(r.w_fwd) + "\t" + std::to_string(r.w_rev) + "\t" + std::to_string(r.found) +
                   "\t" + std::to_string(r.w_all) + "\t" + std::to_string(r.written) + "\n";
    }
  });
  const double tp2 = clk();
  // an unwritable cluster file: the reference stops there (OSError) -- files the other threads wrote past it go,
  // and the stats and smolecule records end before it, as the reference's `with` blocks leave them
  int32_t kbad = -1;
  for (int t = 0; t < T; t++)
    if (bad[t] >= 0 && (kbad < 0 || bad[t] < kbad)) kbad = bad[t];
  const int32_t kkeep = kbad >= 0 ? kbad : kwrite;
  if (kbad >= 0)
    for (int32_t k = kbad + 1; k < kwrite; k++)
      if (wrote[k]) unlink(pjoin(fa_dir, "cluster" + std::to_string(k) + ".fasta").c_str());
  bool smol_ok = true;
  if (smol_map && unmap) unmap->push_back({smol_map, smol_total});
  else if (smol_map) smol_ok = munmap(smol_map, smol_total) == 0;
  for (int t = 0; t < T; t++) smol_ok = smol_ok && !smol_bad[t];
  if (kbad >= 0) smol_ok = ftruncate(smol_fd, (off_t)smol_off[kkeep]) == 0 && smol_ok;
  smol_ok = close(smol_fd) == 0 && smol_ok;
  std::string stats_out = "id_cluster\tn_fwd\tn_rev\twritten_fwd\twritten_rev\tn\twritten\tcluster_written\n", log;
  for (int t = 0; t < T; t++) {
    if (wcut[t] >= kkeep) break;
    stats_out.append(stats_p[t], 0, kkeep < wcut[t + 1] ? stats_beg[kkeep] : stats_p[t].size());
    log += log_p[t];
  }
  if (!write_file(pjoin(work_dir, "vsearch_cluster_stats.tsv"), stats_out))
    throw IoError{UMICLUST_EIO, "cannot write the stats table"};
  if (!smol_ok) throw IoError{UMICLUST_EIO, "cannot write smolecule_clusters.fa"};
  if (kbad >= 0)
    throw IoError{UMICLUST_EIO, "cannot write " + pjoin(fa_dir, "cluster" + std::to_string(kbad) + ".fasta")};
  if (kerr >= 0) throw IoError{res[kerr].err, res[kerr].msg};
  pr->n_clusters = K;
  pr->n_written = n_written;
  pr->reads_found = reads_found;
  pr->reads_written = reads_written;
  pr->empty_region = (n_written == 0 || reads_found == 0) ? 1 : 0;
  pr->pad = 0;
  if (pr->empty_region) return;  // :224-231 (the caller appends the region: it may need the JSON map)
  log += "Clusters: " + std::to_string((int64_t)(n_written * 100.0 / K)) + "% written (" + std::to_string(n_written) +
         ")\n";
  log += "Reads: " + std::to_string(reads_found) + " found\n";
  log += "Reads: " + std::to_string((int64_t)(reads_written * 100.0 / reads_found)) + "% in written clusters\n";
  if (!write_file(pjoin(work_dir, "parse_cluster.log"), log)) throw IoError{UMICLUST_EIO, "cannot write parse_cluster.log"};
  if (debug)
    fprintf(stderr, "umiclust: parse: analysis %.3f s, files + smolecule %.3f s, close + stats + log %.3f s (%d threads)\n",
            tp1 - tp0, tp2 - tp1, clk() - tp2, T);
}

// ---------------------------------------------------------------- detected-UMI FASTA (§8f f1)
int64_t write_detected_umis(const char* path, const Fasta& f, const int32_t* res, int64_t ngood, int32_t a3) {
  std::vector<std::string> strand(ngood), rid(ngood);
  for (int64_t i = 0; i < ngood; i++) {
    const Sv name{f.data + f.hdr_off[i], (size_t)f.hdr_len[i]};
    Sv st;
    split1(name, "strand=", st);
    strand[i] = st.str();
    const char* semi = (const char*)memchr(name.p, ';', name.n);
    rid[i] = std::string(name.p, semi ? (size_t)(semi - name.p) : name.n);  // get_read_name (:129-130)
  }
  const int T = ngood < 4096 ? 1 : io_threads();
  std::vector<std::string> part(T);
  std::vector<int64_t> cnt(T, 0);
  parallel_for(T, [&](int t) {
    std::string& o = part[t];
    for (int64_t i = ngood * t / T; i < ngood * (t + 1) / T; i++) {
      const int32_t* r = res + i * 6;
      if (r[0] < 0 || r[3] < 0) continue;  // `if not umi_5p or not umi_3p`
      const char* s = f.seq.data() + f.seq_off[i];
      const int64_t len = f.seq_off[i + 1] - f.seq_off[i];
      const int64_t w3 = (a3 == 0 || a3 > len) ? len : a3;
      const char* u5 = s + r[1];
      const size_t l5 = (size_t)(r[2] - r[1] + 1);
      const char* u3 = s + (len - w3) + r[4];
      const size_t l3 = (size_t)(r[5] - r[4] + 1);
      cnt[t]++;
      o += ">" + rid[i] + ";strand=" + strand[i] + ";umi_fwd_dist=" + std::to_string(r[0]) + ";umi_rev_dist=" +
           std::to_string(r[3]) + ";umi_fwd_seq=";
      o.append(u5, l5);
      o += ";umi_rev_seq=";
      o.append(u3, l3);
      o += ";seq=";
      o.append(s, (size_t)len);
      o.push_back('\n');
      if (strand[i] == "+") {
        o.append(u5, l5);
        o.append(u3, l3);
      } else {
        revcomp_ref(u3, l3, o);
        revcomp_ref(u5, l5, o);
      }
      o.push_back('\n');
    }
  });
  if (!write_parts(path, part)) throw IoError{UMICLUST_EIO, std::string("cannot write ") + path};
  int64_t tot = 0;
  for (int64_t v : cnt) tot += v;
  return tot;
}

// ---------------------------------------------------------------- vsearch argv grammar
// vsearch --gapopen/--gapext strings: "/"-separated tokens "<int>[QT][ILRE]*"
// (no letter = all positions; E = both ends; Q/T restrict to query/target gaps).
bool parse_gap(const char* s, int32_t* dst) {
  const char* p = s;
  while (*p) {
    char* e = nullptr;
    long v = strtol(p, &e, 10);
    if (e == p) return false;
    p = e;
    bool q = false, t = false, I = false, L = false, R = false;
    while (*p && *p != '/') {
      switch (*p) {
        case 'Q': q = true; break;
        case 'T': t = true; break;
        case 'I': I = true; break;
        case 'E': L = R = true; break;
        case 'L': L = true; break;
        case 'R': R = true; break;
        default: return false;
      }
      p++;
    }
    if (!q && !t) q = t = true;
    if (!I && !L && !R) I = L = R = true;
    if (q) {
      if (L) dst[UMICLUST_QL] = (int32_t)v;
      if (I) dst[UMICLUST_QI] = (int32_t)v;
      if (R) dst[UMICLUST_QR] = (int32_t)v;
    }
    if (t) {
      if (L) dst[UMICLUST_TL] = (int32_t)v;
      if (I) dst[UMICLUST_TI] = (int32_t)v;
      if (R) dst[UMICLUST_TR] = (int32_t)v;
    }
    if (*p == '/') p++;
  }
  return true;
}


}  // namespace io
}  // namespace uc

// ====================================================================== C ABI: parameters
using uc::io::parse_gap;

extern "C" {

int32_t umiclust_params_init(umiclust_params* p, int32_t preset, double identity, int32_t minlen,
                             int32_t maxlen) {
  if (!p) return UMICLUST_EINVAL;
  memset(p, 0, sizeof(*p));
  p->id = identity;
  p->weak_id = identity < 0.10 ? identity : 0.10;
  p->minseqlength = minlen;
  p->maxseqlength = maxlen;
  p->wordlength = 8;
  p->minwordmatches = 12;
  p->maxaccepts = 1;
  p->maxrejects = 32;
  p->strand_both = 1;
  p->qmask_dust = 1;
  p->clusterout_sort = 1;
  p->clusterout_id = 1;
  p->fasta_width = 80;
  p->policy_boundary_open = 1;
  p->threads = 1;
  p->policy_threads = 0;
  for (int k = 0; k < 6; k++) p->gap_ext[k] = (k == UMICLUST_QI || k == UMICLUST_TI) ? 2 : 1;
  if (preset == UMICLUST_PRESET_ROUND1) {
    p->match = 10;
    p->mismatch = -40;
    for (int k = 0; k < 6; k++) p->gap_open[k] = (k == UMICLUST_QI || k == UMICLUST_TI) ? 40 : 0;
  } else if (preset == UMICLUST_PRESET_VSEARCH_DEFAULT) {
    p->match = 2;
    p->mismatch = -4;
    for (int k = 0; k < 6; k++) p->gap_open[k] = (k == UMICLUST_QI || k == UMICLUST_TI) ? 20 : 2;
  } else {
    return UMICLUST_EINVAL;
  }
  return UMICLUST_OK;
}

int32_t umiclust_params_from_argv(umiclust_params* p, int32_t argc, const char* const* argv,
                                  char* in_fasta, char* clusters_prefix, char* consout,
                                  char* log_path, int32_t pathcap) {
  if (!p || argc < 0 || (argc > 0 && !argv)) return UMICLUST_EINVAL;
  umiclust_params_init(p, UMICLUST_PRESET_VSEARCH_DEFAULT, 0.97, 32, 50000);
  p->clusterout_sort = 0;
  p->clusterout_id = 0;
  p->strand_both = 0;
  p->maxseqlength = 50000;
  bool have_in = false;
  auto put = [&](char* dst, const char* v) -> bool {
    if (!dst) return true;
    if ((int32_t)strlen(v) + 1 > pathcap) return false;
    strcpy(dst, v);
    return true;
  };
  if (in_fasta) in_fasta[0] = 0;
  if (clusters_prefix) clusters_prefix[0] = 0;
  if (consout) consout[0] = 0;
  if (log_path) log_path[0] = 0;
  int i = 0;
  if (argc > 0 && argv[0] && argv[0][0] != '-') i = 1;  // program name
  for (; i < argc; i++) {
    const char* a = argv[i];
    auto val = [&]() -> const char* { return (i + 1 < argc) ? argv[++i] : nullptr; };
    if (!strcmp(a, "--clusterout_id")) p->clusterout_id = 1;
    else if (!strcmp(a, "--clusterout_sort")) p->clusterout_sort = 1;
    else if (!strcmp(a, "--quiet") || !strcmp(a, "--no_progress")) {}
    else if (!strcmp(a, "--clusters")) { const char* v = val(); if (!v || !put(clusters_prefix, v)) return UMICLUST_EINVAL; }
    else if (!strcmp(a, "--consout")) { const char* v = val(); if (!v || !put(consout, v)) return UMICLUST_EINVAL; }
    else if (!strcmp(a, "--log")) { const char* v = val(); if (!v || !put(log_path, v)) return UMICLUST_EINVAL; }
    else if (!strcmp(a, "--cluster_fast")) { const char* v = val(); if (!v || !put(in_fasta, v)) return UMICLUST_EINVAL; have_in = true; }
    else if (!strcmp(a, "--minseqlength")) { const char* v = val(); if (!v) return UMICLUST_EINVAL; p->minseqlength = atoi(v); }
    else if (!strcmp(a, "--maxseqlength")) { const char* v = val(); if (!v) return UMICLUST_EINVAL; p->maxseqlength = atoi(v); }
    else if (!strcmp(a, "--threads")) {
      const char* v = val();
      if (!v) return UMICLUST_EINVAL;
      p->threads = std::max(1, atoi(v));
    }
    else if (!strcmp(a, "--strand")) {
      const char* v = val();
      if (!v) return UMICLUST_EINVAL;
      if (!strcmp(v, "both")) p->strand_both = 1;
      else if (!strcmp(v, "plus")) p->strand_both = 0;
      else return UMICLUST_EINVAL;
    }
    else if (!strcmp(a, "--gapopen")) { const char* v = val(); if (!v || !parse_gap(v, p->gap_open)) return UMICLUST_EINVAL; }
    else if (!strcmp(a, "--gapext")) { const char* v = val(); if (!v || !parse_gap(v, p->gap_ext)) return UMICLUST_EINVAL; }
    else if (!strcmp(a, "--match")) { const char* v = val(); if (!v) return UMICLUST_EINVAL; p->match = atoi(v); }
    else if (!strcmp(a, "--mismatch")) { const char* v = val(); if (!v) return UMICLUST_EINVAL; p->mismatch = atoi(v); }
    else if (!strcmp(a, "--id")) {
      const char* v = val();
      if (!v) return UMICLUST_EINVAL;
      p->id = atof(v);
      p->weak_id = p->id < 0.10 ? p->id : 0.10;
    }
    else if (!strcmp(a, "--qmask")) {
      const char* v = val();
      if (!v) return UMICLUST_EINVAL;
      if (!strcmp(v, "dust")) p->qmask_dust = 1;
      else if (!strcmp(v, "none")) p->qmask_dust = 0;
      else return UMICLUST_EINVAL;
    }
    else if (!strcmp(a, "--wordlength")) { const char* v = val(); if (!v) return UMICLUST_EINVAL; p->wordlength = atoi(v); }
    else if (!strcmp(a, "--minwordmatches")) { const char* v = val(); if (!v) return UMICLUST_EINVAL; p->minwordmatches = atoi(v); }
    else if (!strcmp(a, "--maxaccepts")) { const char* v = val(); if (!v) return UMICLUST_EINVAL; p->maxaccepts = atoi(v); }
    else if (!strcmp(a, "--maxrejects")) { const char* v = val(); if (!v) return UMICLUST_EINVAL; p->maxrejects = atoi(v); }
    else if (!strcmp(a, "--fasta_width")) { const char* v = val(); if (!v) return UMICLUST_EINVAL; p->fasta_width = atoi(v); }
    else return UMICLUST_EINVAL;
  }
  if (!have_in) return UMICLUST_EINVAL;
  // O4: the argv's --threads n > 1 selects vsearch's multithreaded clustering (the batched
  // restatement of cluster_core_parallel, rounds of n queries) -- what the reference's vsearch computes, since it
  // always passes --threads n >= 25 (vsearch_umi_cluster.py:33-34,83-84; utils.py:56-63).  --threads 1 (or none) is
  // the sequential definition.  UMICLUST_O4=sequential forces the sequential definition whatever --threads says.
  p->policy_threads = p->threads > 1 ? 1 : 0;
  if (const char* e = getenv("UMICLUST_O4")) {
    if (!strcmp(e, "sequential")) p->policy_threads = 0;
    else if (strcmp(e, "batched") != 0) return UMICLUST_EINVAL;
  }
  return UMICLUST_OK;
}

}  // extern "C"
