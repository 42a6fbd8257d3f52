// resolve_tsan_main.cpp -- host-only replay of recorded resolve_block calls (test infrastructure, no GPU).
//
// driver.cpp writes a pass's inputs, round-B pairs and results, and outputs with UMICLUST_RESOLVE_DUMP
// (write_resolve_dump); this replays each dump through resolve.cpp's resolve_block with a worker pool of 1, 3 and
// 8 threads -- the classify phase on the pool, the in-order phase and round B on the caller, as in a clustering
// run -- and checks every output against the recorded one (states, targets, strands of the block, the new
// centroids, alignments, cells).  Built with -fsanitize=thread by tests/test_sanitizers_cpu.py, so the pool's
// shared state (the window's states read by the classify threads, the per-thread scratch, the pass scratch) is
// checked for data races.  Round B is served from the recorded results (the same pairs must be asked for).
//
// Usage: resolve_tsan_main <dump.bin>...   exit status 0 iff every replay matches.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../ont-tcrconsensus_amd/csrc/resolve.h"

using namespace uc;

namespace {

struct Reader {
  std::vector<uint8_t> b;
  size_t o = 0;
  bool ok = true;
  void get(void* p, size_t n) {
    if (o + n > b.size()) {
      ok = false;
      memset(p, 0, n);
      return;
    }
    memcpy(p, b.data() + o, n);
    o += n;
  }
  int64_t i64() {
    int64_t v = 0;
    get(&v, 8);
    return v;
  }
  template <typename T>
  std::vector<T> vec(int64_t n) {
    std::vector<T> v((size_t)(n > 0 ? n : 0));
    if (n > 0) get(v.data(), (size_t)n * sizeof(T));
    return v;
  }
};

int replay(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "%s: cannot open\n", path);
    return 1;
  }
  Reader r;
  for (int ch; (ch = fgetc(f)) != EOF;) r.b.push_back((uint8_t)ch);
  fclose(f);
  char magic[4];
  r.get(magic, 4);
  int32_t hdr[12];
  r.get(hdr, sizeof hdr);
  if (!r.ok || memcmp(magic, "UCRD", 4) != 0 || hdr[0] != 1) {
    fprintf(stderr, "%s: not a v1 resolve dump\n", path);
    return 1;
  }
  const int32_t q0 = hdr[1], nq = hdr[2], w0 = hdr[3], both = hdr[4], s0 = hdr[10];
  const int64_t nh = r.i64();
  std::vector<uint8_t> hlen((size_t)(q0 + nq), 0);
  r.get(hlen.data() + s0, (size_t)nh);
  std::vector<uint8_t> acc = r.vec<uint8_t>((int64_t)kTabL * kTabM);
  std::vector<uint16_t> rank = r.vec<uint16_t>((int64_t)kTabL * kTabM);
  std::vector<uint8_t> state_in = r.vec<uint8_t>(r.i64());
  const int64_t nqs = r.i64();
  std::vector<HostQs> hq = r.vec<HostQs>(nqs);
  std::vector<uint32_t> recs = r.vec<uint32_t>(r.i64());
  const int64_t nb = r.i64();
  std::vector<uint32_t> bpq = r.vec<uint32_t>(nb), bpt = r.vec<uint32_t>(nb), bres = r.vec<uint32_t>(nb);
  std::vector<uint8_t> state_out = r.vec<uint8_t>(nq);
  std::vector<int32_t> target_out = r.vec<int32_t>(nq);
  std::vector<uint8_t> strand_out = r.vec<uint8_t>(nq);
  std::vector<int32_t> cents_out = r.vec<int32_t>(r.i64());
  const int64_t aln_out = r.i64(), cells_out = r.i64();
  if (!r.ok || (int64_t)state_in.size() != q0 + nq - w0 || nqs != (int64_t)nq * both) {
    fprintf(stderr, "%s: truncated or inconsistent dump\n", path);
    return 1;
  }
  int bad = 0;
  // (threads, in-order phase on the pool from this many open queries): the default threshold, then the pool forced
  for (const auto& [T, par_min] : std::vector<std::pair<int, int>>{{1, kParInorderMin}, {3, kParInorderMin},
                                                                    {8, kParInorderMin}, {3, 1}, {8, 1}}) {
    // the bin's states: [s0, w0) final before the window (never read), the window as recorded
    std::vector<uint8_t> st_buf((size_t)(q0 + nq - s0), ST_MEMBER);
    memcpy(st_buf.data() + (w0 - s0), state_in.data(), state_in.size());
    StateView state{st_buf.data(), s0};
    std::vector<int32_t> target((size_t)(q0 + nq), -1);
    std::vector<uint8_t> strand((size_t)(q0 + nq), 0);
    ResolveEnv env;
    env.hlen = hlen.data();
    env.acc = acc.data();
    env.rank = rank.data();
    env.both = both;
    env.o4_T = hdr[5];
    env.maxaccepts = hdr[6];
    env.maxrejects = hdr[7];
    env.pre_resolve = hdr[8] != 0;
    env.pre_spec = hdr[9] != 0;
    env.par_min = par_min;
    env.target = target.data();
    env.strand = strand.data();
    size_t served = 0;
    bool rb_ok = true;
    RoundB rb = [&](const std::vector<uint32_t>& pq, const std::vector<uint32_t>& pt, std::vector<uint32_t>& res) {
      for (size_t x = 0; x < pq.size(); x++) {
        if (served + x >= bpq.size() || bpq[served + x] != pq[x] || bpt[served + x] != pt[x]) {
          rb_ok = false;
          res[x] = 0;
        } else {
          res[x] = bres[served + x];
        }
      }
      served += pq.size();
    };
    WorkPool pool(T);
    ResolveScratch scr;
    ResolveStats rs;
    std::vector<int32_t> cents;
    const int rc = resolve_block(env, q0, nq, w0, hq.data(), recs.data(), state, scr, pool, cents, rs, rb);
    bool ok = rc == kResolveOk && rb_ok && served == bpq.size() && cents == cents_out && rs.n_alignments == aln_out &&
              rs.cells == cells_out;
    for (int32_t i = 0; i < nq && ok; i++)
      ok = st_buf[(size_t)(q0 + i - s0)] == state_out[i] && target[(size_t)(q0 + i)] == target_out[i] &&
           (state_out[i] != ST_MEMBER || strand[(size_t)(q0 + i)] == strand_out[i]);
    printf("%s threads %d (pool in order from %d): block [%d, %d) window %d, %lld round-B pairs, %zu new centroids, "
           "%lld alignments: %s\n", path, T, par_min, q0, q0 + nq, w0, (long long)nb, cents.size(),
           (long long)rs.n_alignments, ok ? "equal" : "DIFFERENT");
    bad += ok ? 0 : 1;
  }
  return bad;
}

}  // namespace

int main(int argc, char** argv) {
  int bad = 0;
  for (int i = 1; i < argc; i++) bad += replay(argv[i]);
  if (argc < 2) fprintf(stderr, "usage: resolve_tsan_main <dump.bin>...\n");
  return bad || argc < 2 ? 1 : 0;
}
