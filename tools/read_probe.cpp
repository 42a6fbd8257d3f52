// read_probe.cpp -- how fast can the drop-in's FASTA reader get the input into memory?  Variants of
// host_io.cpp read_fasta's first step (measurement only; the product keeps one of them):
//   0 mmap MAP_POPULATE (one thread populates), then T parse threads
//   1 mmap, no populate (the parse threads fault their own slices in)
//   2 mmap, each thread MADV_POPULATE_READ's its slice, then parses it
//   3 T threads pread their slices into one buffer, then parse
// Usage: read_probe <fasta> <threads>   (prints one JSON line per variant and repeat)
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22
#endif

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

// the parse loop's memory pattern: memchr per line, count records and sequence letters
static void parse(const char* d, size_t a, size_t b, size_t& rec, size_t& let) {
  size_t i = a;
  while (i < b) {
    const char* nl = (const char*)memchr(d + i, '\n', b - i);
    const size_t e = nl ? (size_t)(nl - d) : b;
    if (d[i] == '>') rec++;
    else
      for (size_t k = i; k < e; k++) let += (d[k] >= 'A' && d[k] <= 'Z');
    i = e + 1;
  }
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const int T = atoi(argv[2]);
  for (int rep = 0; rep < 3; rep++)
    for (int v = 0; v < 4; v++) {
      const double t0 = now();
      const int fd = open(argv[1], O_RDONLY);
      struct stat sb;
      fstat(fd, &sb);
      const size_t N = (size_t)sb.st_size;
      char* buf = nullptr;
      void* map = nullptr;
      if (v == 3) {
        buf = (char*)malloc(N);
      } else {
        map = mmap(nullptr, N, PROT_READ, MAP_PRIVATE | (v == 0 ? MAP_POPULATE : 0), fd, 0);
        buf = (char*)map;
      }
      const double t1 = now();
      std::vector<size_t> cut(T + 1, N);
      for (int t = 0; t < T; t++) cut[t] = N / T * t;  // byte slices (record alignment does not matter here)
      std::vector<size_t> rec(T, 0), let(T, 0);
      std::vector<std::thread> th;
      for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
          if (v == 2) madvise(buf + (cut[t] & ~(size_t)4095), cut[t + 1] - (cut[t] & ~(size_t)4095), MADV_POPULATE_READ);
          if (v == 3) {
            size_t o = cut[t];
            while (o < cut[t + 1]) {
              const ssize_t r = pread(fd, buf + o, cut[t + 1] - o, (off_t)o);
              if (r <= 0) break;
              o += (size_t)r;
            }
          }
          parse(buf, cut[t], cut[t + 1], rec[t], let[t]);
        });
      for (auto& x : th) x.join();
      const double t2 = now();
      size_t R = 0, L = 0;
      for (int t = 0; t < T; t++) R += rec[t], L += let[t];
      if (v == 3) free(buf);
      else munmap(map, N);
      close(fd);
      printf("{\"variant\": %d, \"rep\": %d, \"threads\": %d, \"map_s\": %.4f, \"total_s\": %.4f, \"records\": %zu, \"letters\": %zu}\n",
             v, rep, T, t1 - t0, t2 - t0, R, L);
      fflush(stdout);
    }
  return 0;
}
