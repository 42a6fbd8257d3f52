/*
 * io_probe.c -- filesystem write-bandwidth probe for bench.py's e2e leg (measurement only; not product code).
 *
 * Writes `total` bytes into `nfiles` files (probe<i>, equal sizes, one open/write/close each) under `dir`
 * from `threads` threads -- the same shape as the drop-in's writers (one file per cluster, written on the
 * I/O threads) -- and returns the seconds taken.  With nfiles == 1 the threads pwrite disjoint slices of
 * one file (the shape of consout / smolecule_clusters.fa).  If `fsync_s` is not NULL every file is then
 * fsync'd and the extra seconds reported there (the disk-commit cost the writers never pay: they close
 * without fsync, as vsearch and Python's file objects do).  Files are removed afterwards (not timed).
 * io_probe_mmap: the one-file shape written through a shared mapping instead (ftruncate, mmap, the threads
 * copy their slices, munmap, close): buffered write()/pwrite() into one file serialise on its inode lock.
 *
 * Built by __graft_entry__.build() into tools/libioprobe.so; loaded by bench.py with ctypes.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <sys/mman.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

typedef struct {
  const char *dir;
  int64_t nfiles, total;
  int threads, t;
  const char *buf;
  int64_t bufsz;
  int err;
} job_t;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int write_all(int fd, const char *p, int64_t n, int64_t off, int positional) {
  while (n > 0) {
    ssize_t w = positional ? pwrite(fd, p, (size_t)n, off) : write(fd, p, (size_t)n);
    if (w < 0) {
      if (errno == EINTR) continue;
      return -1;
    }
    p += w;
    n -= w;
    off += w;
  }
  return 0;
}

static void *files_worker(void *arg) {
  job_t *j = (job_t *)arg;
  char path[4096];
  const int64_t per = j->total / j->nfiles;
  for (int64_t i = j->t; i < j->nfiles; i += j->threads) {
    snprintf(path, sizeof path, "%s/probe%lld", j->dir, (long long)i);
    int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0666);
    if (fd < 0) { j->err = errno; return NULL; }
    int64_t left = per + (i == j->nfiles - 1 ? j->total - per * j->nfiles : 0);
    while (left > 0 && !j->err) {
      int64_t n = left < j->bufsz ? left : j->bufsz;
      if (write_all(fd, j->buf, n, 0, 0)) j->err = errno;
      left -= n;
    }
    if (close(fd)) j->err = errno;
  }
  return NULL;
}

static void *slice_worker(void *arg) {
  job_t *j = (job_t *)arg;
  char path[4096];
  snprintf(path, sizeof path, "%s/probe0", j->dir);
  int fd = open(path, O_WRONLY);
  if (fd < 0) { j->err = errno; return NULL; }
  int64_t a = j->total * j->t / j->threads, b = j->total * (j->t + 1) / j->threads;
  while (a < b && !j->err) {
    int64_t n = b - a < j->bufsz ? b - a : j->bufsz;
    if (write_all(fd, j->buf, n, a, 1)) j->err = errno;
    a += n;
  }
  close(fd);
  return NULL;
}

double io_probe(const char *dir, int64_t nfiles, int64_t total, int threads, double *fsync_s) {
  if (!dir || nfiles < 1 || total < 0 || threads < 1) return -1.0;
  const int64_t bufsz = 1 << 20;
  char *buf = (char *)malloc((size_t)bufsz);
  if (!buf) return -1.0;
  for (int64_t i = 0; i < bufsz; i++) buf[i] = "ACGT\n"[i % 5];
  char path[4096];
  if (nfiles == 1) {  /* one file, pre-sized, threads writing disjoint slices */
    snprintf(path, sizeof path, "%s/probe0", dir);
    int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0666);
    if (fd < 0) { free(buf); return -1.0; }
    close(fd);
  }
  pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  job_t *jobs = (job_t *)calloc((size_t)threads, sizeof(job_t));
  const double t0 = now_s();
  if (nfiles == 1) {
    int fd = open(path, O_WRONLY);
    if (fd >= 0) {
      if (ftruncate(fd, total)) jobs[0].err = errno;
      close(fd);
    }
  }
  for (int t = 0; t < threads; t++) {
    jobs[t] = (job_t){dir, nfiles, total, threads, t, buf, bufsz, 0};
    pthread_create(&th[t], NULL, nfiles == 1 ? slice_worker : files_worker, &jobs[t]);
  }
  int err = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    if (jobs[t].err) err = jobs[t].err;
  }
  const double dt = now_s() - t0;
  if (fsync_s) {
    const double t1 = now_s();
    for (int64_t i = 0; i < nfiles; i++) {
      snprintf(path, sizeof path, "%s/probe%lld", dir, (long long)i);
      int fd = open(path, O_WRONLY);
      if (fd >= 0) {
        if (fsync(fd)) err = errno;
        close(fd);
      }
    }
    *fsync_s = now_s() - t1;
  }
  for (int64_t i = 0; i < nfiles; i++) {
    snprintf(path, sizeof path, "%s/probe%lld", dir, (long long)i);
    unlink(path);
  }
  free(jobs);
  free(th);
  free(buf);
  return err ? -1.0 : dt;
}

typedef struct {
  char *map;
  int64_t total;
  int threads, t;
  const char *buf;
  int64_t bufsz;
} mjob_t;

static void *mmap_worker(void *arg) {
  mjob_t *j = (mjob_t *)arg;
  int64_t a = j->total * j->t / j->threads, b = j->total * (j->t + 1) / j->threads;
  while (a < b) {
    int64_t n = b - a < j->bufsz ? b - a : j->bufsz;
    memcpy(j->map + a, j->buf, (size_t)n);
    a += n;
  }
  return NULL;
}

double io_probe_mmap(const char *dir, int64_t total, int threads) {
  if (!dir || total <= 0 || threads < 1) return -1.0;
  const int64_t bufsz = 1 << 20;
  char *buf = (char *)malloc((size_t)bufsz);
  if (!buf) return -1.0;
  for (int64_t i = 0; i < bufsz; i++) buf[i] = "ACGT\n"[i % 5];
  char path[4096];
  snprintf(path, sizeof path, "%s/probe0", dir);
  const double t0 = now_s();
  int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0666);
  int err = fd < 0;
  char *map = NULL;
  if (!err && ftruncate(fd, total)) err = 1;
  if (!err) {
    map = (char *)mmap(NULL, (size_t)total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (map == MAP_FAILED) err = 1;
  }
  if (!err) {
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    mjob_t *jobs = (mjob_t *)calloc((size_t)threads, sizeof(mjob_t));
    for (int t = 0; t < threads; t++) {
      jobs[t] = (mjob_t){map, total, threads, t, buf, bufsz};
      pthread_create(&th[t], NULL, mmap_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    munmap(map, (size_t)total);
    free(jobs);
    free(th);
  }
  if (fd >= 0) close(fd);
  const double dt = now_s() - t0;
  unlink(path);
  free(buf);
  return err ? -1.0 : dt;
}

/* io_probe_replay: the writers' own system-call sequence with no formatting -- the bound a writer cannot beat on
 * the same filesystem.  nfiles files named <dir>/cluster<i>.fasta of the given sizes, split over `threads` threads
 * in contiguous ranges of about equal bytes (the writers' cluster_slices), each file one open / write / close from a
 * prepared buffer; with one_bytes > 0 one more file <dir>/one is written beside them as the fused writer writes
 * smolecule_clusters.fa: pre-created, every thread pwrite-ing its share (proportional to its files' bytes) at its
 * offset in chunks of 8 MiB as its files accumulate it.  Returns seconds (files removed afterwards, untimed). */
typedef struct {
  const char *dir;
  const int64_t *sizes;
  int64_t f0, f1;          /* files [f0, f1) */
  int one_fd;
  int64_t one_at, one_n;   /* this thread's slice of the one file */
  int64_t files_bytes;     /* bytes of its files (the slice is streamed in proportion) */
  const char *buf;
  int64_t bufsz;
  int err;
} rjob_t;

static void *replay_worker(void *arg) {
  rjob_t *j = (rjob_t *)arg;
  char path[4096];
  const int64_t chunk = 8 << 20;
  int64_t done = 0, sent = 0;
  for (int64_t i = j->f0; i < j->f1 && !j->err; i++) {
    snprintf(path, sizeof path, "%s/cluster%lld.fasta", j->dir, (long long)i);
    int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0666);
    if (fd < 0) { j->err = errno; break; }
    int64_t left = j->sizes[i];
    while (left > 0 && !j->err) {
      int64_t n = left < j->bufsz ? left : j->bufsz;
      if (write_all(fd, j->buf, n, 0, 0)) j->err = errno;
      left -= n;
    }
    if (close(fd)) j->err = errno;
    done += j->sizes[i];
    if (j->one_fd >= 0 && j->one_n > 0) {
      const int64_t due = j->files_bytes > 0 ? (int64_t)((double)j->one_n * (double)done / (double)j->files_bytes) : j->one_n;
      while (due - sent >= chunk && !j->err) {
        int64_t n = chunk;
        for (int64_t o = 0; o < n && !j->err; o += j->bufsz) {
          int64_t m = n - o < j->bufsz ? n - o : j->bufsz;
          if (write_all(j->one_fd, j->buf, m, j->one_at + sent + o, 1)) j->err = errno;
        }
        sent += n;
      }
    }
  }
  while (j->one_fd >= 0 && sent < j->one_n && !j->err) {
    int64_t m = j->one_n - sent < j->bufsz ? j->one_n - sent : j->bufsz;
    if (write_all(j->one_fd, j->buf, m, j->one_at + sent, 1)) j->err = errno;
    sent += m;
  }
  return NULL;
}

double io_probe_replay(const char *dir, int64_t nfiles, const int64_t *sizes, int threads, int64_t one_bytes) {
  if (!dir || nfiles < 0 || (nfiles > 0 && !sizes) || threads < 1 || one_bytes < 0) return -1.0;
  int64_t maxsz = 1 << 20, tot = 0;
  for (int64_t i = 0; i < nfiles; i++) {
    tot += sizes[i];
    if (sizes[i] > maxsz) maxsz = sizes[i];
  }
  const int64_t bufsz = maxsz < (8 << 20) ? maxsz : (8 << 20);
  char *buf = (char *)malloc((size_t)bufsz);
  if (!buf) return -1.0;
  for (int64_t i = 0; i < bufsz; i++) buf[i] = "ACGT\n"[i % 5];
  pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
  rjob_t *jobs = (rjob_t *)calloc((size_t)threads, sizeof(rjob_t));
  char path[4096];
  snprintf(path, sizeof path, "%s/one", dir);
  const double t0 = now_s();
  int one_fd = -1, err = 0;
  if (one_bytes > 0) {
    one_fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0666);
    if (one_fd < 0) err = errno;
  }
  int64_t f = 0, acc = 0, one_at = 0;
  for (int t = 0; t < threads; t++) {
    const int64_t want = tot * (t + 1) / threads;
    const int64_t f0 = f;
    int64_t fb = 0;
    while (f < nfiles && (t == threads - 1 || acc < want)) {
      acc += sizes[f];
      fb += sizes[f];
      f++;
    }
    const int64_t share = tot > 0 ? (int64_t)((double)one_bytes * (double)acc / (double)tot) - one_at
                                  : (t == threads - 1 ? one_bytes : 0);
    jobs[t] = (rjob_t){dir, sizes, f0, f, one_fd, one_at, t == threads - 1 ? one_bytes - one_at : share, fb, buf, bufsz, 0};
    one_at += jobs[t].one_n;
  }
  for (int t = 0; t < threads && !err; t++) pthread_create(&th[t], NULL, replay_worker, &jobs[t]);
  for (int t = 0; t < threads && !err; t++) {
    pthread_join(th[t], NULL);
    if (jobs[t].err) err = jobs[t].err;
  }
  if (one_fd >= 0 && close(one_fd)) err = errno;
  const double dt = now_s() - t0;
  for (int64_t i = 0; i < nfiles; i++) {
    char p2[4096];
    snprintf(p2, sizeof p2, "%s/cluster%lld.fasta", dir, (long long)i);
    unlink(p2);
  }
  if (one_bytes > 0) unlink(path);
  free(jobs);
  free(th);
  free(buf);
  return err ? -1.0 : dt;
}
