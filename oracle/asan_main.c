/*
 * asan_main.c -- TEST INFRASTRUCTURE ONLY: drives the C oracle under AddressSanitizer +
 * UndefinedBehaviorSanitizer (host code; `make -C oracle asan_check`, run by tests/test_sanitizers_cpu.py).
 * Seeded UMI-like sequences (structured 64-nt patterns with substitutions, indels, IUPAC symbols, lengths
 * around the length filter) through orc_cluster (both presets, several identities), orc_align (with CIGAR)
 * and orc_dust/orc_unique_kmers; any sanitizer report aborts with a non-zero exit status.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "umiclust_oracle.h"

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static uint32_t rnd(void) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)(rng >> 11);
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 3000;
  const char *pat = "TTTVVVVTTVVVVTTVVVVTTVVVVTTTAAABBBBAABBBBAABBBBAABBBBAAA";
  const int nmol = n / 12 + 1;
  char **mol = malloc(sizeof(char *) * nmol);
  for (int m = 0; m < nmol; m++) {
    mol[m] = malloc(80);
    int L = (int)strlen(pat);
    for (int i = 0; i < L; i++)
      mol[m][i] = pat[i] == 'V' ? "ACG"[rnd() % 3] : pat[i] == 'B' ? "CGT"[rnd() % 3] : pat[i];
    mol[m][L] = 0;
  }
  char **seqs = malloc(sizeof(char *) * n);
  int32_t *lens = malloc(sizeof(int32_t) * n);
  for (int i = 0; i < n; i++) {
    const char *src = mol[rnd() % nmol];
    char *s = malloc(128);
    int L = 0;
    for (int j = 0; src[j] && L < 120; j++) {
      const uint32_t u = rnd() % 1000;
      if (u < 8) continue;                                   /* deletion */
      if (u < 16) s[L++] = "ACGT"[rnd() % 4];                /* insertion before */
      s[L++] = u < 40 ? "ACGTN"[rnd() % 5] : src[j];         /* substitution / IUPAC N */
    }
    if (rnd() % 50 == 0) L = 20 + (int)(rnd() % 40);         /* short: length-filtered */
    s[L] = 0;
    if (rnd() % 2) { /* reverse complement */
      for (int a = 0, b = L - 1; a < b; a++, b--) { char t = s[a]; s[a] = s[b]; s[b] = t; }
      for (int a = 0; a < L; a++) s[a] = s[a] == 'A' ? 'T' : s[a] == 'C' ? 'G' : s[a] == 'G' ? 'C' : s[a] == 'T' ? 'A' : s[a];
    }
    seqs[i] = s;
    lens[i] = L;
  }
  int32_t *cl = malloc(sizeof(int32_t) * n), *sorted = malloc(sizeof(int32_t) * n);
  uint8_t *st = malloc(n), *ce = malloc(n);
  int64_t *off = malloc(sizeof(int64_t) * (n + 1)), stats[8];
  const int64_t cap = (int64_t)n * 128;
  char *cons = malloc(cap);
  const struct { int preset; double id; } runs[] = {{1, 0.93}, {1, 0.90}, {2, 0.97}, {1, 0.75}};
  for (unsigned r = 0; r < sizeof(runs) / sizeof(runs[0]); r++) {
    orc_params p;
    orc_params_preset(&p, runs[r].preset, runs[r].id, 50, 70);
    const int64_t k = orc_cluster(&p, n, (const char *const *)seqs, lens, cl, st, ce, sorted, cons, cap, off, stats);
    if (k < 0) { fprintf(stderr, "orc_cluster failed: %lld\n", (long long)k); return 2; }
    printf("preset %d id %.2f: %lld clusters, %lld alignments\n", runs[r].preset, runs[r].id, (long long)k,
           (long long)stats[2]);
  }
  orc_params p;
  orc_params_preset(&p, 2, 0.97, 1, 200);
  char cig[2 * 256 + 1];
  uint32_t km[256];
  for (int i = 0; i + 1 < n && i < 2000; i += 2) {
    int cols, m, mm, g, tl, tr, il;
    double id2;
    orc_align(&p, seqs[i], lens[i], seqs[i + 1], lens[i + 1], &cols, &m, &mm, &g, &tl, &tr, &il, &id2, cig);
    char buf[128];
    memcpy(buf, seqs[i], (size_t)lens[i] + 1);
    orc_dust(buf, lens[i]);
    (void)orc_unique_kmers(buf, lens[i], 8, 1, km);
  }
  for (int i = 0; i < n; i++) free(seqs[i]);
  for (int m = 0; m < nmol; m++) free(mol[m]);
  free(mol); free(seqs); free(lens); free(cl); free(sorted); free(st); free(ce); free(off); free(cons);
  printf("ok\n");
  return 0;
}
