/*
 * umiclust_oracle.c -- CPU ORACLE (test infrastructure only; see umiclust_oracle.h).
 *
 * Restates vsearch 2.29 `--cluster_fast` + `--consout` (the arithmetic the reference
 * delegates to at /root/reference/ont_tcr_consensus/vsearch_umi_cluster.py:21-54,71-97).
 * vsearch is an external, un-vendored dependency (pyproject.toml:39 `vsearch>=2.29.0`);
 * each function below names the upstream vsearch routine it restates and the SURVEY.md
 * Appendix A item it follows.  PARITY UNPINNED (no vsearch binary/source/goldens offline).
 *
 * Deliberately written as plain, scalar, allocation-heavy C: it is the checker, not the
 * product.  Nothing here is shared with ont-tcrconsensus_amd/csrc.
 */
#ifdef _OPENMP
#include <omp.h>
#endif
#include "umiclust_oracle.h"

#include <ctype.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NEG_INF (-100000000)
#define MAXDELAYED 8 /* searchcore.cc */

/* ------------------------------------------------------------------ char maps */
/* chrmap_4bit (vsearch maps.cc): IUPAC bitmask A=1 C=2 G=4 T/U=8 */
static unsigned char map4[256];
/* chrmap_2bit: A0 C1 G2 T/U3, everything else 0 */
static unsigned char map2[256];
static char compl_tab[256];
static int maps_ready = 0;

static void init_maps(void) {
  if (maps_ready) return;
  memset(map4, 0, sizeof(map4));
  memset(map2, 0, sizeof(map2));
  const char *iupac = "ACGTURYSWKMBDHVN";
  const unsigned char v4[] = {1, 2, 4, 8, 8, 5, 10, 6, 9, 12, 3, 14, 13, 11, 7, 15};
  for (int i = 0; iupac[i]; i++) {
    map4[(unsigned char)iupac[i]] = v4[i];
    map4[(unsigned char)tolower(iupac[i])] = v4[i];
  }
  map2['A'] = map2['a'] = 0;
  map2['C'] = map2['c'] = 1;
  map2['G'] = map2['g'] = 2;
  map2['T'] = map2['t'] = map2['U'] = map2['u'] = 3;
  for (int i = 0; i < 256; i++) compl_tab[i] = (char)i;
  const char *a = "ACGTURYSWKMBDHVN", *b = "TGCAAYRSWMKVHDBN";
  for (int i = 0; a[i]; i++) {
    compl_tab[(unsigned char)a[i]] = b[i];
    compl_tab[(unsigned char)tolower(a[i])] = (char)tolower(b[i]);
  }
  maps_ready = 1;
}

static int is_ambig(unsigned char c) {
  unsigned v = map4[c];
  return !(v == 1 || v == 2 || v == 4 || v == 8);
}

/* reverse_complement (vsearch util.cc): case preserved */
static void revcomp(char *dst, const char *src, int len) {
  for (int i = 0; i < len; i++) dst[i] = compl_tab[(unsigned char)src[len - 1 - i]];
  dst[len] = 0;
}

/* ------------------------------------------------------------------ params */
void orc_params_preset(orc_params *p, int preset, double id, int minlen, int maxlen) {
  memset(p, 0, sizeof(*p));
  p->id = id;
  p->weak_id = 0.10 < id ? 0.10 : id;  /* opt_weak_id default 10.0 (percent), clipped to id */
  p->minseqlength = minlen;
  p->maxseqlength = maxlen;
  p->wordlength = 8;
  p->minwordmatches = 12;  /* minwordmatches_defaults[8] */
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
  for (int k = 0; k < 6; k++) p->gap_ext[k] = (k == ORC_QI || k == ORC_TI) ? 2 : 1; /* 2I/1E */
  if (preset == 1) {
    /* --gapopen 0E/40I --mismatch -40 --match 10 (vsearch_umi_cluster.py:44-50) */
    p->match = 10;
    p->mismatch = -40;
    for (int k = 0; k < 6; k++) p->gap_open[k] = (k == ORC_QI || k == ORC_TI) ? 40 : 0;
  } else {
    /* vsearch defaults: --match 2 --mismatch -4 --gapopen 20I/2E --gapext 2I/1E */
    p->match = 2;
    p->mismatch = -4;
    for (int k = 0; k < 6; k++) p->gap_open[k] = (k == ORC_QI || k == ORC_TI) ? 20 : 2;
  }
}

/* ------------------------------------------------------------------ DUST (mask.cc) */
/* wo(): best low-complexity interval of one window; vsearch's rewrite of NCBI dust with
 * 2-bit triplet words and "smallest possible region is 8" (l1 = len - word + 1 - 5). */
static int dust_wo(int len, const char *s, int *beg, int *end) {
  const int word = 3;
  int l1 = len - word + 1 - 5;
  if (l1 < 0) {
    *beg = 0;
    *end = len - 1;
    return 0;
  }
  int bestv = 0, besti = 0, bestj = 0;
  int counts[64];
  int words[64];
  unsigned w = 0;  /* only the last triplet (6 bits) is used; unsigned: no overflow on long windows */
  for (int j = 0; j < len; j++) {
    w = (w << 2) | (unsigned)map2[(unsigned char)s[j]];
    words[j] = (int)(w & 63u);
  }
  for (int i = 0; i < l1; i++) {
    memset(counts, 0, sizeof(counts));
    int sum = 0;
    for (int j = word - 1; j < len - i; j++) {
      int x = words[i + j];
      int c = counts[x];
      if (c) {
        sum += c;
        int v = 10 * sum / j;
        if (v > bestv) {
          bestv = v;
          besti = i;
          bestj = j;
        }
      }
      counts[x]++;
    }
  }
  *beg = besti;
  *end = besti + bestj;
  return bestv;
}

void orc_dust(char *m, int len) {
  init_maps();
  const int level = 20, window = 64, window2 = 32;
  char *s = (char *)malloc((size_t)len + 1);
  memcpy(s, m, (size_t)len);
  s[len] = 0;
  for (int i = 0; i < len; i++) m[i] = (char)toupper((unsigned char)m[i]);
  for (int i = 0; i < len; i += window2) {
    int l = (len > i + window) ? window : len - i;
    int a = 0, b = 0;
    int v = dust_wo(l, s + i, &a, &b);
    if (v > level)
      for (int j = a + i; j <= b + i; j++) m[j] = (char)tolower((unsigned char)s[j]);
  }
  free(s);
}

/* ------------------------------------------------------------------ k-mers (unique.cc) */
int orc_unique_kmers(const char *seq, int len, int k, int mask, uint32_t *out) {
  init_maps();
  uint64_t kmask = (k >= 32) ? ~0ULL : ((1ULL << (2 * k)) - 1);
  uint64_t badmask = (1ULL << k) - 1;
  uint64_t bad = 0, kmer = 0;
  int n = 0;
  size_t bmwords = ((size_t)1 << (2 * k)) / 64 + 1;
  uint64_t *seen = (uint64_t *)calloc(bmwords, 8);
  for (int i = 0; i < len; i++) {
    unsigned char c = (unsigned char)seq[i];
    bad = ((bad << 1) | ((mask && islower(c)) ? 1u : 0u)) & badmask;
    kmer = ((kmer << 2) | map2[c]) & kmask;
    if (i >= k - 1 && !bad) {
      if (!(seen[kmer >> 6] & (1ULL << (kmer & 63)))) {
        seen[kmer >> 6] |= 1ULL << (kmer & 63);
        out[n++] = (uint32_t)kmer;
      }
    }
  }
  free(seen);
  return n;
}

/* ------------------------------------------------------------------ alignment */
/* search16 (align_simd.cc) restated as a scalar Gotoh DP in max form:
 *   H(i,j) = best of diag = H(i-1,j-1)+s, F(i,j) (vertical, 'D'), E(i,j) (horizontal, 'I');
 *   a path bit is set only when the alternative is STRICTLY better (diag > D > I on ties),
 *   gap extension is recorded only when strictly better than opening (ties -> open).
 * Boundaries: H(-1,-1)=0, H(-1,j) = -(GO_QL+(j+1)GE_QL), H(i,-1) = -(GO_TL+(i+1)GE_TL).
 * Horizontal gaps in the last query row use the query-right penalties, vertical gaps in
 * the last target column the target-right penalties.
 * backtrack16: from (qlen-1,tlen-1): continue an I run if extleft, a D run if extup, else
 * left (I) if set, else up (D) if set, else M; leftovers -> D run then I run. */
static int score_sub(const orc_params *p, unsigned char a, unsigned char b) {
  if (is_ambig(a) || is_ambig(b)) return 0;
  return (map4[a] == map4[b]) ? p->match : p->mismatch;
}

typedef struct {
  int score, columns, matches, mismatches, gaps;
  int trim_left, trim_right, internal_len;
  double id2;
} aln_result;

static void run_push(char *ops, int *nops, char op) { ops[(*nops)++] = op; }

static void align_core(const orc_params *p, const char *q, int ql, const char *t, int tl,
                       aln_result *r, char *cigar) {
  init_maps();
  const int GOql = p->gap_open[ORC_QL], GEql = p->gap_ext[ORC_QL];
  const int GOtl = p->gap_open[ORC_TL], GEtl = p->gap_ext[ORC_TL];
  int W = tl + 1;
  int *H = (int *)malloc(sizeof(int) * (size_t)(ql + 1) * W); /* H[(i+1)*W + (j+1)] */
  int *F = (int *)malloc(sizeof(int) * (size_t)(tl));
  unsigned char *dir = (unsigned char *)calloc((size_t)ql * tl + 1, 1);
#define HH(i, j) H[((i) + 1) * W + ((j) + 1)]
  HH(-1, -1) = 0;
  for (int j = 0; j < tl; j++) HH(-1, j) = -(GOql + (j + 1) * GEql);
  for (int i = 0; i < ql; i++) HH(i, -1) = -(GOtl + (i + 1) * GEtl);
  for (int j = 0; j < tl; j++) {
    int rt = (j == tl - 1) ? ORC_TR : ORC_TI;
    F[j] = p->policy_boundary_open ? HH(-1, j) - (p->gap_open[rt] + p->gap_ext[rt]) : NEG_INF;
  }
  for (int i = 0; i < ql; i++) {
    int rq = (i == ql - 1) ? ORC_QR : ORC_QI;
    int QRq = p->gap_open[rq] + p->gap_ext[rq], Rq = p->gap_ext[rq];
    int E = p->policy_boundary_open ? HH(i, -1) - QRq : NEG_INF;
    for (int j = 0; j < tl; j++) {
      int rt = (j == tl - 1) ? ORC_TR : ORC_TI;
      int QRt = p->gap_open[rt] + p->gap_ext[rt], Rt = p->gap_ext[rt];
      int h = HH(i - 1, j - 1) + score_sub(p, (unsigned char)q[i], (unsigned char)t[j]);
      int f = F[j];
      unsigned char d = 0;
      if (f > h) { h = f; d |= 1; }          /* up   (D) */
      if (E > h) { h = E; d |= 2; }          /* left (I) */
      HH(i, j) = h;
      int fo = h - QRt, fe = f - Rt;
      if (fe > fo) { F[j] = fe; d |= 4; } else F[j] = fo;   /* extup   */
      int eo = h - QRq, ee = E - Rq;
      if (ee > eo) { E = ee; d |= 8; } else E = eo;          /* extleft */
      dir[(size_t)i * tl + j] = d;
    }
  }
  r->score = HH(ql - 1, tl - 1);
#undef HH
  /* backtrack16 */
  char *ops = (char *)malloc((size_t)(ql + tl) + 1);
  int nops = 0;
  int i = ql - 1, j = tl - 1;
  int aligned = 0, matches = 0, mismatches = 0, gaps = 0;
  char op = 0;
  while (i >= 0 && j >= 0) {
    aligned++;
    unsigned char d = dir[(size_t)i * tl + j];
    if (op == 'I' && (d & 8)) {
      j--;
      run_push(ops, &nops, 'I');
    } else if (op == 'D' && (d & 4)) {
      i--;
      run_push(ops, &nops, 'D');
    } else if (d & 2) {
      if (op != 'I') gaps++;
      j--;
      op = 'I';
      run_push(ops, &nops, 'I');
    } else if (d & 1) {
      if (op != 'D') gaps++;
      i--;
      op = 'D';
      run_push(ops, &nops, 'D');
    } else {
      if (map4[(unsigned char)q[i]] & map4[(unsigned char)t[j]]) matches++;
      else mismatches++;
      i--;
      j--;
      op = 'M';
      run_push(ops, &nops, 'M');
    }
  }
  while (i >= 0) {
    aligned++;
    if (op != 'D') gaps++;
    i--;
    op = 'D';
    run_push(ops, &nops, 'D');
  }
  while (j >= 0) {
    aligned++;
    if (op != 'I') gaps++;
    j--;
    op = 'I';
    run_push(ops, &nops, 'I');
  }
  /* ops[] is in reverse alignment order; alignment order = ops[nops-1 .. 0] */
  r->columns = aligned;
  r->matches = matches;
  r->mismatches = mismatches;
  r->gaps = gaps;
  /* align_trim (searchcore.cc / align.cc): first and last CIGAR runs, if not M */
  int tlft = 0, trgt = 0;
  if (nops > 0) {
    char first = ops[nops - 1];
    if (first != 'M') {
      int k = nops - 1;
      while (k >= 0 && ops[k] == first) { tlft++; k--; }
    }
    char last = ops[0];
    if (last != 'M') {
      int k = 0;
      while (k < nops && ops[k] == last) { trgt++; k++; }
    }
    if (tlft >= aligned) trgt = 0; /* single-run alignment: trimmed once */
  }
  r->trim_left = tlft;
  r->trim_right = trgt;
  r->internal_len = aligned - tlft - trgt;
  r->id2 = r->internal_len > 0 ? 100.0 * r->matches / r->internal_len : 0.0;
  if (cigar) {
    char *c = cigar;
    int k = nops - 1;
    while (k >= 0) {
      char o = ops[k];
      int run = 0;
      while (k >= 0 && ops[k] == o) { run++; k--; }
      if (run > 1) c += sprintf(c, "%d", run);
      *c++ = o;
    }
    *c = 0;
  }
  free(ops);
  free(dir);
  free(F);
  free(H);
}

int orc_align(const orc_params *p, const char *q, int qlen, const char *t, int tlen,
              int *columns, int *matches, int *mismatches, int *gaps,
              int *trim_left, int *trim_right, int *internal_len, double *id2, char *cigar) {
  aln_result r;
  align_core(p, q, qlen, t, tlen, &r, cigar);
  if (columns) *columns = r.columns;
  if (matches) *matches = r.matches;
  if (mismatches) *mismatches = r.mismatches;
  if (gaps) *gaps = r.gaps;
  if (trim_left) *trim_left = r.trim_left;
  if (trim_right) *trim_right = r.trim_right;
  if (internal_len) *internal_len = r.internal_len;
  if (id2) *id2 = r.id2;
  return r.score;
}

/* ------------------------------------------------------------------ clustering */
typedef struct {
  int32_t seqno;  /* sorted index of the centroid */
  int32_t count;
  int32_t len;
} cand_t;

static int cand_cmp(const void *a, const void *b) {
  /* minheap.cc elem_smaller inverted: count desc, length asc, seqno asc */
  const cand_t *x = (const cand_t *)a, *y = (const cand_t *)b;
  if (x->count != y->count) return x->count > y->count ? -1 : 1;
  if (x->len != y->len) return x->len < y->len ? -1 : 1;
  return x->seqno < y->seqno ? -1 : (x->seqno > y->seqno);
}

typedef struct {
  int32_t target;  /* sorted seqno of centroid */
  int accepted;
  double id;
  char *cigar;
  int32_t count;   /* shared unique k-mers */
  int aligned;     /* O4 recheck: hits inserted from the round's new centroids start unaligned */
} hit_t;

typedef struct {
  int32_t n;            /* kept sequences */
  char **seq;           /* sorted order, DUST-masked */
  int32_t *len;
  int32_t *orig;        /* sorted -> input index */
  /* index: centroid list and per-kmer posting lists (indexed centroid ordinal) */
  int32_t ncent;
  int32_t *cent_seqno;  /* ordinal -> sorted seqno */
  int32_t **post;
  int32_t *post_n, *post_cap;
  /* results per sorted seqno */
  int32_t *clusterno;   /* creation number */
  uint8_t *strand;
  char **cigar;
  int64_t alignments, cells, postings, candidates;
} ctx_t;

static void index_add(ctx_t *c, int32_t seqno, const orc_params *p, uint32_t *kbuf) {
  int nk = orc_unique_kmers(c->seq[seqno], c->len[seqno], p->wordlength, p->qmask_dust, kbuf);
  int32_t ord = c->ncent++;
  c->cent_seqno[ord] = seqno;
  for (int k = 0; k < nk; k++) {
    uint32_t km = kbuf[k];
    if (c->post_n[km] == c->post_cap[km]) {
      c->post_cap[km] = c->post_cap[km] ? 2 * c->post_cap[km] : 8;
      c->post[km] = (int32_t *)realloc(c->post[km], sizeof(int32_t) * (size_t)c->post_cap[km]);
    }
    c->post[km][c->post_n[km]++] = ord;
  }
}

/* align one hit (search16 semantics) and apply search_acceptable_aligned; returns accepted */
static int align_hit(ctx_t *c, const orc_params *p, const char *qs, int ql, hit_t *h) {
  int32_t ts = h->target;
  aln_result r;
  char *cg = (char *)malloc((size_t)(2 * (ql + c->len[ts]) + 2));
  align_core(p, qs, ql, c->seq[ts], c->len[ts], &r, cg);
  c->alignments++;
  c->cells += (int64_t)ql * c->len[ts];
  h->id = r.id2;
  free(h->cigar);
  h->cigar = cg;
  h->aligned = 1;
  /* search_acceptable_aligned: defaults leave only the id / weak-id tests */
  int mm = r.matches + r.mismatches;
  int ok = (r.id2 >= 100.0 * p->weak_id) && mm > 0 && (100.0 * r.matches / mm >= 0.0);
  h->accepted = ok && r.id2 >= 100.0 * p->id;
  return h->accepted;
}

/* search_onequery (searchcore.cc) for one strand: top scores + batched-8 alignment. */
static int search_strand(ctx_t *c, const orc_params *p, const char *qs, int ql, int strand,
                         uint32_t *kbuf, int32_t *counts, hit_t *hits) {
  int nk = orc_unique_kmers(qs, ql, p->wordlength, p->qmask_dust, kbuf);
  memset(counts, 0, sizeof(int32_t) * (size_t)c->ncent);
  for (int k = 0; k < nk; k++) {
    uint32_t km = kbuf[k];
    c->postings += c->post_n[km];
    for (int x = 0; x < c->post_n[km]; x++) counts[c->post[km][x]]++;
  }
  int minmatches = p->minwordmatches < nk ? p->minwordmatches : nk;
  cand_t *cand = (cand_t *)malloc(sizeof(cand_t) * (size_t)(c->ncent + 1));
  int nc = 0;
  for (int o = 0; o < c->ncent; o++)
    if (counts[o] >= minmatches) {
      int32_t s = c->cent_seqno[o];
      cand[nc].seqno = s;
      cand[nc].count = counts[o];
      cand[nc].len = c->len[s];
      nc++;
    }
  c->candidates += nc;
  qsort(cand, (size_t)nc, sizeof(cand_t), cand_cmp);
  int tophits = p->maxaccepts + p->maxrejects + MAXDELAYED;
  if (nc > tophits) nc = tophits;

  int hit_count = 0, finalized = 0, accepts = 0, rejects = 0, delayed = 0, pos = 0;
  for (;;) {
    while (finalized + delayed < p->maxaccepts + p->maxrejects - 1 && rejects < p->maxrejects &&
           accepts < p->maxaccepts && pos < nc) {
      hits[hit_count].target = cand[pos].seqno;
      hits[hit_count].count = cand[pos++].count;
      hits[hit_count].accepted = 0;
      hits[hit_count].aligned = 1;  /* align_delayed aligns every popped candidate */
      hits[hit_count].cigar = NULL;
      hit_count++;
      delayed++;
      if (delayed == MAXDELAYED) break;
    }
    if (delayed == 0) break;
    /* align_delayed */
    for (int x = finalized; x < hit_count; x++) {
      if (align_hit(c, p, qs, ql, &hits[x])) accepts++;
      else rejects++;
      finalized++;
    }
    delayed = 0;
  }
  (void)strand;
  free(cand);
  return hit_count;
}

/* per-output-cluster record for sorting */
typedef struct {
  int32_t cno;   /* creation number */
  int32_t size;
} csz_t;

static int csz_cmp(const void *a, const void *b) {
  const csz_t *x = (const csz_t *)a, *y = (const csz_t *)b;
  if (x->size != y->size) return x->size > y->size ? -1 : 1;
  return x->cno < y->cno ? -1 : (x->cno > y->cno);
}

/* msa() (msa.cc): star MSA against the centroid from stored CIGARs + majority consensus. */
static int64_t msa_consensus(ctx_t *c, const int32_t *members, int m, char *out) {
  int32_t cs = members[0];
  int clen = c->len[cs];
  int *maxi = (int *)calloc((size_t)clen + 1, sizeof(int));
  for (int k = 1; k < m; k++) {
    const char *pc = c->cigar[members[k]];
    int pos = 0;
    while (*pc) {
      int run = 0, has = 0;
      while (isdigit((unsigned char)*pc)) { run = run * 10 + (*pc - '0'); pc++; has = 1; }
      if (!has) run = 1;
      char op = *pc++;
      if (op == 'M' || op == 'I') pos += run;
      else if (op == 'D' && run > maxi[pos]) maxi[pos] = run;
    }
  }
  int alnlen = clen;
  for (int i = 0; i <= clen; i++) alnlen += maxi[i];
  int64_t (*prof)[6] = calloc((size_t)alnlen + 1, sizeof(*prof));
  char *rc = NULL;
  int rccap = 0;
  for (int k = 0; k < m; k++) {
    int32_t s = members[k];
    const char *seq = c->seq[s];
    if (k > 0 && c->strand[s]) {
      if (rccap < c->len[s] + 1) { rccap = c->len[s] + 1; rc = (char *)realloc(rc, (size_t)rccap); }
      revcomp(rc, seq, c->len[s]);
      seq = rc;
    }
    int alnpos = 0, qpos = 0, tpos = 0, inserted = 0;
#define ADD(ch) do { char _c = (char)toupper((unsigned char)(ch)); int _k; \
      switch (_c) { case 'A': _k = 0; break; case 'C': _k = 1; break; case 'G': _k = 2; break; \
      case 'T': case 'U': _k = 3; break; case '-': _k = 5; break; default: _k = 4; } \
      prof[alnpos++][_k] += 1; } while (0)
    if (k == 0) {
      for (int x = 0; x < clen; x++) {
        for (int y = 0; y < maxi[qpos]; y++) ADD('-');
        ADD(seq[tpos++]);
        qpos++;
      }
    } else {
      const char *pc = c->cigar[s];
      while (*pc) {
        int run = 0, has = 0;
        while (isdigit((unsigned char)*pc)) { run = run * 10 + (*pc - '0'); pc++; has = 1; }
        if (!has) run = 1;
        char op = *pc++;
        if (op == 'D') {
          for (int x = 0; x < maxi[qpos]; x++) {
            if (x < run) ADD(seq[tpos++]);
            else ADD('-');
          }
          inserted = 1;
        } else {
          for (int x = 0; x < run; x++) {
            if (!inserted)
              for (int y = 0; y < maxi[qpos]; y++) ADD('-');
            if (op == 'M') ADD(seq[tpos++]);
            else ADD('-');
            qpos++;
            inserted = 0;
          }
        }
      }
    }
    if (!inserted)
      for (int y = 0; y < maxi[qpos]; y++) ADD('-');
#undef ADD
  }
  int left = maxi[0], right = maxi[clen];
  int64_t conslen = 0;
  const char sym[5] = {'A', 'C', 'G', 'T', 'N'};
  for (int i = 0; i < alnlen; i++) {
    if (i < left || i >= alnlen - right) continue;
    int best = 0;
    int64_t bestc = 0;
    for (int x = 0; x < 4; x++)
      if (prof[i][x] > bestc) { bestc = prof[i][x]; best = x; }
    if (bestc == 0 && prof[i][4] > 0) { bestc = prof[i][4]; best = 4; }
    if (bestc >= prof[i][5]) out[conslen++] = sym[best];
  }
  free(rc);
  free(prof);
  free(maxi);
  return conslen;
}

int64_t orc_cluster(const orc_params *p, int32_t n, const char *const *seqs, const int32_t *lens,
                    int32_t *out_cluster, uint8_t *out_strand, uint8_t *out_centroid,
                    int32_t *out_sorted, char *cons_buf, int64_t cons_cap, int64_t *cons_off,
                    int64_t *stats) {
  init_maps();
  ctx_t c;
  memset(&c, 0, sizeof(c));
  /* db_read with length filter */
  int32_t *keep = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n + 1));
  int32_t nk = 0;
  for (int32_t i = 0; i < n; i++) {
    out_cluster[i] = -1;
    out_strand[i] = 0;
    out_centroid[i] = 0;
    if (lens[i] >= p->minseqlength && lens[i] <= p->maxseqlength) keep[nk++] = i;
  }
  /* db_sortbylength: length desc, ties in input order (policy O1); counting sort = stable */
  int32_t maxl = 0;
  for (int32_t k = 0; k < nk; k++) if (lens[keep[k]] > maxl) maxl = lens[keep[k]];
  int32_t *bucket = (int32_t *)calloc((size_t)maxl + 2, sizeof(int32_t));
  for (int32_t k = 0; k < nk; k++) bucket[maxl - lens[keep[k]]]++;
  int32_t acc = 0;
  for (int32_t l = 0; l <= maxl; l++) { int32_t t = bucket[l]; bucket[l] = acc; acc += t; }
  c.n = nk;
  c.orig = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nk + 1));
  for (int32_t k = 0; k < nk; k++) c.orig[bucket[maxl - lens[keep[k]]]++] = keep[k];
  free(bucket);
  free(keep);
  c.seq = (char **)malloc(sizeof(char *) * (size_t)(nk + 1));
  c.len = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nk + 1));
  int64_t masked = 0;
  for (int32_t s = 0; s < nk; s++) {
    int32_t i = c.orig[s];
    c.len[s] = lens[i];
    c.seq[s] = (char *)malloc((size_t)lens[i] + 1);
    memcpy(c.seq[s], seqs[i], (size_t)lens[i]);
    c.seq[s][lens[i]] = 0;
    /* dust_all() */
    if (p->qmask_dust) {
      orc_dust(c.seq[s], lens[i]);
      for (int x = 0; x < lens[i]; x++) if (islower((unsigned char)c.seq[s][x])) { masked++; break; }
    }
    if (out_sorted) out_sorted[s] = i;
  }
  int K = 1 << (2 * p->wordlength);
  c.post = (int32_t **)calloc((size_t)K, sizeof(int32_t *));
  c.post_n = (int32_t *)calloc((size_t)K, sizeof(int32_t));
  c.post_cap = (int32_t *)calloc((size_t)K, sizeof(int32_t));
  c.cent_seqno = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nk + 1));
  c.clusterno = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nk + 1));
  c.strand = (uint8_t *)calloc((size_t)nk + 1, 1);
  c.cigar = (char **)calloc((size_t)nk + 1, sizeof(char *));
  uint32_t *kbuf = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(maxl + 8));
  int32_t *counts = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nk + 1));
  int tophits = p->maxaccepts + p->maxrejects + MAXDELAYED;
  hit_t *hp = (hit_t *)malloc(sizeof(hit_t) * (size_t)tophits);
  hit_t *hm = (hit_t *)malloc(sizeof(hit_t) * (size_t)tophits);
  char *rcq = (char *)malloc((size_t)maxl + 2);
  int32_t clusters = 0;
  /* ORC_WALK_DUMP=<file>: alignments per sorted seqno and strand (search + O4 re-check), a parity-debugging aid */
  const char *walk_dump = getenv("ORC_WALK_DUMP");
  int16_t *wd = walk_dump ? (int16_t *)calloc((size_t)nk * 2 + 2, sizeof(int16_t)) : NULL;
  /* assign s from its hits: search_findbest2_byid (accepted hit with max id; tie -> lower target; plus
   * first), then a member of that centroid's cluster or a new centroid */
  #define ASSIGN(s, hp, np, hm, nm) do {                                                            \
    hit_t *best_ = NULL;                                                                            \
    int bs_ = 0;                                                                                    \
    for (int x = 0; x < (np); x++)                                                                  \
      if ((hp)[x].accepted && (!best_ || (hp)[x].id > best_->id ||                                  \
                               ((hp)[x].id == best_->id && (hp)[x].target < best_->target))) {      \
        best_ = &(hp)[x];                                                                           \
        bs_ = 0;                                                                                    \
      }                                                                                             \
    for (int x = 0; x < (nm); x++)                                                                  \
      if ((hm)[x].accepted && (!best_ || (hm)[x].id > best_->id ||                                  \
                               ((hm)[x].id == best_->id && (hm)[x].target < best_->target))) {      \
        best_ = &(hm)[x];                                                                           \
        bs_ = 1;                                                                                    \
      }                                                                                             \
    if (best_) {                                                                                    \
      c.clusterno[s] = c.clusterno[best_->target];                                                  \
      c.strand[s] = (uint8_t)bs_;                                                                   \
      c.cigar[s] = best_->cigar;                                                                    \
      best_->cigar = NULL;                                                                          \
    } else {                                                                                        \
      c.clusterno[s] = clusters++;                                                                  \
      index_add(&c, s, p, kbuf);                                                                    \
    }                                                                                               \
    for (int x = 0; x < (np); x++) free((hp)[x].cigar);                                             \
    for (int x = 0; x < (nm); x++) free((hm)[x].cigar);                                             \
  } while (0)
  const int32_t T = (p->policy_threads && p->threads > 1) ? p->threads : 1;
  if (T == 1) {
    /* cluster_core_serial (cluster.cc) */
    for (int32_t s = 0; s < nk; s++) {
      int64_t a0 = c.alignments;
      int np = search_strand(&c, p, c.seq[s], c.len[s], 0, kbuf, counts, hp);
      if (wd) wd[2 * s] = (int16_t)(c.alignments - a0);
      a0 = c.alignments;
      int nm = 0;
      if (p->strand_both) {
        revcomp(rcq, c.seq[s], c.len[s]);
        nm = search_strand(&c, p, rcq, c.len[s], 1, kbuf, counts, hm);
      }
      if (wd) wd[2 * s + 1] = (int16_t)(c.alignments - a0);
      ASSIGN(s, hp, np, hm, nm);
    }
  } else {
    /* cluster_core_parallel (cluster.cc), policy O4 [L]: rounds of T queries.  The round's searches run
     * against the index as it stood at the round's start (the worker threads), then the results are
     * analysed in order: a query whose k-mers reach minwordmatches (or all of its own) against a centroid
     * created earlier in the round gets that centroid inserted into its hit list by (count desc, shorter
     * target first; after equal ones), and the list is walked again from the top one alignment at a time
     * (accepts/rejects recounted; hits already aligned keep their results, new ones are aligned) until an
     * accept, maxrejects rejects or its end; the best hit is then chosen over every aligned hit. */
    const int cap = tophits + T;
    hit_t *bh = (hit_t *)calloc((size_t)T * 2 * (size_t)cap, sizeof(hit_t));
    int *bn = (int *)calloc((size_t)T * 2, sizeof(int));
    int32_t *extra = (int32_t *)malloc(sizeof(int32_t) * (size_t)T);
    uint32_t *ekm = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(maxl + 8));
    uint64_t *qset = (uint64_t *)calloc(((size_t)1 << (2 * p->wordlength)) / 64 + 1, 8);
    /* ORC_WORKERS=<n> (built with OpenMP): the round's searches on n worker threads, as vsearch's --threads
     * workers run them.  Results do not depend on n: every search reads only the index frozen at the round's
     * start, and the analysis below stays sequential.  Each worker has its own scratch and work counters. */
    int W = 1;
#ifdef _OPENMP
    const char *we = getenv("ORC_WORKERS");
    if (we && atoi(we) > 1) W = atoi(we) < T ? atoi(we) : T;
#endif
    uint32_t **wk_kbuf = (uint32_t **)malloc(sizeof(uint32_t *) * (size_t)W);
    int32_t **wk_counts = (int32_t **)malloc(sizeof(int32_t *) * (size_t)W);
    char **wk_rcq = (char **)malloc(sizeof(char *) * (size_t)W);
    for (int w = 0; w < W; w++) {
      wk_kbuf[w] = w ? (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(maxl + 8)) : kbuf;
      wk_counts[w] = w ? (int32_t *)malloc(sizeof(int32_t) * (size_t)(nk + 1)) : counts;
      wk_rcq[w] = w ? (char *)malloc((size_t)maxl + 2) : rcq;
    }
    for (int32_t b0 = 0; b0 < nk; b0 += T) {
      const int32_t nb = (nk - b0 < T) ? nk - b0 : T;
#ifdef _OPENMP
      #pragma omp parallel for num_threads(W) schedule(dynamic, 1) if (W > 1)
#endif
      for (int32_t i = 0; i < nb; i++) {
#ifdef _OPENMP
        const int w = omp_get_thread_num();
#else
        const int w = 0;
#endif
        ctx_t cw = c;  /* shares the frozen index; own work counters */
        cw.alignments = cw.cells = cw.postings = cw.candidates = 0;
        const int32_t s = b0 + i;
        bn[2 * i] = search_strand(&cw, p, c.seq[s], c.len[s], 0, wk_kbuf[w], wk_counts[w], bh + (size_t)(2 * i) * cap);
        if (wd) wd[2 * s] = (int16_t)cw.alignments;
        const int64_t a0 = cw.alignments;
        bn[2 * i + 1] = 0;
        if (p->strand_both) {
          revcomp(wk_rcq[w], c.seq[s], c.len[s]);
          bn[2 * i + 1] = search_strand(&cw, p, wk_rcq[w], c.len[s], 1, wk_kbuf[w], wk_counts[w],
                                        bh + (size_t)(2 * i + 1) * cap);
        }
        if (wd) wd[2 * s + 1] = (int16_t)(cw.alignments - a0);
#ifdef _OPENMP
        #pragma omp critical(orc_work)
#endif
        {
          c.alignments += cw.alignments;
          c.cells += cw.cells;
          c.postings += cw.postings;
          c.candidates += cw.candidates;
        }
      }
      int nextra = 0;
      for (int32_t i = 0; i < nb; i++) {
        const int32_t s = b0 + i;
        for (int st = 0; st < (p->strand_both ? 2 : 1) && nextra > 0; st++) {
          hit_t *h = bh + (size_t)(2 * i + st) * cap;
          int *nh = &bn[2 * i + st];
          const char *qs = c.seq[s];
          if (st) {
            revcomp(rcq, c.seq[s], c.len[s]);
            qs = rcq;
          }
          const int nq = orc_unique_kmers(qs, c.len[s], p->wordlength, p->qmask_dust, kbuf);
          for (int k = 0; k < nq; k++) qset[kbuf[k] >> 6] |= 1ULL << (kbuf[k] & 63);
          const int minmatches = p->minwordmatches < nq ? p->minwordmatches : nq;
          int added = 0;
          for (int j = 0; j < nextra; j++) {
            const int32_t e = extra[j];
            const int ne = orc_unique_kmers(c.seq[e], c.len[e], p->wordlength, p->qmask_dust, ekm);
            int shared = 0;
            for (int k = 0; k < ne; k++) shared += (int)((qset[ekm[k] >> 6] >> (ekm[k] & 63)) & 1ULL);
            if (shared < minmatches) continue;
            int x = *nh;
            while (x > 0 && (h[x - 1].count < shared ||
                             (h[x - 1].count == shared && c.len[h[x - 1].target] > c.len[e]))) {
              h[x] = h[x - 1];
              x--;
            }
            h[x].target = e;
            h[x].count = shared;
            h[x].accepted = 0;
            h[x].aligned = 0;
            h[x].id = 0.0;
            h[x].cigar = NULL;
            (*nh)++;
            added++;
          }
          for (int k = 0; k < nq; k++) qset[kbuf[k] >> 6] = 0;
          if (added) {
            int accepts = 0, rejects = 0;
            for (int t = 0; accepts < p->maxaccepts && rejects < p->maxrejects && t < *nh; t++) {
              if (!h[t].aligned && wd) wd[2 * s + st]++;
              if (!h[t].aligned) align_hit(&c, p, qs, c.len[s], &h[t]);
              if (h[t].accepted) accepts++;
              else rejects++;
            }
          }
        }
        hit_t *hpi = bh + (size_t)(2 * i) * cap, *hmi = bh + (size_t)(2 * i + 1) * cap;
        const int32_t before = clusters;
        ASSIGN(s, hpi, bn[2 * i], hmi, bn[2 * i + 1]);
        if (clusters > before) extra[nextra++] = s;
      }
    }
    for (int w = 1; w < W; w++) {
      free(wk_kbuf[w]);
      free(wk_counts[w]);
      free(wk_rcq[w]);
    }
    free(wk_kbuf);
    free(wk_counts);
    free(wk_rcq);
    free(qset);
    free(ekm);
    free(extra);
    free(bn);
    free(bh);
  }
  #undef ASSIGN
  if (wd) {
    FILE *wf = fopen(walk_dump, "wb");
    if (wf) {
      fwrite(wd, sizeof(int16_t), (size_t)nk * 2, wf);
      fclose(wf);
    }
    free(wd);
  }
  /* cluster sizes and output numbering (--clusterout_sort: size desc, creation order) */
  csz_t *cs = (csz_t *)calloc((size_t)clusters + 1, sizeof(csz_t));
  for (int32_t k = 0; k < clusters; k++) cs[k].cno = k;
  for (int32_t s = 0; s < nk; s++) cs[c.clusterno[s]].size++;
  if (p->clusterout_sort) qsort(cs, (size_t)clusters, sizeof(csz_t), csz_cmp);
  int32_t *rank = (int32_t *)malloc(sizeof(int32_t) * (size_t)(clusters + 1));
  for (int32_t k = 0; k < clusters; k++) rank[cs[k].cno] = k;
  /* members per output cluster, centroid first then sorted seqno order */
  int32_t *start = (int32_t *)calloc((size_t)clusters + 2, sizeof(int32_t));
  for (int32_t s = 0; s < nk; s++) start[rank[c.clusterno[s]] + 1]++;
  for (int32_t k = 0; k < clusters; k++) start[k + 1] += start[k];
  int32_t *fill = (int32_t *)malloc(sizeof(int32_t) * (size_t)(clusters + 1));
  memcpy(fill, start, sizeof(int32_t) * (size_t)(clusters + 1));
  int32_t *memb = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nk + 1));
  for (int32_t s = 0; s < nk; s++) memb[fill[rank[c.clusterno[s]]]++] = s;
  for (int32_t s = 0; s < nk; s++) {
    int32_t i = c.orig[s];
    out_cluster[i] = rank[c.clusterno[s]];
    out_strand[i] = c.strand[s];
  }
  int64_t off = 0;
  char *tmp = (char *)malloc((size_t)(4 * maxl + 16) * 2);
  for (int32_t k = 0; k < clusters; k++) {
    int32_t m = start[k + 1] - start[k];
    out_centroid[c.orig[memb[start[k]]]] = 1;
    int32_t *mb = memb + start[k];
    /* msa() can exceed 2*maxl columns only with deep insertions; size generously */
    int maxcols = c.len[mb[0]];
    for (int x = 1; x < m; x++) maxcols += c.len[mb[x]];
    char *cbuf = (maxcols + 1 > (4 * maxl + 16) * 2) ? (char *)malloc((size_t)maxcols + 1) : tmp;
    int64_t cl = msa_consensus(&c, mb, m, cbuf);
    if (cons_off) cons_off[k] = off;
    if (cons_buf) {
      if (off + cl > cons_cap) { off = -1; if (cbuf != tmp) free(cbuf); break; }
      memcpy(cons_buf + off, cbuf, (size_t)cl);
    }
    off += cl;
    if (cbuf != tmp) free(cbuf);
  }
  if (cons_off && off >= 0) cons_off[clusters] = off;
  if (stats) {
    stats[0] = nk;
    stats[1] = clusters;
    stats[2] = c.alignments;
    stats[3] = c.cells;
    stats[4] = c.postings;
    stats[5] = c.candidates;
    stats[6] = masked;
    stats[7] = 0;
  }
  free(tmp);
  free(memb);
  free(fill);
  free(start);
  free(rank);
  free(cs);
  free(rcq);
  free(hp);
  free(hm);
  free(counts);
  free(kbuf);
  for (int k = 0; k < K; k++) free(c.post[k]);
  free(c.post);
  free(c.post_n);
  free(c.post_cap);
  free(c.cent_seqno);
  for (int32_t s = 0; s < nk; s++) { free(c.seq[s]); free(c.cigar[s]); }
  free(c.seq);
  free(c.len);
  free(c.orig);
  free(c.clusterno);
  free(c.strand);
  free(c.cigar);
  if (off < 0) return -ENOSPC;
  return clusters;
}

/* ------------------------------------------------------------------ FASTA CLI path */
typedef struct {
  char **hdr;
  char **seq;
  int32_t *len;
  int32_t n, cap;
} fasta_t;

static int read_fasta(const char *path, fasta_t *f) {
  FILE *fp = fopen(path, "rb");
  if (!fp) return -errno;
  memset(f, 0, sizeof(*f));
  char *line = NULL;
  size_t lcap = 0;
  ssize_t ll;
  char *sbuf = NULL;
  size_t scap = 0, slen = 0;
  int have = 0;
  while ((ll = getline(&line, &lcap, fp)) >= 0) {
    while (ll > 0 && (line[ll - 1] == '\n' || line[ll - 1] == '\r')) line[--ll] = 0;
    if (line[0] == '>') {
      if (have) {
        f->seq[f->n - 1] = (char *)malloc(slen + 1);
        memcpy(f->seq[f->n - 1], sbuf, slen);
        f->seq[f->n - 1][slen] = 0;
        f->len[f->n - 1] = (int32_t)slen;
      }
      if (f->n == f->cap) {
        f->cap = f->cap ? 2 * f->cap : 1024;
        f->hdr = (char **)realloc(f->hdr, sizeof(char *) * (size_t)f->cap);
        f->seq = (char **)realloc(f->seq, sizeof(char *) * (size_t)f->cap);
        f->len = (int32_t *)realloc(f->len, sizeof(int32_t) * (size_t)f->cap);
      }
      /* label truncated at first whitespace (no --notrunclabels) */
      size_t hl = 0;
      while (line[1 + hl] && line[1 + hl] != ' ' && line[1 + hl] != '\t') hl++;
      f->hdr[f->n] = (char *)malloc(hl + 1);
      memcpy(f->hdr[f->n], line + 1, hl);
      f->hdr[f->n][hl] = 0;
      f->n++;
      have = 1;
      slen = 0;
    } else if (have) {
      for (ssize_t k = 0; k < ll; k++) {
        unsigned char ch = (unsigned char)line[k];
        if (!isalpha(ch)) continue;
        if (slen + 1 >= scap) { scap = scap ? 2 * scap : 256; sbuf = (char *)realloc(sbuf, scap); }
        sbuf[slen++] = (char)ch;
      }
    }
  }
  if (have) {
    f->seq[f->n - 1] = (char *)malloc(slen + 1);
    memcpy(f->seq[f->n - 1], sbuf ? sbuf : "", slen);
    f->seq[f->n - 1][slen] = 0;
    f->len[f->n - 1] = (int32_t)slen;
  }
  free(sbuf);
  free(line);
  fclose(fp);
  return 0;
}

static void print_wrapped(FILE *fp, const char *s, int64_t len, int width) {
  if (width <= 0) {
    fwrite(s, 1, (size_t)len, fp);
    fputc('\n', fp);
    return;
  }
  for (int64_t i = 0; i < len; i += width) {
    int64_t w = (len - i < width) ? len - i : width;
    fwrite(s + i, 1, (size_t)w, fp);
    fputc('\n', fp);
  }
  if (len == 0) fputc('\n', fp);
}

int64_t orc_run_fasta(const orc_params *p, const char *in_fasta, const char *clusters_prefix,
                      const char *consout, int64_t *stats) {
  init_maps();
  fasta_t f;
  memset(&f, 0, sizeof(f));
  int rc = read_fasta(in_fasta, &f);
  if (rc) return rc;
  int32_t n = f.n;
  int32_t *ocl = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n + 1));
  uint8_t *ost = (uint8_t *)malloc((size_t)n + 1);
  uint8_t *oce = (uint8_t *)malloc((size_t)n + 1);
  int32_t *osr = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n + 1));
  int64_t cap = 0;
  for (int32_t i = 0; i < n; i++) cap += 2 * (int64_t)f.len[i] + 2;
  char *cbuf = (char *)malloc((size_t)cap + 1);
  int64_t *coff = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 2));
  int64_t st[8];
  int64_t k = orc_cluster(p, n, (const char *const *)f.seq, f.len, ocl, ost, oce, osr, cbuf, cap,
                          coff, st);
  if (stats) memcpy(stats, st, sizeof(st));
  if (k >= 0) {
    /* masked sequences are what vsearch prints; recompute the masks here */
    int32_t nkeep = (int32_t)st[0];
    /* members of each output cluster in sorted order: centroid first */
    int32_t *cnt = (int32_t *)calloc((size_t)k + 2, sizeof(int32_t));
    for (int32_t s = 0; s < nkeep; s++) cnt[ocl[osr[s]] + 1]++;
    for (int64_t c = 0; c < k; c++) cnt[c + 1] += cnt[c];
    int32_t *memb = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nkeep + 1));
    int32_t *fill = (int32_t *)malloc(sizeof(int32_t) * (size_t)(k + 1));
    memcpy(fill, cnt, sizeof(int32_t) * (size_t)(k + 1));
    for (int32_t s = 0; s < nkeep; s++) memb[fill[ocl[osr[s]]]++] = osr[s];
    FILE *fc = consout ? fopen(consout, "w") : NULL;
    size_t plen = clusters_prefix ? strlen(clusters_prefix) : 0;
    char *fn = (char *)malloc(plen + 32);
    char *mbuf = (char *)malloc(1024);
    int mcap = 1024;
    for (int64_t c = 0; c < k; c++) {
      int32_t cent = memb[cnt[c]];
      if (fc) {
        fprintf(fc, ">centroid=%s;seqs=%d", f.hdr[cent], cnt[c + 1] - cnt[c]);
        if (p->clusterout_id) fprintf(fc, ";clusterid=%lld", (long long)c);
        fputc('\n', fc);
        print_wrapped(fc, cbuf + coff[c], coff[c + 1] - coff[c], p->fasta_width);
      }
      if (clusters_prefix) {
        sprintf(fn, "%s%lld", clusters_prefix, (long long)c);
        FILE *fo = fopen(fn, "w");
        if (!fo) { rc = -errno; break; }
        for (int32_t x = cnt[c]; x < cnt[c + 1]; x++) {
          int32_t i = memb[x];
          if (f.len[i] + 1 > mcap) { mcap = f.len[i] + 1; mbuf = (char *)realloc(mbuf, (size_t)mcap); }
          memcpy(mbuf, f.seq[i], (size_t)f.len[i]);
          if (p->qmask_dust) orc_dust(mbuf, f.len[i]);
          fprintf(fo, ">%s\n", f.hdr[i]);
          print_wrapped(fo, mbuf, f.len[i], p->fasta_width);
        }
        fclose(fo);
      }
    }
    if (fc) fclose(fc);
    free(mbuf);
    free(fn);
    free(fill);
    free(memb);
    free(cnt);
  }
  for (int32_t i = 0; i < n; i++) { free(f.hdr[i]); free(f.seq[i]); }
  free(f.hdr);
  free(f.seq);
  free(f.len);
  free(ocl);
  free(ost);
  free(oce);
  free(osr);
  free(cbuf);
  free(coff);
  return rc ? rc : k;
}
