// align_kernels.h -- the per-query-length alignment kernel templates (K3 k_align, K3P k_align_pk,
// K3T k_traceback).  Rows are unrolled per query length, so every length is its own instantiation;
// the instantiations are split over several translation units (align_inst.hip, one per length range,
// built in parallel) that each fill their slice of the launch tables in kernels.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "umiclust_internal.h"

namespace uc {

// ------------------------------------------------------------------ K3: alignment (stats)
__device__ __forceinline__ int sx16(uint32_t v) { return (int)(int16_t)(v & 0xffffu); }
__device__ __forceinline__ uint32_t pack_hf(int h, int f) {
  return ((uint32_t)f << 16) | ((uint32_t)h & 0xffffu);
}

constexpr int kNegInf = -16000;  // below any reachable score (|score| <= kMaxLen*40 + gaps)

// Query rows are unrolled: QL is a compile-time constant (the driver cuts greedy blocks at length
// changes, so every pair of a launch has the same query length) and the per-row state lives in
// VGPRs with compile-time indices.  Target columns run as a runtime loop (lanes may have different
// target lengths); the target's last column takes the target-right gap penalties (one select per
// column, shared by all rows).
//
// Forward-carried traceback (no direction matrix).  vsearch's acceptance needs, along the path
// backtrack16 picks, the matches m and internal_len = columns - leading gap run - trailing gap run
// (align_trim).  For every real DP cell the leading CIGAR run is exactly the boundary run (row -1
// or column -1) the path starts with, so columns - leading run = the number of moves INTO real
// cells, a.  Each DP state carries the summary a | m << 8 of the path the traceback would follow
// from it (boundary states carry 0), selected with backtrack16's strict priorities
// (diagonal > up/D > left/I; a gap extends only if strictly better than reopening).
// The trailing gap run is backtrack16's first run from the end cell (last row, last column):
//  * an I run walks left along the last row; with Lext(j) = run length when arriving at column j in
//    an I run: Lh(j) = left(j) ? 1 + Lext(j-1) : 0, Lext(j) = extleft(j) ? 1 + Lext(j-1) : Lh(j);
//  * a D run walks up the last column: the F state's summary carries the length of its trailing D
//    run in bits 16-23 (opening from H inherits H's run, so consecutive D runs merge exactly as
//    CIGAR runs do); H inherits it only when it takes F.
// Per row: HE[i] = H(i, j-1) | E(i, j) << 16 and SS[i] = S_H(i, j-1) | S_E(i, j) << 16, 16 bits each.
template <int QL, bool AMB>
__device__ __forceinline__ void align_column(uint32_t (&HE)[QL], uint32_t (&SS)[QL],
                                             const uint32_t (&qw)[(QL + 7) / 8], uint32_t tcode,
                                             int j, const Scoring& sc, int QRt, int Rt, int& Lext,
                                             int& trail) {
  const int QRqi = sc.go[2] + sc.ge[2], Rqi = sc.ge[2];
  const int QRqr = sc.go[4] + sc.ge[4], Rqr = sc.ge[4];
  const bool tamb = AMB && ((tcode & (tcode - 1u)) != 0u || tcode == 0u);
  // row -1 of this column: H(-1, j-1) (diagonal of row 0) and F(0, j); boundary summaries are 0
  int Hd = (j == 0) ? 0 : -(sc.go[0] + j * sc.ge[0]);
  uint32_t SHd = 0;
  int F = sc.boundary_open ? -(sc.go[0] + (j + 1) * sc.ge[0]) - QRt : kNegInf;
  uint32_t SF = 0x10001u;  // one real D move, trailing D run 1
#pragma unroll
  for (int i = 0; i < QL; i++) {
    const uint32_t qcode = (qw[i >> 3] >> ((i & 7) * 4)) & 15u;
    int sub;
    uint32_t e;
    if (AMB) {
      // IUPAC: any ambiguous symbol scores 0; a match is a non-empty code intersection
      const bool amb = tamb || (qcode & (qcode - 1u)) != 0u || qcode == 0u;
      sub = amb ? 0 : (qcode == tcode ? sc.match : sc.mismatch);
      e = (qcode & tcode) ? (1u << 8) : 0u;
    } else {
      const bool eq = qcode == tcode;
      sub = eq ? sc.match : sc.mismatch;
      e = eq ? (1u << 8) : 0u;
    }
    const uint32_t he = HE[i];
    const uint32_t ss = SS[i];
    const int Hl = sx16(he);
    const int E = (int)he >> 16;
    const uint32_t SE = ss >> 16;
    int h = Hd + sub;
    uint32_t sh = SHd + 1u + e;
    const bool fb = F > h;  // up: D chosen
    h = fb ? F : h;
    sh = fb ? SF : sh;
    const bool eb = E > h;  // left: I chosen
    h = eb ? E : h;
    sh = eb ? SE : sh;
    const int fo = h - QRt, fe = F - Rt;
    const bool fx = fe > fo;  // extup
    SF = (fx ? SF : sh) + 0x10001u;
    const int qrq = (i == QL - 1) ? QRqr : QRqi;
    const int rq = (i == QL - 1) ? Rqr : Rqi;
    const int eo = h - qrq, ee = E - rq;
    const bool ex = ee > eo;  // extleft
    const uint32_t sen = (ex ? SE : sh) + 1u;
    if (i == QL - 1) {
      // last row: I-run counters; the value left by the last column is the end cell's
      const int lh = eb ? 1 + Lext : 0;
      Lext = ex ? 1 + Lext : lh;
      trail = eb ? lh : (int)(sh >> 16);
    }
    F = fx ? fe : fo;
    Hd = Hl;
    SHd = ss & 0xffffu;
    // materialise the next row's diagonal now: otherwise SDWA folding reads the old packed words
    // in row i+1, both generations stay live and every column ends in a 2*QL-register copy
    asm volatile("" : "+v"(Hd), "+v"(SHd));
    HE[i] = pack_hf(h, ex ? ee : eo);
    SS[i] = (sh & 0xffffu) | (sen << 16);
  }
}

template <int QL, bool AMB>
__global__ __launch_bounds__(64) void k_align(DevSeqs s, const uint32_t* __restrict__ pq,
                                              const uint32_t* __restrict__ pt, int32_t npairs,
                                              const uint32_t* __restrict__ dev_npairs,
                                              const uint32_t* __restrict__ outidx, Scoring sc,
                                              uint32_t* __restrict__ out) {
  constexpr int CW = (QL + 7) / 8;
  if (sc.wave_prio) __builtin_amdgcn_s_setprio(3);
  const int k = blockIdx.x * 64 + threadIdx.x;
  if (k >= npairs) return;
  if (dev_npairs && k >= (int)*dev_npairs) return;
  const uint32_t qv = pq[k];
  const int32_t q = (int32_t)(qv >> 1);
  const int qstr = (int)(qv & 1u);
  const int32_t t = (int32_t)pt[k];
  const int tl = s.lens[t];
  uint32_t qw[CW];
#pragma unroll
  for (int w = 0; w < CW; w++) qw[w] = s.codes[((int64_t)q * 2 + qstr) * kCodeWords + w];
  const uint32_t* tcp = s.codes + (int64_t)t * 2 * kCodeWords;
  const int QRti = sc.go[3] + sc.ge[3], Rti = sc.ge[3];
  const int QRtr = sc.go[5] + sc.ge[5], Rtr = sc.ge[5];
  uint32_t HE[QL], SS[QL];
  {
    // boundary column -1: H(i,-1) = -(GO_TL + (i+1) GE_TL), E(i,0) opened from it; built
    // incrementally in VGPRs (an opaque zero keeps the compiler from materialising 2*QL scalars)
    int vz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
    int hleft = vz - sc.go[1];
    const int QRqi = sc.go[2] + sc.ge[2], QRqr = sc.go[4] + sc.ge[4];
#pragma unroll
    for (int i = 0; i < QL; i++) {
      hleft -= sc.ge[1];
      const int qrq = (i == QL - 1) ? QRqr : QRqi;
      HE[i] = pack_hf(hleft, sc.boundary_open ? hleft - qrq : kNegInf);
      SS[i] = 1u << 16;  // S_H(i,-1) = 0 (boundary), S_E(i,0) = one real move
    }
  }
  int Lext = 0, trail = 0;
  uint32_t tword = 0;
  for (int j = 0; j < tl; j++) {
    if ((j & 7) == 0) tword = tcp[j >> 3];
    const uint32_t tcode = tword & 15u;
    tword >>= 4;
    // keep the per-row query codes from being hoisted out of the column loop (that would pin
    // QL extra VGPRs); re-extracting them is one v_bfe per cell
#pragma unroll
    for (int w = 0; w < CW; w++) asm volatile("" : "+v"(qw[w]));
    const bool lc = (j == tl - 1);
    align_column<QL, AMB>(HE, SS, qw, tcode, j, sc, lc ? QRtr : QRti, lc ? Rtr : Rti, Lext, trail);
  }
  const int H = sx16(HE[QL - 1]);
  const uint32_t S = SS[QL - 1] & 0xffffu;
  const uint32_t m = S >> 8, acols = S & 0xffu;
  const uint32_t internal = acols - (uint32_t)trail;
  out[outidx ? outidx[k] : (uint32_t)k] = m | (internal << 8) | (((uint32_t)H & 0xffffu) << 16);
}

// ------------------------------------------------------------------ K3P: packed 16-bit alignment
// The same recurrences, summaries and strict priorities as k_align, two DP cells per 32-bit VALU
// op (VOP3P v_pk_* on int16 halves).  A column is split into a top half (rows [0, TOP)) and a
// bottom half (rows [TOP, QL)) that runs one column behind: register k holds row k of column j in
// its low half and row TOP+k of column j-1 in its high half.  Within a step the rows are
// processed in order, so the bottom half's upper neighbour (row TOP-1 of column j-1) is the top
// half's carry-out of the previous step; one step costs one pass over TOP packed rows.
// Branch-free selection: for |values| well inside int16, (a - b) >> 15 (arithmetic, per half) is
// the mask of "b > a", which drives v_bfi for the summaries and v_pk_max for the scores.
// Substitution: per 16-row group a match bit-mask of the column's target base, selected per step
// from per-base masks built once per pair (non-ambiguous sequences only: one-hot codes; k_align_pk
// keeps them in lane-private LDS, k_align_band in VGPRs).
typedef short v2s __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2s as_v2(uint32_t x) { return __builtin_bit_cast(v2s, x); }
__device__ __forceinline__ uint32_t as_u(v2s x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }
__device__ __forceinline__ uint32_t pk2(int lo, int hi) { return ((uint32_t)hi << 16) | ((uint32_t)lo & 0xffffu); }
// mask of (b > a) per half
// (opaque to the compiler, which otherwise rewrites it into per-half compares and selects)
__device__ __forceinline__ uint32_t gt_mask(v2s b, v2s a) {
  uint32_t d;
  // op_sel_hi:[0,1]: the inline constant's low half serves both halves (its high half is 0)
  asm("v_pk_sub_i16 %0, %1, %2\n\tv_pk_ashrrev_i16 %0, 15, %0 op_sel_hi:[0,1]" : "=&v"(d) : "v"(a), "v"(b));
  return d;
}

// Cheaper cells than a literal restatement of the recurrences (24 VALU ops per packed cell pair):
//  * row potential: the kernel works on H'(i,j) = H(i,j) - X (i+1) with X the mismatch score (E and
//    F shifted alike).  Every comparison is between states of one cell, so the offset changes no
//    decision; a diagonal step becomes H'd + e DELTA (no mismatch add) and a vertical step costs
//    X more (folded into the F gap constants).  The end score adds X QL back.
//  * summaries count matches m (bits 0-7) and u + 1 (bits 8-15), with u = the boundary index the
//    path starts from (row r of column -1, or column c of row -1; the corner is u = -1) plus its
//    diagonal moves.  Moves into real cells are a = i + j + 2 - (u + 1): a gap move changes
//    neither field, a diagonal move adds e + 0x100, so the summaries need no per-cell increments.
//  * the trailing-D-run tracker (the D run length of the F state; H inherits it when it takes F)
//    only matters in the end cell's column, i.e. in the last two steps; the main loop runs without it.
//  * each row's diagonal candidate is formed from the previous row's old H / S_H before that row
//    overwrites them, so the register rotation needs no copies.
//  * the boundary initialisation is an inlined function, not a lambda captured by the step lambda
//    (that closure kept the row arrays in scratch).

// k_align_pk's boundary column -1: H'(i,-1) = -(GO_TL + (i+1) GE_TL) - X (i+1), E'(i,0) opened
// from it; summaries u + 1 = i + 1, no matches; keep_mask selects the halves to (re)initialise.  X is the row
// potential's coefficient (k_align_pk: mismatch + Bq, k_align_band: mismatch) and QRqi / QRqr the E openings in
// the caller's frame.
template <int QL, int TOP>
__device__ __forceinline__ void pk_init_rows(v2s (&H)[TOP], v2s (&E)[TOP], uint32_t (&SH)[TOP],
                                             uint32_t (&SE)[TOP], uint32_t keep_mask,
                                             const Scoring& sc, int X, int QRqi, int QRqr) {
  int vz;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
#pragma unroll
  for (int kk = 0; kk < TOP; kk++) {
    const int i0 = kk, i1 = TOP + kk;
    const int h0 = vz - sc.go[1] - (i0 + 1) * (sc.ge[1] + X);
    const int h1 = vz - sc.go[1] - (i1 + 1) * (sc.ge[1] + X);
    const int q1 = (i1 == QL - 1) ? QRqr : QRqi;
    const int e0 = sc.boundary_open ? h0 - QRqi : kNegInf;
    const int e1 = sc.boundary_open ? h1 - q1 : kNegInf;
    const uint32_t s01 = pk2((i0 + 1) << 8, (i1 + 1) << 8);
    H[kk] = as_v2(bfi(keep_mask, pk2(h0, h1), as_u(H[kk])));
    E[kk] = as_v2(bfi(keep_mask, pk2(e0, e1), as_u(E[kk])));
    SH[kk] = bfi(keep_mask, s01, SH[kk]);
    SE[kk] = bfi(keep_mask, s01, SE[kk]);
  }
}

template <bool B> struct BTag { static constexpr bool value = B; };

// one pair per lane (k_align_pk below loops a wave over its pairs)
template <int QL>
__device__ __forceinline__ void align_pk_pair(const DevSeqs& s, const uint32_t* __restrict__ pq,
                                              const uint32_t* __restrict__ pt, int k,
                                              const uint32_t* __restrict__ outidx, const Scoring& sc,
                                              uint32_t* __restrict__ out, uint16_t* sM) {
  constexpr int TOP = (QL + 1) / 2, BOT = QL - TOP;  // BOT == TOP or TOP - 1
  constexpr int NG = (TOP + 15) / 16;
  constexpr int KL = BOT - 1;                        // register holding row QL-1 (high half)
  const uint32_t qv = pq[k];
  const int32_t q = (int32_t)(qv >> 1);
  const int qstr = (int)(qv & 1u);
  const int32_t t = (int32_t)pt[k];
  const int tl = s.lens[t];
  // per-base row masks: MT[g] / MB[g] hold, for base b at bits [16b, 16b+16), the rows of group g
  // (top half / bottom half) whose query base is b
  uint64_t MT[NG], MB[NG];
#pragma unroll
  for (int g = 0; g < NG; g++) MT[g] = MB[g] = 0;
  {
    const uint32_t* qc = s.codes + ((int64_t)q * 2 + qstr) * kCodeWords;
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < QL; i++) {
      if ((i & 7) == 0) w = qc[i >> 3];
      const uint32_t b = (uint32_t)__builtin_ctz((w & 15u) | 16u) & 3u;
      w >>= 4;
      if (i < TOP) MT[i >> 4] |= 1ull << (16 * b + (i & 15));
      else MB[(i - TOP) >> 4] |= 1ull << (16 * b + ((i - TOP) & 15));
    }
  }
  // the per-base row masks move to LDS (lane-private, [base][group][half][lane] u16): two 16-bit reads
  // per group and column instead of 4 NG live VGPRs and the 64-bit shifts
  uint16_t* const pM = sM + threadIdx.x;
#pragma unroll
  for (int b = 0; b < 4; b++)
#pragma unroll
    for (int g = 0; g < NG; g++) {
      pM[((b * NG + g) * 2 + 0) * 64] = (uint16_t)(MT[g] >> (16 * b));
      pM[((b * NG + g) * 2 + 1) * 64] = (uint16_t)(MB[g] >> (16 * b));
    }
  const uint32_t* tcp = s.codes + (int64_t)t * 2 * kCodeWords;
  // potentials (round 6): the kernel works on H''(i,j) = H(i,j) - (X + Bq)(i+1) + Bq (j+1), E and F alike.  Every
  // comparison is between states of one cell, so no decision changes; a diagonal step is H'' + e DELTA (the row term
  // -(X + Bq) and the column term Bq cancel the mismatch score), an interior horizontal gap extension (E) costs
  // nothing (Bq = its penalty: one v_pk_sub_i16 less per packed row), a vertical step costs X + Bq more (folded into
  // the F constants) and an E opening Bq less; the end score takes the potentials back off.
  const int X = sc.mismatch, Bq = sc.ge[2];
  const int QRti = sc.go[3] + sc.ge[3] + X + Bq, Rti = sc.ge[3] + X + Bq;  // vertical gaps
  const int QRtr = sc.go[5] + sc.ge[5] + X + Bq, Rtr = sc.ge[5] + X + Bq;
  const int QRqi = sc.go[2] + sc.ge[2] - Bq;  // horizontal openings; interior extension 0
  const int QRqr = sc.go[4] + sc.ge[4] - Bq, Rqr = sc.ge[4] - Bq;  // last row (the query's right end)
  const v2s DELTA = as_v2(pk2(sc.match - sc.mismatch, sc.match - sc.mismatch));
  v2s H[TOP], E[TOP];
  uint32_t SH[TOP], SE[TOP];
#pragma unroll
  for (int kk = 0; kk < TOP; kk++) {
    H[kk] = as_v2(0u);
    E[kk] = as_v2(0u);
    SH[kk] = SE[kk] = 0;
  }
  pk_init_rows<QL, TOP>(H, E, SH, SE, 0xffffffffu, sc, X + Bq, QRqi, QRqr);
  // carries of the top half's last row, consumed by the bottom half in the next step
  uint32_t cHd = 0, cSHd = 0, cF = 0, cSF = 0, cDL = 0;
  int Lext = 0, trail = 0;
  // the target's code words one ahead (the load of word w + 1 is in flight while word w's 8 columns run; a
  // load at its use cost every wave a full memory wait per 8 columns).  Word w + 1 may lie past the target's
  // words: it is then the other strand's first word (same row of the codes array), never used.
  uint32_t tword = 0, tprev = 1, tnext = tcp[0];
  // one step: top half at column j, bottom half at column j-1; LAST: one of the end cell's two steps
  auto step = [&](int j, auto last_tag) __attribute__((always_inline)) {
    constexpr bool LAST = decltype(last_tag)::value;
    if ((j & 7) == 0) {
      tword = tnext;
      tnext = tcp[(j >> 3) + 1];
    }
    const uint32_t tcode = tword & 15u;
    tword >>= 4;
    const uint32_t bl = (uint32_t)__builtin_ctz(tcode | 16u) & 3u, bh = (uint32_t)__builtin_ctz(tprev | 16u) & 3u;
    tprev = tcode;
    uint32_t M[NG];
#pragma unroll
    for (int g = 0; g < NG; g++)
      M[g] = (uint32_t)pM[((bl * NG + g) * 2 + 0) * 64] | ((uint32_t)pM[((bh * NG + g) * 2 + 1) * 64] << 16);
    const bool lc0 = LAST && (j == tl - 1), lc1 = LAST && (j == tl);
    const uint32_t QRt = LAST ? pk2(lc0 ? QRtr : QRti, lc1 ? QRtr : QRti) : pk2(QRti, QRti);
    const uint32_t Rt = LAST ? pk2(lc0 ? Rtr : Rti, lc1 ? Rtr : Rti) : pk2(Rti, Rti);
    // row -1 (top half, column j: potential Bq j for H(-1, j-1), Bq (j + 1) for F(0, j)) | carry (bottom half)
    const int hd0 = ((j == 0) ? 0 : -(sc.go[0] + j * sc.ge[0])) + Bq * j;
    const int f0 = sc.boundary_open ? -(sc.go[0] + (j + 1) * sc.ge[0]) - (lc0 ? QRtr : QRti) + Bq * (j + 1) : kNegInf;
    v2s Hd = as_v2(pk2(hd0, (int)cHd));
    uint32_t SHd = pk2(j << 8, (int)cSHd);  // H(-1, j-1): u = j - 1
    v2s F = as_v2(pk2(f0, (int)cF));
    uint32_t SF = pk2((j + 1) << 8, (int)cSF);  // F(0, j) opened from H(-1, j): u = j
    uint32_t DL = pk2(1, (int)cDL);             // D run of the F state (F(0, j): one move)
    // each row's diagonal candidate is formed from the previous row's old H / S_H before that row
    // overwrites them (no register copies for the rotation)
    uint32_t e = M[0] & 0x00010001u;
    v2s hn = as_v2(e) * DELTA + Hd;
    uint32_t shn = SHd + e + 0x01000100u;
#pragma unroll
    for (int kk = 0; kk < TOP; kk++) {
      v2s h = hn;
      uint32_t sh = shn;
      if (kk + 1 < TOP) {
        e = (M[(kk + 1) >> 4] >> ((kk + 1) & 15)) & 0x00010001u;
        hn = as_v2(e) * DELTA + H[kk];
        shn = SH[kk] + e + 0x01000100u;
      } else {
        Hd = H[kk];
        SHd = SH[kk];
      }
      const uint32_t mF = gt_mask(F, h);
      h = __builtin_elementwise_max(h, F);
      sh = bfi(mF, SF, sh);
      const v2s Ec = E[kk];
      const uint32_t mE = gt_mask(Ec, h);
      h = __builtin_elementwise_max(h, Ec);
      sh = bfi(mE, SE[kk], sh);
      int dr_last = 0;
      bool eb_last = false;
      if (kk == KL) {
        eb_last = (mE >> 31) != 0;
        // last row (high half): D run of the chosen F = rows since it opened (before DF moves on)
        if (LAST) dr_last = (mF >> 31) != 0 ? (int)(DL >> 16) : 0;
      }
      const v2s fo = h - as_v2(QRt), fe = F - as_v2(Rt);
      const uint32_t mfx = gt_mask(fe, fo);
      F = __builtin_elementwise_max(fo, fe);
      // a new D run opened from H continues H's own D run when H took F
      if (LAST) {
        // extended, or opened from an H that took F (continuing H's run): one more; else a new run of 1
        DL = bfi(mfx | (mF & ~mE), DL + 0x00010001u, 0x00010001u);
        asm volatile("" : "+v"(DL));  // keep the tracker in its row (sinking it keeps 3 masks per row live)
      }
      SF = bfi(mfx, SF, sh);
      const uint32_t qrq = pk2(QRqi, (TOP + kk == QL - 1) ? QRqr : QRqi);
      // interior rows extend E for free; the last row (high half of register KL) pays its terminal extension
      const v2s eo = h - as_v2(qrq), ee = (TOP + kk == QL - 1) ? Ec - as_v2(pk2(0, Rqr)) : Ec;
      const uint32_t mex = gt_mask(ee, eo);
      if (kk == KL) {
        // trailing I-run counters along the last row; the value left by the last column is the
        // end cell's (vsearch align_trim's trailing run)
        const bool ex = (mex >> 31) != 0;
        const int lh = eb_last ? 1 + Lext : 0;
        if (LAST) trail = eb_last ? lh : dr_last;
        Lext = ex ? 1 + Lext : lh;
      }
      E[kk] = __builtin_elementwise_max(eo, ee);
      SE[kk] = bfi(mex, SE[kk], sh);
      H[kk] = h;
      SH[kk] = sh;
    }
    // carry the top half's outputs into the bottom half of the next step
    cHd = as_u(Hd) & 0xffffu;
    cSHd = SHd & 0xffffu;
    cF = as_u(F) & 0xffffu;
    cSF = SF & 0xffffu;
    if (LAST) cDL = DL & 0xffffu;
  };
  // the bottom half processes column -1 in step 0: the boundary column is restored after it
  int j = 0;
  for (; j < tl - 1; j++) {
    step(j, BTag<false>{});
    if (j == 0) {
      pk_init_rows<QL, TOP>(H, E, SH, SE, 0xffff0000u, sc, X + Bq, QRqi, QRqr);
      Lext = 0;
      trail = 0;
    }
  }
  for (; j <= tl; j++) {
    step(j, BTag<true>{});
    if (j == 0) {
      pk_init_rows<QL, TOP>(H, E, SH, SE, 0xffff0000u, sc, X + Bq, QRqi, QRqr);
      Lext = 0;
      trail = 0;
    }
  }
  const int Hend = (int)(short)(as_u(H[KL]) >> 16) + (X + Bq) * QL - Bq * tl;
  const uint32_t S = (SH[KL] >> 16) & 0xffffu;
  const uint32_t m = S & 0xffu;
  const uint32_t acols = (uint32_t)(QL + tl) - (S >> 8);
  const uint32_t internal = acols - (uint32_t)trail;
  out[outidx ? outidx[k] : (uint32_t)k] = m | (internal << 8) | (((uint32_t)Hend & 0xffffu) << 16);
}

// A wave loops over pairs k0 + lane, k0 += 64 x grid: the launch may hold fewer waves than pairs / 64
// (launch_align's UMICLUST_AL_WAVES cap), so that alignment waves leave VGPRs for the counting kernel's waves
// instead of filling every SIMD (166 VGPRs x 3 waves) while a launch is in flight.
template <int QL>
__global__ __launch_bounds__(64) void k_align_pk(DevSeqs s, const uint32_t* __restrict__ pq,
                                                 const uint32_t* __restrict__ pt, int32_t npairs,
                                                 const uint32_t* __restrict__ dev_npairs,
                                                 const uint32_t* __restrict__ outidx, Scoring sc,
                                                 uint32_t* __restrict__ out) {
  constexpr int NG = ((QL + 1) / 2 + 15) / 16;
  __shared__ uint16_t sM[4 * NG * 2 * 64];
  if (sc.wave_prio) __builtin_amdgcn_s_setprio(3);
  const int n = dev_npairs ? min(npairs, (int)*dev_npairs) : npairs;
  for (int k0 = (int)blockIdx.x * 64; k0 < n; k0 += (int)gridDim.x * 64) {  // wave-uniform
    const int k = k0 + (int)threadIdx.x;
    if (k < n) align_pk_pair<QL>(s, pq, pt, k, outidx, sc, out, sM);
  }
}

// ------------------------------------------------------------------ K3B: banded packed alignment
// k_align_pk's recurrences, summaries and strict priorities with one pair spread over a group of G lanes
// (inside one 16-lane DPP row), for launches too small to fill the GPU with one lane per pair: deep
// clusters cut greedy blocks to a few hundred query-strands, ~10k pairs = 150 waves for 1,024 SIMDs, each
// wave bound by one alignment's QL x TL cells in series.  Lane g of a group holds the B = ceil(QL / G)
// query rows [g B - P, (g + 1) B - P) as k_align_pk's top and bottom halves.  The P = G B - QL virtual
// rows on top of lane 0 end in one forced to the boundary row -1, so the last lane ends exactly at row
// QL - 1 and its last-row penalties and trailing-run counters stay compile-time rows.  Lane g runs two
// columns behind lane g - 1 and takes, by DPP row_shr:1, the carries lane g - 1's last row left in the
// previous step (the role k_align_pk's top-to-bottom carries play inside a lane): TL + 2G - 1 steps of
// B / 2 packed rows per pair.
constexpr int band_lanes(int ql) { return ql >= 57 ? 8 : 4; }  // keeps P < B (virtual rows in lane 0)

__device__ __forceinline__ uint32_t row_shr1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
}

template <int QL, int G>
__global__ __launch_bounds__(64) void k_align_band(DevSeqs s, const uint32_t* __restrict__ pq,
                                                   const uint32_t* __restrict__ pt, int32_t npairs,
                                                   const uint32_t* __restrict__ dev_npairs,
                                                   const uint32_t* __restrict__ outidx, Scoring sc,
                                                   uint32_t* __restrict__ out) {
  constexpr int B = (QL + G - 1) / G;
  constexpr int P = G * B - QL;  // virtual rows on top of lane 0
  constexpr int TOP = (B + 1) / 2, BOT = B - TOP;
  constexpr int NG = (TOP + 15) / 16;
  constexpr int KL = BOT - 1;                              // register holding the lane's last row (high half)
  constexpr int VR = P - 1;                                // lane 0's local row standing for row -1
  constexpr int VK = VR < TOP ? VR : VR - TOP;             // its register
  constexpr uint32_t VM = VR < TOP ? 0x0000ffffu : 0xffff0000u;  // and half
  static_assert(16 % G == 0 && P < B && BOT >= 1, "band layout");
  if (sc.wave_prio) __builtin_amdgcn_s_setprio(3);
  const int gid = (int)(blockIdx.x * 64 + threadIdx.x);
  const int k = gid / G, g = gid % G;
  if (k >= npairs) return;  // group-uniform
  if (dev_npairs && k >= (int)*dev_npairs) return;
  const bool first = g == 0, last = g == G - 1;
  const uint32_t fm = first ? 0xffffffffu : 0u;
  const int r0 = g * B - P;  // global row of local row 0
  const uint32_t qv = pq[k];
  const int32_t q = (int32_t)(qv >> 1);
  const int qstr = (int)(qv & 1u);
  const int32_t t = (int32_t)pt[k];
  const int tl = s.lens[t];
  uint64_t MT[NG], MB[NG];
#pragma unroll
  for (int gg = 0; gg < NG; gg++) MT[gg] = MB[gg] = 0;
  {
    const uint32_t* qc = s.codes + ((int64_t)q * 2 + qstr) * kCodeWords;
#pragma unroll
    for (int i = 0; i < B; i++) {
      const int r = r0 + i;
      const int rc = r < 0 ? 0 : r;  // virtual rows read row 0's word (never before the sequence)
      const uint32_t w = qc[rc >> 3] >> ((rc & 7) * 4);
      const uint64_t bit = r >= 0 ? 1ull : 0ull;
      const uint32_t b = (uint32_t)__builtin_ctz((w & 15u) | 16u) & 3u;
      if (i < TOP) MT[i >> 4] |= bit << (16 * b + (i & 15));
      else MB[(i - TOP) >> 4] |= bit << (16 * b + ((i - TOP) & 15));
    }
  }
  const uint32_t* tcp = s.codes + (int64_t)t * 2 * kCodeWords;
  // k_align_pk's potentials: H'' = H - (X + Bq)(global row + 1) + Bq (column + 1), so an interior E extension is free
  const int X = sc.mismatch, Bq = sc.ge[2];
  const int QRti = sc.go[3] + sc.ge[3] + X + Bq, Rti = sc.ge[3] + X + Bq;
  const int QRtr = sc.go[5] + sc.ge[5] + X + Bq, Rtr = sc.ge[5] + X + Bq;
  const int QRqi = sc.go[2] + sc.ge[2] - Bq;
  const int QRqr = sc.go[4] + sc.ge[4] - Bq, Rqr = sc.ge[4] - Bq;
  const v2s DELTA = as_v2(pk2(sc.match - sc.mismatch, sc.match - sc.mismatch));
  const uint32_t qrqL = pk2(QRqi, last ? QRqr : QRqi), rqL = pk2(0, last ? Rqr : 0);
  v2s H[TOP], E[TOP];
  // summaries: k_align_pk's m | (u + 1) << 8 with u biased by kSB (> the virtual rows' depth P - 1, so the
  // virtual rows' start values are not negative either)
  constexpr int kSB = 8;
  static_assert(P <= kSB, "summary bias");
  uint32_t SH[TOP], SE[TOP];
  auto init_rows = [&](uint32_t keep_mask) {
    // boundary column -1 (k_align_pk's pk_init_rows at global rows); lane 0's row -1 stand-in holds
    // H(-1,-1) = 0 and the corner's summary (u + 1 = 0).  The opaque zero keeps the loop-invariant row
    // values from being hoisted into 2 TOP live VGPRs.
    int vz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
    const int hbase = vz - sc.go[1] - (r0 + 1) * (sc.ge[1] + X + Bq);
    const uint32_t sbase = (uint32_t)vz + pk2((r0 + 1 + kSB) << 8, (r0 + TOP + 1 + kSB) << 8);
#pragma unroll
    for (int kk = 0; kk < TOP; kk++) {
      const int h0 = hbase - kk * (sc.ge[1] + X + Bq);
      const int h1 = hbase - (TOP + kk) * (sc.ge[1] + X + Bq);
      const int q1 = (kk == KL && last) ? QRqr : QRqi;
      const int e0 = sc.boundary_open ? h0 - QRqi : kNegInf;
      const int e1 = sc.boundary_open ? h1 - q1 : kNegInf;
      uint32_t hp = pk2(h0, h1);
      if constexpr (P > 0)
        if (kk == VK) hp &= ~(VM & fm);
      H[kk] = as_v2(bfi(keep_mask, hp, as_u(H[kk])));
      E[kk] = as_v2(bfi(keep_mask, pk2(e0, e1), as_u(E[kk])));
      const uint32_t s01 = sbase + (uint32_t)kk * 0x01000100u;
      SH[kk] = bfi(keep_mask, s01, SH[kk]);
      SE[kk] = bfi(keep_mask, s01, SE[kk]);
    }
  };
#pragma unroll
  for (int kk = 0; kk < TOP; kk++) {
    H[kk] = as_v2(0u);
    E[kk] = as_v2(0u);
    SH[kk] = SE[kk] = 0;
  }
  init_rows(0xffffffffu);
  uint32_t cHd = 0, cSHd = 0, cF = 0, cSF = 0, cDL = 0;  // top half's last row -> bottom half (next step)
  uint32_t xHF = 0, xSS = 0, xDL = 0;                    // last row (Hd | F, SHd | SF, DL) -> lane g+1
  int Lext = 0, trail = 0;
  uint32_t tword = 0, tprev = 1;
  const int nsteps = tl + 2 * G - 1;
  for (int st = 0; st < nsteps; st++) {
    const int j = st - 2 * g;  // top half's column; the bottom half's is j - 1
    const uint32_t rHF = row_shr1(xHF), rSS = row_shr1(xSS), rDL = row_shr1(xDL);
    uint32_t tcode = 0;
    if (j >= 0 && j <= tl) {
      if ((j & 7) == 0) tword = tcp[j >> 3];
      tcode = tword & 15u;
      tword >>= 4;
    }
    const uint32_t bl = (uint32_t)__builtin_ctz(tcode | 16u) & 3u, bh = (uint32_t)__builtin_ctz(tprev | 16u) & 3u;
    tprev = tcode;
    uint32_t M[NG];
#pragma unroll
    for (int gg = 0; gg < NG; gg++)
      M[gg] = ((uint32_t)(MT[gg] >> (16 * bl)) & 0xffffu) | ((uint32_t)(MB[gg] >> (16 * bh)) << 16);
    const bool lc0 = (j == tl - 1), lc1 = (j == tl);
    const uint32_t QRt = pk2(lc0 ? QRtr : QRti, lc1 ? QRtr : QRti);
    const uint32_t Rt = pk2(lc0 ? Rtr : Rti, lc1 ? Rtr : Rti);
    // the row above the top half: the boundary row -1 (lane 0) or lane g-1's last row | carry (bottom half)
    const int hd0 = (j <= 0) ? 0 : -(sc.go[0] + j * sc.ge[0]) + Bq * j;
    const int f0 = sc.boundary_open ? -(sc.go[0] + (j + 1) * sc.ge[0]) - (lc0 ? QRtr : QRti) + Bq * (j + 1) : kNegInf;
    // boundary row -1 for lane 0: H(-1, j-1) (u = j - 1), F(0, j) (u = j, one D move)
    const int jb = (j < 0 ? 0 : j) + kSB;
    v2s Hd = as_v2(bfi(fm, (uint32_t)hd0 & 0xffffu, rHF & 0xffffu) | (cHd << 16));
    uint32_t SHd = bfi(fm, (uint32_t)jb << 8, rSS & 0xffffu) | (cSHd << 16);
    v2s F = as_v2(bfi(fm, (uint32_t)f0 & 0xffffu, rHF >> 16) | (cF << 16));
    uint32_t SF = bfi(fm, (uint32_t)(jb + 1) << 8, rSS >> 16) | (cSF << 16);
    uint32_t DL = bfi(fm, 1u, rDL & 0xffffu) | (cDL << 16);  // D run of the F state
    // each row's diagonal candidate is formed before the row above overwrites its H / S_H (k_align_pk)
    uint32_t e = M[0] & 0x00010001u;
    v2s hn = as_v2(e) * DELTA + Hd;
    uint32_t shn = SHd + e + 0x01000100u;
#pragma unroll
    for (int kk = 0; kk < TOP; kk++) {
      v2s h = hn;
      uint32_t sh = shn;
      const uint32_t oldH = as_u(H[kk]), oldS = SH[kk];  // (the last row's carry for lane g+1)
      if (kk + 1 < TOP) {
        e = (M[(kk + 1) >> 4] >> ((kk + 1) & 15)) & 0x00010001u;
        hn = as_v2(e) * DELTA + H[kk];
        shn = SH[kk] + e + 0x01000100u;
      } else {
        Hd = H[kk];
        SHd = SH[kk];
      }
      const uint32_t mF = gt_mask(F, h);
      h = __builtin_elementwise_max(h, F);
      sh = bfi(mF, SF, sh);
      const v2s Ec = E[kk];
      const uint32_t mE = gt_mask(Ec, h);
      h = __builtin_elementwise_max(h, Ec);
      sh = bfi(mE, SE[kk], sh);
      int dr_last = 0;
      bool eb_last = false;
      if (kk == KL) {
        eb_last = (mE >> 31) != 0;
        dr_last = (mF >> 31) != 0 ? (int)(DL >> 16) : 0;
      }
      const v2s fo = h - as_v2(QRt), fe = F - as_v2(Rt);
      const uint32_t mfx = gt_mask(fe, fo);
      F = __builtin_elementwise_max(fo, fe);
      // extended, or opened from an H that took F (continuing H's run): one more; else a new run of 1
      DL = bfi(mfx | (mF & ~mE), DL + 0x00010001u, 0x00010001u);
      SF = bfi(mfx, SF, sh);
      const uint32_t qrq = kk == KL ? qrqL : pk2(QRqi, QRqi);
      const v2s eo = h - as_v2(qrq), ee = kk == KL ? Ec - as_v2(rqL) : Ec;  // interior E extension: free
      const uint32_t mex = gt_mask(ee, eo);
      if (kk == KL) {
        const bool ex = (mex >> 31) != 0;
        const int lh = eb_last ? 1 + Lext : 0;
        trail = eb_last ? lh : dr_last;
        Lext = ex ? 1 + Lext : lh;
      }
      E[kk] = __builtin_elementwise_max(eo, ee);
      SE[kk] = bfi(mex, SE[kk], sh);
      H[kk] = h;
      SH[kk] = sh;
      if constexpr (P > 0) {
        if (kk == VK) {
          // lane 0's stand-in row leaves exactly what the boundary row -1 gives the row below it
          const int cv = VR < TOP ? j : j - 1;
          const int hb = cv < 0 ? 0 : -(sc.go[0] + (cv + 1) * sc.ge[0]) + Bq * (cv + 1);
          const int fb = sc.boundary_open ? hb - (cv == tl - 1 ? QRtr : QRti) : kNegInf;
          const int sb = (cv < -1 ? -1 : cv) + 1 + kSB;  // H(-1, cv) and F(0, cv): u = cv
          const uint32_t vm = VM & fm;
          H[kk] = as_v2(bfi(vm, pk2(hb, hb), as_u(H[kk])));
          SH[kk] = bfi(vm, pk2(sb << 8, sb << 8), SH[kk]);
          F = as_v2(bfi(vm, pk2(fb, fb), as_u(F)));
          SF = bfi(vm, pk2(sb << 8, sb << 8), SF);
          DL = bfi(vm, 0x00010001u, DL);
        }
      }
      if (kk == KL) {
        // carries for lane g+1: H(last, j-2) and S_H before this step's update, F / S_F / DL out of it
        xHF = (oldH >> 16) | (as_u(F) & 0xffff0000u);
        xSS = (oldS >> 16) | (SF & 0xffff0000u);
        xDL = DL >> 16;
      }
    }
    cHd = as_u(Hd) & 0xffffu;
    cSHd = SHd & 0xffffu;
    cF = as_u(F) & 0xffffu;
    cSF = SF & 0xffffu;
    cDL = DL & 0xffffu;
    if (j <= 0) {
      // columns before 0 (this lane has not started) and the bottom half's column -1: restore
      init_rows(j < 0 ? 0xffffffffu : 0xffff0000u);
      Lext = 0;
      trail = 0;
    }
  }
  if (!last) return;
  const int Hend = (int)(short)(as_u(H[KL]) >> 16) + (X + Bq) * QL - Bq * tl;
  const uint32_t S = (SH[KL] >> 16) & 0xffffu;
  const uint32_t m = S & 0xffu;
  const uint32_t acols = (uint32_t)(QL + tl + kSB) - (S >> 8);
  const uint32_t internal = acols - (uint32_t)trail;
  out[outidx ? outidx[k] : (uint32_t)k] = m | (internal << 8) | (((uint32_t)Hend & 0xffffu) << 16);
}

typedef void (*AlignFn)(DevSeqs, const uint32_t*, const uint32_t*, int32_t, const uint32_t*,
                        const uint32_t*, Scoring, uint32_t*);

// launch table: align[kAlignSlots L + v] (v: 0 packed, 1 IUPAC (one cell per op), 2 banded packed over
// band_lanes(L) lanes; a 2-lane band measured 1.5 % slower than one lane per pair on config 2)
constexpr int kAlignSlots = 3;
template <int L, int LO>
struct AlignRange {
  static void fill(AlignFn* a) {
    a[kAlignSlots * L] = k_align_pk<L>;
    a[kAlignSlots * L + 1] = k_align<L, true>;
    a[kAlignSlots * L + 2] = k_align_band<L, band_lanes(L)>;
    if constexpr (L > LO) AlignRange<L - 1, LO>::fill(a);
  }
};

// one per translation unit of align_inst.hip (lengths [kAlignPartLo[p], kAlignPartLo[p + 1]))
constexpr int kAlignParts = 6;
constexpr int kAlignPartLo[kAlignParts + 1] = {kMinTplLen, 56, 66, 76, 88, 100, kMaxLen + 1};
void fill_align_part0(AlignFn*);
void fill_align_part1(AlignFn*);
void fill_align_part2(AlignFn*);
void fill_align_part3(AlignFn*);
void fill_align_part4(AlignFn*);
void fill_align_part5(AlignFn*);

}  // namespace uc
