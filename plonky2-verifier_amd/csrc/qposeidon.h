// qposeidon.h — Poseidon-12 spread over a lane QUAD (device only).
//
// Used where the permutation is on a serial critical path (the Fiat–Shamir transcript,
// ~114 dependent permutations per proof, Challenge/Pure.hs): lane t = lane & 3 of the
// quad owns state words 3t, 3t+1, 3t+2.  Full rounds run three S-boxes per lane instead of
// twelve; the MDS row i = 3t + m needs every word: the other lanes' words are fetched with
// DPP quad_perm rotations (lane t reads lane (t+d) & 3), which makes the circulant
// coefficient of every term wave-uniform: M(3t+m, 3((t+d)&3)+k) = circ[(3d + k - m) mod 12]
// (+8 on the diagonal entry (0,0), Hash/Constants.hs:21-25).  ~3.6x lower latency per
// permutation than one lane holding all 12 words.  The 22 partial rounds run as the merged
// blocks of poseidon.h (PBlock) in this layout (qblock below).
#pragma once
#include "gl.h"
#include "poseidon.h"
#include "lposeidon.h"

namespace qp {

#ifndef P2V_QUAD_SBOX
#define P2V_QUAD_SBOX 1
#endif
// The chain's S-box (latency-bound waves: an instruction's cost is its issue slot, s_nop padding
// included): 1 = the asm-block multiply of lposeidon.h (one statement, one padding per multiply,
// round 5), 0 = p2::sbox_lat (the branch-free multiply, five asm statements per multiply)
__device__ __forceinline__ uint64_t sbox_q(uint64_t x) {
#if P2V_QUAD_SBOX && defined(__HIP_DEVICE_COMPILE__)
  return lp::sbox(x);
#else
  return p2::sbox_lat(x);
#endif
}

// quad_perm rotation: lane t reads lane (t + D) & 3
template <int D>
__device__ __forceinline__ uint32_t rot32(uint32_t v) {
  constexpr int ctrl = ((0 + D) & 3) | (((1 + D) & 3) << 2) | (((2 + D) & 3) << 4) | (((3 + D) & 3) << 6);
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, ctrl, 0xf, 0xf, false);
}
template <int D>
__device__ __forceinline__ uint64_t rot64(uint64_t v) {
  return ((uint64_t)rot32<D>((uint32_t)(v >> 32)) << 32) | rot32<D>((uint32_t)v);
}
// broadcast lane `src` (uniform, 0..3) of each quad
__device__ __forceinline__ uint32_t bcast32(uint32_t v, int src) {
  switch (src) {
    case 0: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x00, 0xf, 0xf, false);
    case 1: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x55, 0xf, 0xf, false);
    case 2: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xAA, 0xf, 0xf, false);
    default: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xFF, 0xf, 0xf, false);
  }
}
__device__ __forceinline__ uint64_t bcast64(uint64_t v, int src) {
  return ((uint64_t)bcast32((uint32_t)(v >> 32), src) << 32) | bcast32((uint32_t)v, src);
}

// this lane's round constants (words 3t..3t+2 of round r) as 32-bit halves: they start the
// MDS row accumulators of round r-1 (the constant addition folded into the previous MDS, as
// in p2::permute_dev).  In the natural table layout they are contiguous, so each lane does a
// plain (LDS) load; the caller prefetches one round ahead.
__device__ __forceinline__ void lane_rc(const p2::RcSplit& rc, int r, int t, uint64_t kl[3], uint64_t kh[3]) {
  const uint64_t* L = rc.lo + 12 * r + 3 * t;
  const uint64_t* H = rc.hi + 12 * r + 3 * t;
#pragma unroll
  for (int k = 0; k < 3; k++) { kl[k] = L[k]; kh[k] = H[k]; }
}

// one MDS row M of this lane (global row 3t + M): the 12 terms in (rotation d, word k) order
template <int M, int Q>
__device__ __forceinline__ void qrow(const uint64_t (&X)[4][3], uint64_t& al, uint64_t& ah, uint64_t c00) {
  if constexpr (Q < 12) {
    constexpr int d = Q / 3, k = Q % 3;
    constexpr int idx = ((3 * d + k - M) % 12 + 12) % 12;
    if constexpr (M == 0 && Q == 0) {   // the diagonal entry: 25 on global row 0, else 17
      al += (uint64_t)(uint32_t)X[d][k] * c00;
      ah += (X[d][k] >> 32) * c00;
    } else {
      // plain MADs: an asm MAD costs a wait state before its consumer, which lands on
      // this latency-bound chain (measured equal throughput, lower latency)
      al += (uint64_t)(uint32_t)X[d][k] * p2::MDS_CIRC[idx];
      ah += (X[d][k] >> 32) * p2::MDS_CIRC[idx];
    }
    qrow<M, Q + 1>(X, al, ah, c00);
  }
}

// (al, ah)[m] = rows 3t+m of M x + k, unreduced (k = the next round's constants of this lane's
// rows, split into halves)
__device__ __forceinline__ void mds_acc(const uint64_t x[3], int t, const uint64_t kl[3], const uint64_t kh[3],
                                        uint64_t al[3], uint64_t ah[3]) {
  uint64_t X[4][3];
#pragma unroll
  for (int k = 0; k < 3; k++) { X[0][k] = x[k]; X[1][k] = rot64<1>(x[k]); X[2][k] = rot64<2>(x[k]); X[3][k] = rot64<3>(x[k]); }
  const uint64_t c00 = t == 0 ? 25 : 17;   // circ[0] (+ diag[0] on row 0)
#pragma unroll
  for (int m = 0; m < 3; m++) { al[m] = kl[m]; ah[m] = kh[m]; }
  qrow<0, 0>(X, al[0], ah[0], c00);
  qrow<1, 0>(X, al[1], ah[1], c00);
  qrow<2, 0>(X, al[2], ah[2], c00);
}

// ---- merged partial rounds in the quad layout (p2::PBlock algebra).  The merged matrices are
// not circulant, so the rotation trick above does not make their coefficients uniform:
//  * chain rows (row 0 of each level) are evaluated in lane 0's frame, where rotation d, slot k
//    holds word 3d + k, with the wave-uniform p2::c_pm coefficients, and broadcast from lane 0;
//  * output rows 3t + m use per-lane coefficients from QBlock (cf[t][m][3d + k] = G_D[3t + m]
//    [3((t + d) & 3) + k], the y terms after them), loaded at the start of the block.
struct QBlock {
  uint32_t cf[4][3][16];   // [t][m]: 12 word coefficients in rotation order, then H_D[m'][3t + m] for m' = 2..D
  uint64_t d[4][3];        // d_D[3t + m]
};
struct QMTab { QBlock b[p2::PM_NB]; };
__host__ __device__ constexpr QMTab make_qm() {
  QMTab T{};
  const p2::PMAlg A = p2::pm_alg();
  int r = 4;
  for (int b = 0; b < p2::PM_NB; b++) {
    const int D = p2::PM_SCHED[b];
    const p2::PMD dd = p2::pm_d(r, D);
    for (int t = 0; t < 4; t++)
      for (int m = 0; m < 3; m++) {
        const int i = 3 * t + m;
        for (int d = 0; d < 4; d++)
          for (int k = 0; k < 3; k++) T.b[b].cf[t][m][3 * d + k] = (uint32_t)A.G[D][i][3 * ((t + d) & 3) + k];
        for (int mm = 2; mm <= D; mm++) T.b[b].cf[t][m][12 + mm - 2] = (uint32_t)A.H[D][mm][i];
        T.b[b].d[t][m] = dd.d[D][i];
      }
    r += D;
  }
  return T;
}
#if P2V_PMERGE
static __constant__ QMTab c_qm = make_qm();
#endif

// The permutation's per-lane tables, copied into LDS once per transcript workgroup (tlds_fill).
// A serial chain cannot afford a vector-memory wait inside the permutation: vmcnt retires in
// issue order, so the first wait on a constant load would also wait for the next chunk's proof
// loads issued before the permutation (kernels.hip) and expose their HBM latency on the chain.
// From LDS the tables come back under lgkmcnt, and the proof loads stay in flight throughout.
struct TLds {
  p2::RcSplit rc;          // round constants as 32-bit halves, rows 0..30
  uint64_t rc0[12];        // round 0's constants (added before the first S-box)
  QBlock qb[p2::PM_NB];    // merged partial-round blocks, per-lane output-row coefficients
};
// cooperative copy by the n threads of the workgroup (tid = threadIdx.x); ends with a barrier,
// so every thread of the workgroup must call it
__device__ __forceinline__ void tlds_fill(TLds& T, int tid, int n) {
  const uint64_t* rs = (const uint64_t*)&p2::c_rc_split;
  uint64_t* rd = (uint64_t*)&T.rc;
  for (int i = tid; i < (int)(sizeof(p2::RcSplit) / 8); i += n) rd[i] = rs[i];
  if (tid < 12) T.rc0[tid] = p2::c_round_constants[tid];
#if P2V_PMERGE
  const uint64_t* qs = (const uint64_t*)&c_qm;
  uint64_t* qd = (uint64_t*)T.qb;
  for (int i = tid; i < (int)(sizeof(QMTab) / 8); i += n) qd[i] = qs[i];
#endif
  __syncthreads();
}

#if P2V_PMERGE && defined(__HIP_DEVICE_COMPILE__)
#define P2V_QMERGE 1

// acc + a c, c a per-lane VGPR coefficient
__device__ __forceinline__ uint64_t madl(uint32_t a, uint32_t c, uint64_t acc) {
  return (uint64_t)a * c + acc;
}
// lane-0 frame dot product of the rotated state with 12 uniform coefficients (template: inline
// MDS row 0 for level 1, else a c_pm chain row)
template <int K>
__device__ __forceinline__ void chain_part(const uint64_t (&X)[4][3], const p2::PBlock& B, uint64_t& al, uint64_t& ah) {
  al = B.dlo[K - 1];
  ah = B.dhi[K - 1];
#pragma unroll
  for (int q = 0; q < 12; q++) {
    const uint64_t w = X[q / 3][q % 3];
    uint32_t c;
    if constexpr (K == 1) c = p2::mds_coeff(0, q);
    else c = B.cf[K - 2][q];
    al += (uint64_t)(uint32_t)w * c;
    ah += (w >> 32) * c;
  }
}
// The chain's S-boxes (inputs the same in all four lanes of the quad): x^3 on lanes 0, 2 and x^4 on
// lanes 1, 3, swapped and multiplied (lp::sbox_u, round 6): three multiplies per lane instead of
// four, bit-identical (P2V_QUAD_SBOX2=0: sbox_q)
#ifndef P2V_QUAD_SBOX2
#define P2V_QUAD_SBOX2 1
#endif
__device__ __forceinline__ uint64_t sbox_qu(uint64_t x, int t) {
#if P2V_QUAD_SBOX2 && P2V_QUAD_SBOX
  return lp::sbox_u(x, t);
#else
  (void)t;
  return sbox_q(x);
#endif
}
template <int D>
__device__ __forceinline__ void qblock(uint64_t x[3], int t, const p2::PBlock& B, const QBlock& Q) {
  // y1 = sbox(word 0) from lane 0; s' = the state with y1 in word 0
  uint64_t y[D + 1];
#if P2V_QUAD_SBOX2 && P2V_QUAD_SBOX
  y[1] = sbox_qu(bcast64(x[0], 0), t);
#else
  y[1] = bcast64(sbox_q(x[0]), 0);
#endif
  x[0] = t == 0 ? y[1] : x[0];
  uint64_t X[4][3];
#pragma unroll
  for (int k = 0; k < 3; k++) { X[0][k] = x[k]; X[1][k] = rot64<1>(x[k]); X[2][k] = rot64<2>(x[k]); X[3][k] = rot64<3>(x[k]); }
  // the chain: z_k = part_k + sum_{m=2..k} H_k[m][0] y_m, y_{k+1} = sbox(z_k); part_k, the
  // s'-part of chain row k, is evaluated in lane 0's frame and broadcast (it does not depend on
  // the S-box chain, so the scheduler can overlap it with the previous S-box)
  uint64_t pl[D], ph[D];
  chain_part<1>(X, B, pl[1], ph[1]);
  pl[1] = bcast64(pl[1], 0); ph[1] = bcast64(ph[1], 0);
  if constexpr (D >= 3) { chain_part<2>(X, B, pl[2], ph[2]); pl[2] = bcast64(pl[2], 0); ph[2] = bcast64(ph[2], 0); }
  y[2] = sbox_qu(p2::mds_reduce(pl[1], ph[1]), t);
  if constexpr (D >= 4) { chain_part<3>(X, B, pl[3], ph[3]); pl[3] = bcast64(pl[3], 0); ph[3] = bcast64(ph[3], 0); }
  if constexpr (D >= 3) {
    constexpr uint32_t c = p2::mds_coeff(0, 0);
    y[3] = sbox_qu(p2::mds_reduce(pl[2] + (uint64_t)(uint32_t)y[2] * c, ph[2] + (y[2] >> 32) * c), t);
  }
  // per-lane output-row coefficients, one row at a time (row m + 1's loads overlap row m), the
  // first row's before the last S-box: 17 VGPRs in flight instead of 51
  uint32_t cf[3][12 + D - 1];
  uint64_t dq[3];
  const auto load_row = [&](int m) {
#pragma unroll
    for (int j = 0; j < 12 + D - 1; j++) cf[m][j] = Q.cf[t][m][j];
    dq[m] = Q.d[t][m];
  };
  if constexpr (D >= 4) {
    constexpr uint32_t c = p2::mds_coeff(0, 0);
    const uint32_t h2 = B.cf[1][12];
    const uint64_t al = pl[3] + (uint64_t)(uint32_t)y[2] * h2 + (uint64_t)(uint32_t)y[3] * c;
    const uint64_t ah = ph[3] + (y[2] >> 32) * h2 + (y[3] >> 32) * c;
    load_row(0);
    y[4] = sbox_qu(p2::mds_reduce(al, ah), t);
  } else {
    load_row(0);
  }
  // output rows 3t + m
#pragma unroll
  for (int m = 0; m < 3; m++) {
    if (m < 2) load_row(m + 1);
    uint64_t al = dq[m] & 0xFFFFFFFFull, ah = dq[m] >> 32;
#pragma unroll
    for (int q = 0; q < 12; q++) {
      al = madl((uint32_t)X[q / 3][q % 3], cf[m][q], al);
      ah = madl((uint32_t)(X[q / 3][q % 3] >> 32), cf[m][q], ah);
    }
#pragma unroll
    for (int mm = 2; mm <= D; mm++) {
      al = madl((uint32_t)y[mm], cf[m][12 + mm - 2], al);
      ah = madl((uint32_t)(y[mm] >> 32), cf[m][12 + mm - 2], ah);
    }
    x[m] = D == 4 ? p2::dv::reduce_w(al, ah) : p2::dv::reduce_t(al, ah);
  }
}
#endif

// the quad's permutation; x = this lane's three words (inputs < 2^64, outputs canonical).
// Partial rounds take the S-box off the critical path: the MDS runs on the state with word 0
// zeroed while lane 0's S-box chain is in flight, then sbox(word 0), broadcast from lane 0,
// is added with column 0 of M (M[3t+m][0], per lane).
__device__ __forceinline__ void permute(uint64_t x[3], int t, const TLds& T) {
  {
    const uint64_t* R = T.rc0 + 3 * t;
#pragma unroll
    for (int k = 0; k < 3; k++) x[k] = p2::add_nc(x[k], R[k]);
  }
  // M[i][0] = circ[(12 - i) % 12] (+ 8 for i = 0), rows i = 3t .. 3t+2 (Hash/Constants.hs:19-25)
  const uint32_t col0[3] = {t == 0 ? 25u : t == 1 ? 18u : t == 2 ? 13u : 16u,
                            t == 0 ? 20u : t == 1 ? 39u : t == 2 ? 28u : 41u,
                            t == 0 ? 34u : t == 1 ? 13u : t == 2 ? 2u : 15u};
  uint64_t kl[3], kh[3], nkl[3], nkh[3];
#if P2V_QMERGE
  // full rounds 0..3, the merged partial-round blocks, full rounds 26..29
  lane_rc(T.rc, 1, t, nkl, nkh);
#pragma unroll 1
  for (int r = 0; r < 8; r++) {
    if (r == 4) {
#if P2V_PMERGE == 4
#pragma unroll 1
      for (int b = 0; b < 5; b++) qblock<4>(x, t, p2::c_pm.b[b], T.qb[b]);
      qblock<2>(x, t, p2::c_pm.b[5], T.qb[5]);
#elif P2V_PMERGE == 3
#pragma unroll 1
      for (int b = 0; b < 7; b++) qblock<3>(x, t, p2::c_pm.b[b], T.qb[b]);
#else
#pragma unroll 1
      for (int b = 0; b < 11; b++) qblock<2>(x, t, p2::c_pm.b[b], T.qb[b]);
#endif
      lane_rc(T.rc, 27, t, nkl, nkh);
    }
#if P2V_PMERGE == 3
    if (r == 4) {   // the schedule's single plain partial round (25)
      lane_rc(T.rc, 26, t, kl, kh);
      const uint64_t w0 = x[0];
      x[0] = t == 0 ? 0 : w0;
      uint64_t al[3], ah[3];
      mds_acc(x, t, kl, kh, al, ah);
      const uint64_t sb = bcast64(sbox_q(w0), 0);
#pragma unroll
      for (int m = 0; m < 3; m++) { al[m] += (uint64_t)(uint32_t)sb * col0[m]; ah[m] += (sb >> 32) * col0[m]; }
#pragma unroll
      for (int m = 0; m < 3; m++) x[m] = p2::mds_reduce(al[m], ah[m]);
    }
#endif
    const int rr = r < 4 ? r : r + 22;   // 0..3, 26..29
#pragma unroll
    for (int k = 0; k < 3; k++) { kl[k] = nkl[k]; kh[k] = nkh[k]; }
    lane_rc(T.rc, rr + 2 <= 30 ? rr + 2 : 30, t, nkl, nkh);   // row 30 of the split table is zero
    uint64_t al[3], ah[3];
#pragma unroll
    for (int k = 0; k < 3; k++) x[k] = sbox_q(x[k]);
    mds_acc(x, t, kl, kh, al, ah);
#pragma unroll
    for (int m = 0; m < 3; m++) x[m] = p2::mds_reduce(al[m], ah[m]);
  }
  (void)col0;
#else
  lane_rc(T.rc, 1, t, nkl, nkh);
#pragma unroll 1
  for (int r = 0; r < 30; r++) {
#pragma unroll
    for (int k = 0; k < 3; k++) { kl[k] = nkl[k]; kh[k] = nkh[k]; }
    lane_rc(T.rc, r + 2 <= 30 ? r + 2 : 30, t, nkl, nkh);   // row 30 of the split table is zero
    uint64_t al[3], ah[3];
    if (r < 4 || r >= 26) {
#pragma unroll
      for (int k = 0; k < 3; k++) x[k] = sbox_q(x[k]);
      mds_acc(x, t, kl, kh, al, ah);
    } else {
      const uint64_t w0 = x[0];
      x[0] = t == 0 ? 0 : w0;
      mds_acc(x, t, kl, kh, al, ah);           // independent of the S-box below
      const uint64_t s = bcast64(sbox_q(w0), 0);
#pragma unroll
      for (int m = 0; m < 3; m++) {
        al[m] += (uint64_t)(uint32_t)s * col0[m];
        ah[m] += (s >> 32) * col0[m];
      }
    }
#pragma unroll
    for (int m = 0; m < 3; m++) x[m] = p2::mds_reduce(al[m], ah[m]);
  }
#endif
#pragma unroll
  for (int k = 0; k < 3; k++) x[k] = gl::canon(x[k]);
}

// word `pos` (uniform, 0..11) of the quad's state, broadcast to all four lanes
__device__ __forceinline__ uint64_t get_word(const uint64_t x[3], int pos) {
  const int k = pos % 3;
  const uint64_t v = k == 0 ? x[0] : (k == 1 ? x[1] : x[2]);
  return bcast64(v, pos / 3);
}
// write word `pos` (uniform) of the quad's state
__device__ __forceinline__ void set_word(uint64_t x[3], int t, int pos, uint64_t v) {
  const int owner = pos / 3, k = pos % 3;
  const bool mine = t == owner;
  if (k == 0) x[0] = mine ? v : x[0];
  else if (k == 1) x[1] = mine ? v : x[1];
  else x[2] = mine ? v : x[2];
}

}  // namespace qp
