// pposeidon.h — Poseidon-12 spread over a lane PAIR (device only).
//
// The Fiat–Shamir transcript (~115 dependent permutations per proof, Challenge/Pure.hs) in the
// layout between the quad (qposeidon.h, 4 lanes x 3 words) and one lane per proof: lane
// t = lane & 1 of the pair owns state words 6t .. 6t+5.  A single wave issues its chain at
// about one instruction per 4-cycle slot, so the chain's length is the instructions per lane;
// the batch's cost is the instructions per lane times the lanes per proof.  The pair runs 6
// S-boxes and 6 MDS rows per lane per full round (the quad 3 + 3 with 4 lanes, and it repeats
// the partial rounds' S-box chain and chain rows on all 4), so per proof it issues about half
// of the quad's instructions (round 4).
//
// MDS (Hash/Constants.hs:19-25): row 6t + m needs all 12 words; the partner's six arrive by one
// DPP quad_perm swap (lane t reads lane t ^ 1).  Because the circulant's shift by 6 is the same
// both ways (6 = -6 mod 12), every coefficient is wave-uniform:
//   M[6t+m][6t+k] = circ[(k - m) mod 12],  M[6t+m][6(1-t)+k] = circ[(6 + k - m) mod 12],
// plus diag 8 on (0, 0) (lane 0, m = k = 0: a per-lane constant).
// Partial rounds run as poseidon.h's merged blocks (PBlock algebra): the S-box chain and the
// chain rows are computed on both lanes (each holds all 12 words after the swap, so no
// broadcast is needed), the output rows 6t + m with per-lane coefficients (PBlockP).
#pragma once
#include "gl.h"
#include "poseidon.h"
#include "qposeidon.h"

namespace pp {

// lane t reads lane t ^ 1 (quad_perm [1, 0, 3, 2])
__device__ __forceinline__ uint32_t swap32(uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false); }
__device__ __forceinline__ uint64_t swap64(uint64_t v) { return ((uint64_t)swap32((uint32_t)(v >> 32)) << 32) | swap32((uint32_t)v); }
// lane `src` (uniform, 0 or 1) of each pair: quad_perm [0, 0, 2, 2] / [1, 1, 3, 3]
__device__ __forceinline__ uint32_t bcast32(uint32_t v, int src) {
  return src == 0 ? (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xA0, 0xf, 0xf, false)
                  : (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xF5, 0xf, 0xf, false);
}
__device__ __forceinline__ uint64_t bcast64(uint64_t v, int src) {
  return ((uint64_t)bcast32((uint32_t)(v >> 32), src) << 32) | bcast32((uint32_t)v, src);
}

// per-lane coefficients of the merged blocks' output rows (the PBlock algebra of poseidon.h):
// cf[t][m] = G_D[6t + m][own words 6t .. 6t+5, then partner words 6(1-t) ..], then H_D[m'][6t + m]
struct PBlockP {
  uint32_t cf[2][6][16];
  uint64_t d[2][6];
};
struct PMTabP { PBlockP b[p2::PM_NB]; };
__host__ __device__ constexpr PMTabP make_pmp() {
  PMTabP T{};
  const p2::PMAlg A = p2::pm_alg();
  int r = 4;
  for (int b = 0; b < p2::PM_NB; b++) {
    const int D = p2::PM_SCHED[b];
    const p2::PMD dd = p2::pm_d(r, D);
    for (int t = 0; t < 2; t++)
      for (int m = 0; m < 6; m++) {
        const int i = 6 * t + m;
        for (int k = 0; k < 6; k++) {
          T.b[b].cf[t][m][k] = (uint32_t)A.G[D][i][6 * t + k];
          T.b[b].cf[t][m][6 + k] = (uint32_t)A.G[D][i][6 * (1 - t) + k];
        }
        for (int mm = 2; mm <= D; mm++) T.b[b].cf[t][m][12 + mm - 2] = (uint32_t)A.H[D][mm][i];
        T.b[b].d[t][m] = dd.d[D][i];
      }
    r += D;
  }
  return T;
}
#if defined(__HIPCC__)
static __constant__ PMTabP c_pmp = make_pmp();
#endif

// The pair permutation's tables in LDS (the reason: qposeidon.h TLds)
struct TLdsP {
  p2::RcSplit rc;          // round constants as 32-bit halves, rows 0..30
  uint64_t rc0[12];        // round 0's constants
  PBlockP pb[p2::PM_NB];   // merged blocks, per-lane output-row coefficients
};
__device__ __forceinline__ void tlds_fill(TLdsP& T, int tid, int n) {
  const uint64_t* rs = (const uint64_t*)&p2::c_rc_split;
  uint64_t* rd = (uint64_t*)&T.rc;
  for (int i = tid; i < (int)(sizeof(p2::RcSplit) / 8); i += n) rd[i] = rs[i];
  if (tid < 12) T.rc0[tid] = p2::c_round_constants[tid];
  const uint64_t* qs = (const uint64_t*)&c_pmp;
  uint64_t* qd = (uint64_t*)T.pb;
  for (int i = tid; i < (int)(sizeof(PMTabP) / 8); i += n) qd[i] = qs[i];
  __syncthreads();
}

#if defined(__HIP_DEVICE_COMPILE__)
// row 6t + M: the 12 terms (own word k, then partner word k), plain MADs (no inline-asm SGPR
// outputs: no wait states on this latency-bound chain)
template <int M, int K>
__device__ __forceinline__ void prow(const uint64_t (&own)[6], const uint64_t (&par)[6], uint64_t& al, uint64_t& ah, uint64_t c00) {
  if constexpr (K < 12) {
    const uint64_t w = K < 6 ? own[K % 6] : par[K % 6];
    constexpr int idx = K < 6 ? ((K - M) % 12 + 12) % 12 : ((6 + (K - 6) - M) % 12 + 12) % 12;
    if constexpr (M == 0 && K == 0) {   // the diagonal entry: 25 on global row 0 (lane 0), else 17
      al += (uint64_t)(uint32_t)w * c00;
      ah += (w >> 32) * c00;
    } else {
      al += (uint64_t)(uint32_t)w * p2::MDS_CIRC[idx];
      ah += (w >> 32) * p2::MDS_CIRC[idx];
    }
    prow<M, K + 1>(own, par, al, ah, c00);
  }
}
// rows 6t + M.. of M x + k (k: this lane's six constants of the next round, kl / kh the
// halves in LDS, read per row)
template <int M>
__device__ __forceinline__ void mds_rows(const uint64_t (&own)[6], const uint64_t (&par)[6], const uint64_t* kl,
                                         const uint64_t* kh, uint64_t (&out)[6], uint64_t c00) {
  if constexpr (M < 6) {
    uint64_t al = kl[M], ah = kh[M];
    prow<M, 0>(own, par, al, ah, c00);
    out[M] = p2::mds_reduce(al, ah);
    mds_rows<M + 1>(own, par, kl, kh, out, c00);
  }
}

// chain row K of a block (K = 1: MDS row 0, inline entries; else PBlock.cf[K - 2]) plus its
// constant, in lane 0's frame (own words 0..5, partner words 6..11): right on lane 0, discarded
// on lane 1 (the chain's values are broadcast from lane 0)
template <int K>
__device__ __forceinline__ void chain_part(const uint64_t (&x)[6], const uint64_t (&par)[6], const p2::PBlock& B, uint64_t& al, uint64_t& ah) {
  al = B.dlo[K - 1];
  ah = B.dhi[K - 1];
#pragma unroll
  for (int q = 0; q < 12; q++) {
    const uint64_t w = q < 6 ? x[q] : par[q - 6];
    uint32_t c;
    if constexpr (K == 1) c = p2::mds_coeff(0, q);
    else c = B.cf[K - 2][q];
    al += (uint64_t)(uint32_t)w * c;
    ah += (w >> 32) * c;
  }
}

// D merged partial rounds (p2::pblock's algebra) in the pair layout.  The S-box chain (word 0 and
// the chain rows) runs in lane 0's frame and each S-box output is broadcast from lane 0; the
// output rows 6t + m use per-lane coefficients.
template <int D>
__device__ __forceinline__ void pblock(uint64_t (&x)[6], int t, const p2::PBlock& B, const PBlockP& Q) {
  uint64_t y[D + 1];
  y[1] = bcast64(qp::sbox_q(x[0]), 0);   // word 0 lives in lane 0
  uint64_t par[6];
#pragma unroll
  for (int k = 0; k < 6; k++) par[k] = swap64(x[k]);
  if (t == 0) x[0] = y[1]; else par[0] = y[1];   // s' (y1 in word 0)
  uint64_t pl[D], ph[D];
  chain_part<1>(x, par, B, pl[1], ph[1]);
  if constexpr (D >= 3) chain_part<2>(x, par, B, pl[2], ph[2]);
  y[2] = bcast64(qp::sbox_q(p2::mds_reduce(pl[1], ph[1])), 0);
  if constexpr (D >= 4) chain_part<3>(x, par, B, pl[3], ph[3]);
  if constexpr (D >= 3) {
    constexpr uint32_t c = p2::mds_coeff(0, 0);
    y[3] = bcast64(qp::sbox_q(p2::mds_reduce(pl[2] + (uint64_t)(uint32_t)y[2] * c, ph[2] + (y[2] >> 32) * c)), 0);
  }
  if constexpr (D >= 4) {
    constexpr uint32_t c = p2::mds_coeff(0, 0);
    const uint32_t h2 = B.cf[1][12];
    const uint64_t al = pl[3] + (uint64_t)(uint32_t)y[2] * h2 + (uint64_t)(uint32_t)y[3] * c;
    const uint64_t ah = ph[3] + (y[2] >> 32) * h2 + (y[3] >> 32) * c;
    y[4] = bcast64(qp::sbox_q(p2::mds_reduce(al, ah)), 0);
  }
  // output rows 6t + m: per-lane coefficients (LDS), one row at a time
  uint64_t out[6];
#pragma unroll
  for (int m = 0; m < 6; m++) {
    const uint32_t* cf = Q.cf[t][m];
    uint64_t al = Q.d[t][m] & 0xFFFFFFFFull, ah = Q.d[t][m] >> 32;
#pragma unroll
    for (int k = 0; k < 6; k++) {
      al += (uint64_t)(uint32_t)x[k] * cf[k];
      ah += (x[k] >> 32) * cf[k];
      al += (uint64_t)(uint32_t)par[k] * cf[6 + k];
      ah += (par[k] >> 32) * cf[6 + k];
    }
#pragma unroll
    for (int mm = 2; mm <= D; mm++) {
      al += (uint64_t)(uint32_t)y[mm] * cf[12 + mm - 2];
      ah += (y[mm] >> 32) * cf[12 + mm - 2];
    }
    out[m] = D == 4 ? p2::dv::reduce_w(al, ah) : p2::dv::reduce_t(al, ah);
  }
#pragma unroll
  for (int m = 0; m < 6; m++) x[m] = out[m];
}
#endif

// the pair's permutation; x = this lane's six words (inputs < 2^64, outputs canonical)
__device__ __forceinline__ void permute(uint64_t (&x)[6], int t, const TLdsP& T) {
#if defined(__HIP_DEVICE_COMPILE__)
  {
    const uint64_t* R = T.rc0 + 6 * t;
#pragma unroll
    for (int k = 0; k < 6; k++) x[k] = p2::add_nc(x[k], R[k]);
  }
  const uint64_t c00 = t == 0 ? 25 : 17;   // circ[0] (+ diag[0] on row 0)
#pragma unroll 1
  for (int r = 0; r < 8; r++) {   // full rounds 0..3, the merged partial blocks, full rounds 26..29
    if (r == 4) {
#pragma unroll 1
      for (int b = 0; b < 5; b++) pblock<4>(x, t, p2::c_pm.b[b], T.pb[b]);
      pblock<2>(x, t, p2::c_pm.b[5], T.pb[5]);
    }
    const int rr = r < 4 ? r : r + 22;   // 0..3, 26..29
#pragma unroll
    for (int k = 0; k < 6; k++) x[k] = qp::sbox_q(x[k]);
    uint64_t par[6], out[6];
#pragma unroll
    for (int k = 0; k < 6; k++) par[k] = swap64(x[k]);
    // the next round's constants start the MDS rows (row 30 of the split table is 0)
    mds_rows<0>(x, par, T.rc.lo + 12 * (rr + 1) + 6 * t, T.rc.hi + 12 * (rr + 1) + 6 * t, out, c00);
#pragma unroll
    for (int k = 0; k < 6; k++) x[k] = out[k];
  }
#pragma unroll
  for (int k = 0; k < 6; k++) x[k] = gl::canon(x[k]);
#else
  (void)x; (void)t; (void)T;
#endif
}

// word `pos` (uniform, 0..11) of the pair's state, broadcast to both lanes
// (a switch on the uniform position: a select chain over x[] would be turned into a
// dynamically indexed private array, i.e. scratch memory)
__device__ __forceinline__ uint64_t get_word(const uint64_t (&x)[6], int pos) {
  switch (pos) {
    case 0: return bcast64(x[0], 0);
    case 1: return bcast64(x[1], 0);
    case 2: return bcast64(x[2], 0);
    case 3: return bcast64(x[3], 0);
    case 4: return bcast64(x[4], 0);
    case 5: return bcast64(x[5], 0);
    case 6: return bcast64(x[0], 1);
    case 7: return bcast64(x[1], 1);
    case 8: return bcast64(x[2], 1);
    case 9: return bcast64(x[3], 1);
    case 10: return bcast64(x[4], 1);
    default: return bcast64(x[5], 1);
  }
}

}  // namespace pp
