// rposeidon.h — Poseidon-12 spread over a 16-lane DPP row (device only).
//
// The Fiat–Shamir transcript (~115 strictly dependent permutations per proof,
// Challenge/Pure.hs) is latency-bound: a single wave issues at most one instruction per
// 4-cycle slot, so its time is (instructions per lane) x 4 cycles.  Spreading the state over
// a row of 16 lanes (lane L < 12 holds word L, lanes 12..15 idle) leaves one S-box per lane
// per round.  The MDS product y_i = sum_j M_ij x_j becomes a sum over the 16 DPP row
// rotations: rotation m delivers word src_L(m) to lane L, so with a per-lane coefficient
// table coef_L[m] = M[L][src_L(m)] (0 for idle sources) y = sum_m coef[m] * ror_m(x).  The
// table is built at start-up by rotating the lane id itself, so it does not depend on the
// direction convention of row_ror.
//
// Partial rounds (only word 0 goes through the S-box) are written for ILP: the MDS of the
// other eleven words does not depend on the S-box output and is accumulated while the
// S-box chain is in flight; sbox(x_0) is then added with a row broadcast and one column of M.
#pragma once
#include "gl.h"
#include "poseidon.h"

namespace rp {

static __constant__ uint32_t c_mds_circ[12] = {17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20};

template <int M>
__device__ __forceinline__ uint32_t ror32(uint32_t v) {
  if constexpr (M == 0) return v;
  else return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x120 + M, 0xf, 0xf, true);   // row_ror:M (all lanes valid)
}
template <int S>
__device__ __forceinline__ uint32_t nbcast32(uint32_t v) {   // row_newbcast:S (lane S of each row)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150 + S, 0xf, 0xf, true);
}
template <int S>
__device__ __forceinline__ uint64_t nbcast64(uint64_t v) {
  return ((uint64_t)nbcast32<S>((uint32_t)(v >> 32)) << 32) | nbcast32<S>((uint32_t)v);
}
// broadcast word `pos` (wave-uniform, 0..11) of the row
__device__ __forceinline__ uint64_t get_word(uint64_t x, int pos) {
  switch (pos) {
    case 0: return nbcast64<0>(x);
    case 1: return nbcast64<1>(x);
    case 2: return nbcast64<2>(x);
    case 3: return nbcast64<3>(x);
    case 4: return nbcast64<4>(x);
    case 5: return nbcast64<5>(x);
    case 6: return nbcast64<6>(x);
    case 7: return nbcast64<7>(x);
    case 8: return nbcast64<8>(x);
    case 9: return nbcast64<9>(x);
    case 10: return nbcast64<10>(x);
    default: return nbcast64<11>(x);
  }
}

struct Row {
  uint32_t coef[16];   // coef[m] = M[L][src_L(m)]
  uint32_t col0;       // M[L][0]
  int L;
  bool plus;           // row_ror:m reads lane (L + m) & 15 (else (L - m) & 15)
};

__device__ __forceinline__ uint32_t mds_entry(int i, int j) {   // Hash/Constants.hs:19-25
  return c_mds_circ[(j - i + 12) % 12] + ((i == 0 && j == 0) ? 8u : 0u);
}

template <int M>
__device__ __forceinline__ void init_coef(Row& R) {
  const int src = (int)ror32<M>((uint32_t)R.L);
  R.coef[M] = (R.L < 12 && src < 12) ? mds_entry(R.L, src) : 0u;
}

__device__ __forceinline__ void init(Row& R, int lane) {
  R.L = lane & 15;
  init_coef<0>(R); init_coef<1>(R); init_coef<2>(R); init_coef<3>(R);
  init_coef<4>(R); init_coef<5>(R); init_coef<6>(R); init_coef<7>(R);
  init_coef<8>(R); init_coef<9>(R); init_coef<10>(R); init_coef<11>(R);
  init_coef<12>(R); init_coef<13>(R); init_coef<14>(R); init_coef<15>(R);
  R.col0 = R.L < 12 ? mds_entry(R.L, 0) : 0u;
  R.plus = (int)ror32<1>((uint32_t)R.L) == ((R.L + 1) & 15);
}

template <int M>
__device__ __forceinline__ void acc_rot(const Row& R, uint32_t lo, uint32_t hi, uint64_t& al, uint64_t& ah) {
  al += (uint64_t)ror32<M>(lo) * R.coef[M];
  ah += (uint64_t)ror32<M>(hi) * R.coef[M];
}
// (al, ah) += sum_m coef[m] ror_m(v), accumulated over the 32-bit halves; even and odd
// rotations go to separate accumulators (4 independent mad chains) so the scheduler can
// overlap them
__device__ __forceinline__ void conv(const Row& R, uint64_t v, uint64_t& al, uint64_t& ah) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  uint64_t al0 = (uint64_t)lo * R.coef[0] + al, ah0 = (uint64_t)hi * R.coef[0] + ah;
  uint64_t al1 = (uint64_t)ror32<1>(lo) * R.coef[1], ah1 = (uint64_t)ror32<1>(hi) * R.coef[1];
  acc_rot<2>(R, lo, hi, al0, ah0); acc_rot<3>(R, lo, hi, al1, ah1);
  acc_rot<4>(R, lo, hi, al0, ah0); acc_rot<5>(R, lo, hi, al1, ah1);
  acc_rot<6>(R, lo, hi, al0, ah0); acc_rot<7>(R, lo, hi, al1, ah1);
  acc_rot<8>(R, lo, hi, al0, ah0); acc_rot<9>(R, lo, hi, al1, ah1);
  acc_rot<10>(R, lo, hi, al0, ah0); acc_rot<11>(R, lo, hi, al1, ah1);
  acc_rot<12>(R, lo, hi, al0, ah0); acc_rot<13>(R, lo, hi, al1, ah1);
  acc_rot<14>(R, lo, hi, al0, ah0); acc_rot<15>(R, lo, hi, al1, ah1);
  al = al0 + al1;
  ah = ah0 + ah1;
}

#ifndef P2V_ROW_SBOX
#define P2V_ROW_SBOX 0
#endif
// The row form's S-box: a lone wave on its chain pays for every instruction it issues, so the
// form matters here more than in the throughput kernels.  0: p2::sbox_lat_br (the S-box multiply
// with one uniform branch per stage); 1: the multiply in plain C (the compiler's own carries:
// no inline-asm statement, so no s_nop padding after one); 2: each multiply one asm block
// (p2asm::mul_blk, 16 VALU, padding once per multiply); 3: p2::sbox_lat (branch-free).
__device__ __forceinline__ uint64_t mul_c(uint64_t a, uint64_t b) {
  const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  const uint64_t p00 = (uint64_t)a0 * b0;
  const uint64_t x = (uint64_t)a0 * b1 + (p00 >> 32);    // < 2^64
  const uint64_t y = (uint64_t)a1 * b0 + x;              // may wrap: weight 2^96
  const uint64_t cm = y < x ? 1 : 0;
  const uint64_t hh = (uint64_t)a1 * b1 + (y >> 32);     // < 2^64
  const uint64_t lo = (y << 32) | (uint32_t)p00;
  // lo + h0 (2^32 - 1) - h1 - cm  (2^64 == 2^32 - 1, 2^96 == -1 mod p)
  uint64_t t = (hh & 0xFFFFFFFFULL) * 0xFFFFFFFFULL + lo;
  t += t < lo ? gl::EPS : 0;
  const uint64_t d = (hh >> 32) + cm;                    // <= 2^32
  uint64_t r = t - d;
  r -= t < d ? gl::EPS : 0;
  return r;
}
__device__ __forceinline__ uint64_t sbox_row(uint64_t x) {
#if P2V_ROW_SBOX == 1
  const uint64_t x2 = mul_c(x, x), x3 = mul_c(x, x2), x4 = mul_c(x2, x2);
  return mul_c(x3, x4);
#elif P2V_ROW_SBOX == 2 && defined(__HIP_DEVICE_COMPILE__)
  const uint64_t x2 = p2asm::mul_blk(x, x), x3 = p2asm::mul_blk(x, x2), x4 = p2asm::mul_blk(x2, x2);
  return p2asm::mul_blk(x3, x4);
#elif P2V_ROW_SBOX == 3
  return p2::sbox_lat(x);
#else
  return p2::sbox_lat_br(x);
#endif
}

// this lane's round constant (idle lanes read word 11) as 32-bit halves, prefetched one
// round ahead: it starts the lane's MDS accumulators of the previous round (the constant
// addition folded into the MDS, as in p2::permute_dev)
__device__ __forceinline__ void lane_rc(const p2::RcSplit& rc, int r, int L, uint64_t& kl, uint64_t& kh) {
  const int i = 12 * r + (L < 12 ? L : 11);
  kl = rc.lo[i];
  kh = rc.hi[i];
}

// the row's permutation; x = this lane's word (inputs < 2^64, outputs canonical).  T: the
// constant tables in LDS (qposeidon.h TLds: rc, rc0), for the reason given there
template <class TT>
__device__ __forceinline__ uint64_t permute(uint64_t x, const Row& R, const TT& T) {
  x = p2::add_nc(x, T.rc0[R.L < 12 ? R.L : 11]);
  uint64_t nkl, nkh;
  lane_rc(T.rc, 1, R.L, nkl, nkh);
#pragma unroll 1
  for (int r = 0; r < 30; r++) {
    uint64_t al = nkl, ah = nkh;
    lane_rc(T.rc, r + 2 <= 30 ? r + 2 : 30, R.L, nkl, nkh);   // row 30 of the split table is zero
    if (r < 4 || r >= 26) {
      conv(R, sbox_row(x), al, ah);
    } else {
      conv(R, R.L == 0 ? 0 : x, al, ah);   // words 1..11: independent of the S-box chain
      const uint64_t s = nbcast64<0>(sbox_row(x));
      al += (uint64_t)(uint32_t)s * R.col0;
      ah += (s >> 32) * R.col0;
    }
    x = p2::mds_reduce(al, ah);
  }
  return gl::canon(x);
}

__device__ __forceinline__ uint64_t set_word(uint64_t x, const Row& R, int pos, uint64_t v) { return R.L == pos ? v : x; }

}  // namespace rp
