// poseidon.h — Plonky2 Poseidon-12 permutation over Goldilocks, host + gfx950 device.
//
// Restates src/Hash/Poseidon.hs:42-101 (4 full + 22 partial + 4 full rounds, x^7 S-box,
// MDS = circulant(MDS_MATRIX_CIRC) + diag(MDS_MATRIX_DIAG), Hash/Constants.hs:19-25).
// The device form keeps the 12-word state in VGPRs (one permutation per lane); round
// constants are wave-uniform scalar loads from __constant__ memory; the MDS entries are
// compile-time immediates (< 2^6) so each row is a 12-term small-constant dot product
// accumulated in 64-bit halves and reduced once.
#pragma once
#include "gl.h"
#include "poseidon_constants.h"

namespace p2 {

static constexpr uint32_t MDS_CIRC[12] = {17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20};
static constexpr uint32_t MDS_DIAG0 = 8;
__host__ __device__ constexpr uint32_t mds_coeff(int i, int j) {
  return MDS_CIRC[((j - i) % 12 + 12) % 12] + (i == j && i == 0 ? MDS_DIAG0 : 0);
}

#if defined(__HIPCC__)
static __constant__ uint64_t c_round_constants[360] = P2V_ALL_ROUND_CONSTANTS_INIT;
// fast partial-round tables, used only by the PoseidonGate constraint program
// (Gate/Custom/Poseidon.hs:92-137, Hash/Constants.hs:27-113)
static __constant__ uint64_t c_fast_first_rc[12] = P2V_FAST_PARTIAL_FIRST_ROUND_CONSTANT_INIT;
static __constant__ uint64_t c_fast_rc[22] = P2V_FAST_PARTIAL_ROUND_CONSTANTS_INIT;
static __constant__ uint64_t c_fast_vs[22 * 11] = P2V_FAST_PARTIAL_ROUND_VS_INIT;
static __constant__ uint64_t c_fast_w_hats[22 * 11] = P2V_FAST_PARTIAL_ROUND_W_HATS_INIT;
static __constant__ uint64_t c_fast_init_matrix[11 * 11] = P2V_FAST_PARTIAL_ROUND_INITIAL_MATRIX_INIT;
#endif
static const uint64_t h_round_constants[360] = P2V_ALL_ROUND_CONSTANTS_INIT;

// Inside the permutation values are kept in [0, 2^64) (congruent mod p, not necessarily
// canonical); the 12 outputs are canonicalised once at the end.  This removes the
// compare/select of every add and multiply (~13% of the instruction stream).
__host__ __device__ __forceinline__ uint64_t add_nc(uint64_t a, uint64_t b) {   // a < 2^64, b < p
  uint64_t s = a + b;
  return s + ((s < a) ? gl::EPS : 0);   // a + b - 2^64 + EPS < 2^64: no second carry
}
__host__ __device__ __forceinline__ uint64_t mul_nc(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return gl::mul_nc_dev(a, b);
#else
  uint64_t hi, lo;
  gl::mul128(a, b, hi, lo);
  return gl::reduce128_nc(hi, lo);
#endif
}
// x^7
__host__ __device__ __forceinline__ uint64_t sbox(uint64_t x) {
  uint64_t x2 = mul_nc(x, x);
  uint64_t x3 = mul_nc(x, x2);
  uint64_t x4 = mul_nc(x2, x2);
  return mul_nc(x3, x4);
}

#if defined(__HIP_DEVICE_COMPILE__) || defined(__clang__)
#define P2_UNROLL _Pragma("unroll")
#else
#define P2_UNROLL _Pragma("GCC unroll 12")
#endif

// ah * 2^32 + al (al, ah < 2^43) -> [0, 2^64): with ah = ah_hi 2^32 + ah_lo the value is
// ah_hi 2^64 + ah_lo 2^32 + al == ah_hi (2^32 - 1) + al + ah_lo 2^32 (mod p); the first two
// terms stay below 2^44, so one wrap fix-up suffices (v_mad_u64_u32 + 3 VALU).
__host__ __device__ __forceinline__ uint64_t mds_reduce(uint64_t al, uint64_t ah) {
  const uint64_t t = (ah >> 32) * 0xFFFFFFFFULL + al;
  const uint64_t r = t + (ah << 32);
  return r + (r < t ? gl::EPS : 0);
}

// y = M x with M = circ + diag; inputs any value < 2^64, outputs < 2^64 (lazy).
// Each row is sum_j c_j x_j with c_j < 2^6, accumulated separately over the 32-bit halves.
__host__ __device__ __forceinline__ void mds(uint64_t s[12]) {
  uint64_t out[12];
  P2_UNROLL
  for (int i = 0; i < 12; i++) {
    uint64_t al = 0, ah = 0;
    P2_UNROLL
    for (int j = 0; j < 12; j++) {
      const uint64_t c = mds_coeff(i, j);
      al += (uint64_t)(uint32_t)s[j] * c;
      ah += (s[j] >> 32) * c;
    }
    out[i] = mds_reduce(al, ah);
  }
  P2_UNROLL
  for (int i = 0; i < 12; i++) s[i] = out[i];
}

__host__ __device__ __forceinline__ uint64_t round_constant(int idx) {
#if defined(__HIP_DEVICE_COMPILE__)
  return c_round_constants[idx];
#else
  return h_round_constants[idx];
#endif
}

__host__ __device__ __forceinline__ void full_round(uint64_t s[12], int r) {
  P2_UNROLL
  for (int i = 0; i < 12; i++) s[i] = sbox(add_nc(s[i], round_constant(12 * r + i)));
  mds(s);
}
__host__ __device__ __forceinline__ void partial_round(uint64_t s[12], int r) {
  s[0] = sbox(add_nc(s[0], round_constant(12 * r)));
  P2_UNROLL
  for (int i = 1; i < 12; i++) s[i] = add_nc(s[i], round_constant(12 * r + i));
  mds(s);
}

// Hash/Poseidon.hs:42-46.  Inputs may be any value < 2^64; outputs are canonical.
__host__ __device__ __forceinline__ void permute(uint64_t s[12]) {
#pragma unroll 1
  for (int r = 0; r < 4; r++) full_round(s, r);
#pragma unroll 1
  for (int r = 4; r < 26; r++) partial_round(s, r);
#pragma unroll 1
  for (int r = 26; r < 30; r++) full_round(s, r);
  P2_UNROLL
  for (int i = 0; i < 12; i++) s[i] = gl::canon(s[i]);
}

}  // namespace p2
