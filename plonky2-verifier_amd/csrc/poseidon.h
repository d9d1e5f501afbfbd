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
#include "pasm.h"
#ifndef P2V_POSEIDON_ASMBLK
#define P2V_POSEIDON_ASMBLK 0   // measured: no faster in the verifier kernels (VGPR pressure), see DESIGN.md §5.1
#endif

#ifndef P2V_MDS_BRANCH
#define P2V_MDS_BRANCH 2   // MDS row reduction: the rare carry fix-up in a uniform branch (1: per row, 2: per group of 4 rows)
#endif
#ifndef P2V_SBOX_MUL
#define P2V_SBOX_MUL 2   // S-box multiply form (gl::mul_nc_dev_v): 2 = rare wrap as a uniform branch
#endif

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
  return gl::mul_nc_dev_v<P2V_SBOX_MUL>(a, b);
#else
  uint64_t hi, lo;
  gl::mul128(a, b, hi, lo);
  return gl::reduce128_nc(hi, lo);
#endif
}
// x^7, latency forms for the transcript chains (qposeidon.h, rposeidon.h, pposeidon.h).
// sbox_lat_br: the S-box multiply (11 VALU) with its rare -2^64 fix-up behind one wave-uniform
// branch per stage (x^2; x^3 and x^4; x^7), as the throughput S-box (sbox_n); the row form
// (rposeidon.h) uses it (k_merkle_row 0.142 -> 0.134 ms).  sbox_lat: the branch-free multiply
// (14 VALU), straight-line code; the quad form keeps it (with the branch form its k_phase1 went
// 1.93 -> 2.03 ms, profiles/r04u_sbox_lat_branch.txt).
__host__ __device__ __forceinline__ uint64_t sbox_lat(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t x2 = gl::mul_nc_dev(x, x), x3 = gl::mul_nc_dev(x, x2), x4 = gl::mul_nc_dev(x2, x2);
  return gl::mul_nc_dev(x3, x4);
#else
  uint64_t hi, lo, x2, x3, x4;
  gl::mul128(x, x, hi, lo); x2 = gl::reduce128_nc(hi, lo);
  gl::mul128(x, x2, hi, lo); x3 = gl::reduce128_nc(hi, lo);
  gl::mul128(x2, x2, hi, lo); x4 = gl::reduce128_nc(hi, lo);
  gl::mul128(x3, x4, hi, lo); return gl::reduce128_nc(hi, lo);
#endif
}
__host__ __device__ __forceinline__ uint64_t sbox_lat_br(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t n2, n3, n4, n7;
  uint64_t x2 = gl::mul_nc_part(x, x, n2);
  if (__builtin_expect(n2 != 0, 0)) x2 = gl::mul_fix_neg(x2, n2);
  uint64_t x3 = gl::mul_nc_part(x, x2, n3), x4 = gl::mul_nc_part(x2, x2, n4);
  if (__builtin_expect((n3 | n4) != 0, 0)) { x3 = gl::mul_fix_neg(x3, n3); x4 = gl::mul_fix_neg(x4, n4); }
  uint64_t r = gl::mul_nc_part(x3, x4, n7);
  if (__builtin_expect(n7 != 0, 0)) r = gl::mul_fix_neg(r, n7);
  return r;
#else
  return sbox_lat(x);
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

// ah * 2^32 + al (al, ah < 2^63) -> [0, 2^64): with ah = ah_hi 2^32 + ah_lo the value is
// ah_hi 2^64 + ah_lo 2^32 + al == ah_hi (2^32 - 1) + al + ah_lo 2^32 (mod p); the first two
// terms stay below 2^64 and adding ah_lo 2^32 wraps at most once, after which the sum is
// below 2^63, so one wrap fix-up suffices (v_mad_u64_u32 + 3 VALU).
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

#if defined(__HIPCC__)
// ---------------------------------------------------------------- device permutation
// Same function, restructured for the gfx950 VALU (one permutation per lane):
//  * the round constant of round r+1 is folded into round r's MDS: each row's two 32-bit-half
//    accumulators START at the constant's halves (the first v_mad_u64_u32's addend), so
//    rounds 1..29 spend no instruction on constant addition;
//  * every MDS multiply-add is an explicit v_mad_u64_u32 with the matrix entry as an inline
//    constant (the compiler otherwise turns 2/16 into 64-bit shifts of zero-extended register
//    pairs and pays a v_mov per pair);
//  * rounds alternate between two register sets (s -> t -> s), so no copies are needed at
//    loop edges; full rounds run as 4 pairs, the 22 partial rounds as merged blocks (PBlock,
//    P2V_PMERGE; 11 pairs of single rounds with P2V_PMERGE=0).
struct RcSplit { uint64_t lo[31 * 12], hi[31 * 12]; };   // round 30 = 0 (after the last MDS)
__host__ __device__ constexpr RcSplit make_rc_split() {
  RcSplit t{};
  constexpr uint64_t rc[360] = P2V_ALL_ROUND_CONSTANTS_INIT;
  for (int k = 0; k < 360; k++) { t.lo[k] = rc[k] & 0xFFFFFFFFull; t.hi[k] = rc[k] >> 32; }
  return t;
}
// S-box outputs of round 0 for state words 8..11 when they enter as 0 (2-to-1 compression
// and the first block of every sponge): sbox(rc[0][8 + i]).
struct ZhConst { uint64_t z[4]; };
__host__ __device__ constexpr uint64_t cx_mul(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) % gl::P); }
__host__ __device__ constexpr ZhConst make_zh() {
  ZhConst t{};
  constexpr uint64_t rc[360] = P2V_ALL_ROUND_CONSTANTS_INIT;
  for (int i = 0; i < 4; i++) {
    const uint64_t x = rc[8 + i] % gl::P, x2 = cx_mul(x, x), x3 = cx_mul(x2, x), x4 = cx_mul(x2, x2);
    t.z[i] = cx_mul(x3, x4);
  }
  return t;
}
static __constant__ RcSplit c_rc_split = make_rc_split();
static __constant__ ZhConst c_zh = make_zh();
#ifndef P2V_ZH_FOLD
#define P2V_ZH_FOLD 1   // round 0 of a zh permutation peeled before the round loop, its constant columns folded (below)
#endif
// Round 0 of a permutation whose words 8..11 enter as 0 (2-to-1 compression, first sponge block):
// their S-box outputs z_j are constants (c_zh), so row i of that round's MDS plus round 1's constant
// is sum_{j<8} M_ij y_j + K_i with K_i = rc[1][i] + sum_{j>=8} M_ij z_j (mod p), whose 32-bit halves
// start the row's accumulators: 8 MADs per row less (96 per permutation).  Same field elements as
// Hash/Poseidon.hs:48-52 (fullRound, mdsLayer).
struct ZrcSplit { uint64_t lo[12], hi[12]; };
__host__ __device__ constexpr ZrcSplit make_zrc() {
  ZrcSplit t{};
  constexpr uint64_t rc[360] = P2V_ALL_ROUND_CONSTANTS_INIT;
  const ZhConst z = make_zh();
  for (int i = 0; i < 12; i++) {
    unsigned __int128 a = rc[12 + i] % gl::P;
    for (int j = 8; j < 12; j++) a += (unsigned __int128)mds_coeff(i, j) * z.z[j - 8];
    const uint64_t k = (uint64_t)(a % gl::P);
    t.lo[i] = k & 0xFFFFFFFFull;
    t.hi[i] = k >> 32;
  }
  return t;
}
static __constant__ ZrcSplit c_zrc = make_zrc();
#endif

// ---------------------------------------------------------------- merged partial rounds
// A partial round changes only word 0 before its MDS, so D consecutive partial rounds need
// only D scalars through the S-box.  With s' = the block's input state after the first S-box
// (y1 in word 0) and y_k the S-box output of round k of the block, the state after the block is
//   out = G_D s' + sum_{m=2..D} H_D[:,m] y_m + d_D,   G_1 = M, G_k = M[:,1:] G_{k-1}[1:,:],
//   H_k[:,k] = M[:,0], H_k[:,m] = M[:,1:] H_{k-1}[1:,m] (m < k),
//   d_1 = rc[r+1], d_k = M[:,1:] d_{k-1}[1:] + rc[r+k]  (mod p),
// and the S-box input of round k+1 is row 0 of the same expression at depth k.  Because the
// MDS entries are < 2^6 and non-negative, every entry of G_k and H_k stays non-negative and
// small (row sums < 2^(8k)): up to D = 4 a row is still a dot product over the 32-bit halves
// of 64-bit words that cannot overflow (row sums < 2^31.8, so al, ah < 2^64), with one
// reduction per row.  The 22 partial rounds then cost 6 blocks of (D S-boxes + D-1 chain rows
// + 12 output rows) instead of 22 full MDS layers: about 4 000 VALU instead of 7 900.
// Same function as Hash/Poseidon.hs:48-60 (partialRound, mdsLayer) applied 22 times.
struct PBlock {
  uint32_t cf[14][16];      // rows: chain k = 2, 3 at [k - 2], output row i at [2 + i]; G coefs [0..11], H (m = 2..D-1) at [12 + m - 2]
  uint64_t dlo[16], dhi[16];  // halves of d: chain k = 1..D-1 at [k - 1], output row i at [4 + i]
};
#ifndef P2V_PMERGE
#define P2V_PMERGE 4   // partial rounds per block: 4 (blocks 4,4,4,4,4,2), 3 (3 x 7 + 1), 2 (2 x 11), 0 (one MDS per round)
#endif
#if P2V_PMERGE == 4
static constexpr int PM_NB = 6;
static constexpr int PM_SCHED[PM_NB] = {4, 4, 4, 4, 4, 2};
#elif P2V_PMERGE == 3
static constexpr int PM_NB = 8;
static constexpr int PM_SCHED[PM_NB] = {3, 3, 3, 3, 3, 3, 3, 1};
#else
static constexpr int PM_NB = 11;
static constexpr int PM_SCHED[PM_NB] = {2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2};
#endif
struct PMTab { PBlock b[PM_NB]; };
__host__ __device__ constexpr uint64_t cx_addp(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a + b) % gl::P); }
__host__ __device__ constexpr uint64_t cx_mulp(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) % gl::P); }
__host__ __device__ constexpr int pm_rounds() { int n = 0; for (int b = 0; b < PM_NB; b++) n += PM_SCHED[b]; return n; }
static_assert(pm_rounds() == 22, "the merge schedule must cover the 22 partial rounds");
// G_k, H_k of the block algebra above (k = 1..4), exact non-negative integers
struct PMAlg { uint64_t G[5][12][12], H[5][5][12]; };   // H[k][m][i]
__host__ __device__ constexpr PMAlg pm_alg() {
  PMAlg A{};
  for (int i = 0; i < 12; i++)
    for (int j = 0; j < 12; j++) A.G[1][i][j] = mds_coeff(i, j);
  for (int k = 2; k <= 4; k++) {
    for (int i = 0; i < 12; i++) {
      for (int j = 0; j < 12; j++) {
        uint64_t a = 0;
        for (int l = 1; l < 12; l++) a += mds_coeff(i, l) * A.G[k - 1][l][j];
        A.G[k][i][j] = a;
      }
      for (int m = 2; m < k; m++) {
        uint64_t a = 0;
        for (int l = 1; l < 12; l++) a += mds_coeff(i, l) * A.H[k - 1][m][l];
        A.H[k][m][i] = a;
      }
      A.H[k][k][i] = mds_coeff(i, 0);
    }
  }
  return A;
}
// d_1..d_D (mod p) of the block of D partial rounds starting at round r
struct PMD { uint64_t d[5][12]; };
__host__ __device__ constexpr PMD pm_d(int r, int D) {
  PMD R{};
  constexpr uint64_t rc[360] = P2V_ALL_ROUND_CONSTANTS_INIT;
  for (int i = 0; i < 12; i++) R.d[1][i] = rc[12 * (r + 1) + i] % gl::P;
  for (int k = 2; k <= D; k++)
    for (int i = 0; i < 12; i++) {
      uint64_t a = rc[12 * (r + k) + i] % gl::P;
      for (int l = 1; l < 12; l++) a = cx_addp(a, cx_mulp(mds_coeff(i, l), R.d[k - 1][l]));
      R.d[k][i] = a;
    }
  return R;
}
__host__ __device__ constexpr PMTab make_pm() {
  PMTab T{};
  const PMAlg A = pm_alg();
  int r = 4;
  for (int b = 0; b < PM_NB; b++) {
    const int D = PM_SCHED[b];
    const PMD dd = pm_d(r, D);
    PBlock& B = T.b[b];
    for (int k = 1; k < D; k++) { B.dlo[k - 1] = dd.d[k][0] & 0xFFFFFFFFull; B.dhi[k - 1] = dd.d[k][0] >> 32; }
    for (int k = 2; k < D; k++) {
      for (int j = 0; j < 12; j++) B.cf[k - 2][j] = (uint32_t)A.G[k][0][j];
      for (int m = 2; m < k; m++) B.cf[k - 2][12 + m - 2] = (uint32_t)A.H[k][m][0];
    }
    for (int i = 0; i < 12; i++) {
      for (int j = 0; j < 12; j++) B.cf[2 + i][j] = (uint32_t)A.G[D][i][j];
      for (int m = 2; m < D; m++) B.cf[2 + i][12 + m - 2] = (uint32_t)A.H[D][m][i];
      B.dlo[4 + i] = dd.d[D][i] & 0xFFFFFFFFull;
      B.dhi[4 + i] = dd.d[D][i] >> 32;
    }
    r += D;
  }
  return T;
}
#if defined(__HIPCC__)
static __constant__ PMTab c_pm = make_pm();
#endif

#if defined(__HIP_DEVICE_COMPILE__)
namespace dv {
// acc + C a as one v_mad_u64_u32 with the matrix entry C as an inline constant.  The carry-out
// is never needed: it goes to a fixed, clobbered SGPR pair rather than an asm output (an asm
// SGPR output costs a wait state before every consumer, and the compiler would turn C = 2, 16
// into 64-bit shifts of zero-extended register pairs).  The pair must lie inside the kernel's
// SGPR budget: a build that forces a higher occupancy (e.g. amdgpu_waves_per_eu(7) on k_merkle)
// makes hipcc warn "clobber list contains reserved registers: s94, s95", and is not valid.
#ifndef P2V_MADK_C
#define P2V_MADK_C 0   // 1: MDS MADs in plain C (measured slower, round 5: below)
#endif
// P2V_MADK_C = 1 writes the MDS MADs as plain C (a * C + acc, C an inline constant; powers of two
// stay asm, the compiler would turn them into 64-bit shifts and masks), so that no s_nop pads them
// as it pads every inline-asm statement with an SGPR output (k_merkle: 2 855 -> 2 219 static
// s_nop).  Measured (profiles/r05c_madk.txt): the isolated permutation 3.22 -> 2.69 G perm/s
// (generic) and 3.35 -> 2.71-2.80 (compression), the quick line 1.10 M: the compiler's schedule of
// the plain MADs (more moves and 64-bit adds) costs far more than the padding.  Kept for the record.
template <uint32_t C>
__device__ __forceinline__ uint64_t madk(uint32_t a, uint64_t acc) {
#if P2V_MADK_C
  if constexpr ((C & (C - 1)) != 0) return (uint64_t)a * C + acc;
#endif
  uint64_t d;
  asm("v_mad_u64_u32 %0, s[94:95], %1, %2, %3" : "=v"(d) : "v"(a), "n"(C), "v"(acc) : "s94", "s95");
  return d;
}
template <uint32_t C>
__device__ __forceinline__ uint64_t madk_s(uint32_t a, uint64_t acc) {   // acc wave-uniform (SGPR pair)
#if P2V_MADK_C
  if constexpr ((C & (C - 1)) != 0) return (uint64_t)a * C + acc;
#endif
  uint64_t d;
  asm("v_mad_u64_u32 %0, s[94:95], %1, %2, %3" : "=v"(d) : "v"(a), "n"(C), "s"(acc) : "s94", "s95");
  return d;
}
// al + 2^32 ah (al, ah < 2^44) -> [0, 2^64), congruent mod p: t = al + ah_hi (2^32 - 1), then
// + ah_lo 2^32 on the high word; a carry out (2^64 == 2^32 - 1) adds (2^32 - 1) * carry back
// with one more MAD (the wrapped sum is < 2^45, so that cannot carry).  4 VALU.
__device__ __forceinline__ uint64_t reduce_rows(uint64_t al, uint64_t ah) {
  using namespace gl::ax;
  uint64_t c1, c2;
  const uint64_t t = madm1_co((uint32_t)(ah >> 32), al, c1);   // < 2^45: no carry
  const uint32_t rh = add_co((uint32_t)(t >> 32), (uint32_t)ah, c1);
#if P2V_MDS_BRANCH
  // t >> 32 < 2^11, so the carry needs ah_lo > 2^32 - 2^11: ~2^-21 per row for data that is
  // not chosen to hit it.  A wave-uniform branch around the fix-up: 2 VALU per row less.
  uint64_t r = ((uint64_t)rh << 32) | (uint32_t)t;
  if (__builtin_expect(c1 != 0, 0)) r = madm1_co(mask_1(c1), r, c2);
  return r;
#else
  return madm1_co(mask_1(c1), ((uint64_t)rh << 32) | (uint32_t)t, c2);
#endif
}
template <int I, int J, int E = 12>
__device__ __forceinline__ void mds_acc(const uint64_t* s, uint64_t& al, uint64_t& ah) {
  if constexpr (J < E) {
    constexpr uint32_t C = mds_coeff(I, J);
    al = madk<C>((uint32_t)s[J], al);
    ah = madk<C>((uint32_t)(s[J] >> 32), ah);
    mds_acc<I, J + 1, E>(s, al, ah);
  }
}
#if P2V_MDS_BRANCH == 2
// one row before its (rare) fix-up: r = t + ah_lo 2^32 with the carry-out mask c.  NW = 8: the
// row over words 0..7 only (the peeled round 0 of a zh permutation: words 8..11 folded into k)
template <int I, int NW = 12>
__device__ __forceinline__ void row_unfixed(const uint64_t* s, const uint64_t* kl, const uint64_t* kh, uint64_t& r, uint64_t& c) {
  using namespace gl::ax;
  constexpr uint32_t C = mds_coeff(I, 0);
  uint64_t al = madk_s<C>((uint32_t)s[0], kl[I]);
  uint64_t ah = madk_s<C>((uint32_t)(s[0] >> 32), kh[I]);
  mds_acc<I, 1, NW>(s, al, ah);
  uint64_t c0;
  const uint64_t t = madm1_co((uint32_t)(ah >> 32), al, c0);   // < 2^45: no carry
  const uint32_t rh = add_co((uint32_t)(t >> 32), (uint32_t)ah, c);
  r = ((uint64_t)rh << 32) | (uint32_t)t;
}
// rows I..I+3 with one uniform branch for the group's fix-ups (one basic block per group, so
// the compiler can batch the group's scalar constant loads)
template <int I, int NW = 12>
__device__ __forceinline__ void mds_group(const uint64_t* s, uint64_t* t, const uint64_t* kl, const uint64_t* kh) {
  using namespace gl::ax;
  uint64_t r0, r1, r2, r3, c0, c1, c2, c3, d;
  row_unfixed<I, NW>(s, kl, kh, r0, c0);
  row_unfixed<I + 1, NW>(s, kl, kh, r1, c1);
  row_unfixed<I + 2, NW>(s, kl, kh, r2, c2);
  row_unfixed<I + 3, NW>(s, kl, kh, r3, c3);
  if (__builtin_expect((c0 | c1 | c2 | c3) != 0, 0)) {
    r0 = madm1_co(mask_1(c0), r0, d);
    r1 = madm1_co(mask_1(c1), r1, d);
    r2 = madm1_co(mask_1(c2), r2, d);
    r3 = madm1_co(mask_1(c3), r3, d);
  }
  t[I] = r0; t[I + 1] = r1; t[I + 2] = r2; t[I + 3] = r3;
}
#endif
// t[I..E) = (M s)[I..E) + k (k = the next round's constants, split into halves)
template <int I, int E>
__device__ __forceinline__ void mds_rows(const uint64_t* s, uint64_t* t, const uint64_t* kl, const uint64_t* kh) {
#if P2V_POSEIDON_ASMBLK
  if constexpr (I < E) {
    t[I] = p2asm::mds_row<I>(s, kl[I], kh[I]);
    mds_rows<I + 1, E>(s, t, kl, kh);
  }
#else
  if constexpr (I < E) {
    constexpr uint32_t C = mds_coeff(I, 0);
    uint64_t al = madk_s<C>((uint32_t)s[0], kl[I]);
    uint64_t ah = madk_s<C>((uint32_t)(s[0] >> 32), kh[I]);
    mds_acc<I, 1>(s, al, ah);
    t[I] = reduce_rows(al, ah);
    mds_rows<I + 1, E>(s, t, kl, kh);
  }
#endif
}
__device__ __forceinline__ uint64_t sbox_dev(uint64_t x) {
#if P2V_POSEIDON_ASMBLK
  const uint64_t x2 = p2asm::mul_blk(x, x), x3 = p2asm::mul_blk(x, x2), x4 = p2asm::mul_blk(x2, x2);
  return p2asm::mul_blk(x3, x4);
#else
  return sbox(x);
#endif
}
// N independent S-boxes x -> x^7 in place, their products interleaved: each stage (x^2; x^3 and
// x^4; x^7) is one basic block of 1-2 N independent multiplies, and the rare -2^64 fix-up of
// all of them is one wave-uniform branch per stage (the per-multiply branch of p2::mul_nc made
// every multiply a basic block of its own: 11 dependent instructions the scheduler could not
// interleave with the next S-box's).  Round 4.
template <int N>
__device__ __forceinline__ void sbox_n(uint64_t* x) {
  uint64_t x2[N], x3[N], x4[N], n2[N], n3[N], n4[N];
#pragma unroll
  for (int i = 0; i < N; i++) x2[i] = gl::mul_nc_part(x[i], x[i], n2[i]);
  uint64_t any = 0;
#pragma unroll
  for (int i = 0; i < N; i++) any |= n2[i];
  if (__builtin_expect(any != 0, 0)) {
#pragma unroll
    for (int i = 0; i < N; i++) x2[i] = gl::mul_fix_neg(x2[i], n2[i]);
  }
#pragma unroll
  for (int i = 0; i < N; i++) { x3[i] = gl::mul_nc_part(x[i], x2[i], n3[i]); x4[i] = gl::mul_nc_part(x2[i], x2[i], n4[i]); }
  any = 0;
#pragma unroll
  for (int i = 0; i < N; i++) any |= n3[i] | n4[i];
  if (__builtin_expect(any != 0, 0)) {
#pragma unroll
    for (int i = 0; i < N; i++) { x3[i] = gl::mul_fix_neg(x3[i], n3[i]); x4[i] = gl::mul_fix_neg(x4[i], n4[i]); }
  }
#pragma unroll
  for (int i = 0; i < N; i++) x[i] = gl::mul_nc_part(x3[i], x4[i], n2[i]);
  any = 0;
#pragma unroll
  for (int i = 0; i < N; i++) any |= n2[i];
  if (__builtin_expect(any != 0, 0)) {
#pragma unroll
    for (int i = 0; i < N; i++) x[i] = gl::mul_fix_neg(x[i], n2[i]);
  }
}
#ifndef P2V_SBOX_ILP
#define P2V_SBOX_ILP 2   // S-boxes per interleaved group in the full rounds (sbox_n); 0: one p2::sbox per word
#endif
// the S-boxes of words [I, E) of a full round
template <int I, int E>
__device__ __forceinline__ void sbox_range(uint64_t* s) {
#if P2V_SBOX_ILP > 0
  if constexpr (I < E) {
    constexpr int K = (E - I) < P2V_SBOX_ILP ? (E - I) : P2V_SBOX_ILP;
    sbox_n<K>(s + I);
    sbox_range<I + K, E>(s);
  }
#else
#pragma unroll
  for (int i = I; i < E; i++) s[i] = sbox_dev(s[i]);
#endif
}
__device__ __forceinline__ uint64_t sbox_one(uint64_t x) {
#if P2V_SBOX_ILP > 0
  sbox_n<1>(&x);
  return x;
#else
  return sbox_dev(x);
#endif
}
// round r: s -> t (s is clobbered by the S-boxes); t = M sbox(s) + rc[r + 1].
// zh0: round 0 with state words 8..11 entering as 0 (their S-box outputs are constants).
// g: which groups of 4 output rows are needed (bit k = rows 4k..4k+3); wave-uniform.
template <bool FULL>
__device__ __forceinline__ void round_pp(uint64_t* s, uint64_t* t, int r, bool zh0, int g) {
  if (FULL) {
    sbox_range<0, 8>(s);
    if (zh0) {
#pragma unroll
      for (int i = 8; i < 12; i++) s[i] = c_zh.z[i - 8];
    } else {
      sbox_range<8, 12>(s);
    }
  } else {
    s[0] = sbox_one(s[0]);
  }
  const uint64_t* kl = c_rc_split.lo + 12 * (r + 1);
  const uint64_t* kh = c_rc_split.hi + 12 * (r + 1);
#if P2V_MDS_BRANCH == 2
  if (g & 1) mds_group<0>(s, t, kl, kh);
  if (g & 2) mds_group<4>(s, t, kl, kh);
  if (g & 4) mds_group<8>(s, t, kl, kh);
#else
  if (g & 1) mds_rows<0, 4>(s, t, kl, kh);
  if (g & 2) mds_rows<4, 8>(s, t, kl, kh);
  if (g & 4) mds_rows<8, 12>(s, t, kl, kh);
#endif
}

#if P2V_MDS_BRANCH == 2 && P2V_ZH_FOLD
// the peeled round 0 of a zh permutation: s -> t = M sbox(s) + rc[1] with s[8..11] = 0 + rc[0][8..11]
// never formed (their S-boxes and MDS columns are c_zrc); s[0..7] already hold + rc[0]
__device__ __forceinline__ void round0_zh(uint64_t* s, uint64_t* t) {
  sbox_range<0, 8>(s);
  mds_group<0, 8>(s, t, c_zrc.lo, c_zrc.hi);
  mds_group<4, 8>(s, t, c_zrc.lo, c_zrc.hi);
  mds_group<8, 8>(s, t, c_zrc.lo, c_zrc.hi);
}
#endif

// ---- merged partial rounds (see PBlock): coefficients are wave-uniform table entries (SGPR
// operands; gfx950 VOP3 takes no literal, and one SGPR per instruction, so the row's first
// MAD -- the one that takes the SGPR-pair constant as its addend -- is the newest y with its
// inline MDS entry)
__device__ __forceinline__ uint64_t madv(uint32_t a, uint32_t c, uint64_t acc) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, s[94:95], %1, %2, %3" : "=v"(d) : "v"(a), "s"(c), "v"(acc) : "s94", "s95");
  return d;
}
// al + 2^32 ah for row sums < 2^24 (D <= 3): as reduce_rows, the carry fix-up without a branch
__device__ __forceinline__ uint64_t reduce_t(uint64_t al, uint64_t ah) {
  using namespace gl::ax;
  uint64_t c0, c1, c2;
  const uint64_t t = madm1_co((uint32_t)(ah >> 32), al, c0);   // < 2^57: no carry
  const uint32_t rh = add_co((uint32_t)(t >> 32), (uint32_t)ah, c1);
  return madm1_co(mask_1(c1), ((uint64_t)rh << 32) | (uint32_t)t, c2);
}
// al + 2^32 ah for al, ah < 2^64 (D = 4): lo = al + ah_lo 2^32 (carry c), hi = ah_hi + c < 2^32,
// then lo + hi (2^32 - 1) with one wrap fix-up (the wrapped sum is < hi 2^32, no second wrap).  5 VALU.
__device__ __forceinline__ uint64_t reduce_w(uint64_t al, uint64_t ah) {
  using namespace gl::ax;
  uint64_t c0, c1, c2;
  const uint32_t lh = add_co((uint32_t)(al >> 32), (uint32_t)ah, c0);
  const uint32_t hi = addc0((uint32_t)(ah >> 32), c0);
  const uint64_t r = madm1_co(hi, ((uint64_t)lh << 32) | (uint32_t)al, c1);
  return madm1_co(mask_1(c1), r, c2);
}
// one row: (newest y) * CI + sum_j cf[j] s'_j + sum_m cf[12 + m] y_{m+2} + (dl, dh)
template <uint32_t CI, int NH>
__device__ __forceinline__ void prow(const uint64_t* s, const uint64_t* yh, uint64_t yn, const uint32_t* cf,
                                     uint64_t dl, uint64_t dh, uint64_t& al, uint64_t& ah) {
  al = madk_s<CI>((uint32_t)yn, dl);
  ah = madk_s<CI>((uint32_t)(yn >> 32), dh);
#pragma unroll
  for (int j = 0; j < 12; j++) {
    al = madv((uint32_t)s[j], cf[j], al);
    ah = madv((uint32_t)(s[j] >> 32), cf[j], ah);
  }
#pragma unroll
  for (int m = 0; m < NH; m++) {
    al = madv((uint32_t)yh[m], cf[12 + m], al);
    ah = madv((uint32_t)(yh[m] >> 32), cf[12 + m], ah);
  }
}
template <int D, int I>
__device__ __forceinline__ void pblock_rows(const uint64_t* s, const uint64_t* y, uint64_t* t, const PBlock& B) {
  if constexpr (I < 12) {
    uint64_t al, ah;
    prow<mds_coeff(I, 0), D - 2>(s, y + 2, y[D], B.cf[2 + I], B.dlo[4 + I], B.dhi[4 + I], al, ah);
    t[I] = D == 4 ? reduce_w(al, ah) : reduce_t(al, ah);
    pblock_rows<D, I + 1>(s, y, t, B);
  }
}
#if P2V_MDS_BRANCH == 2
// D = 2 output row before its (rare: ~2^-15) carry fix-up, as row_unfixed
template <int I>
__device__ __forceinline__ void prow2_unfixed(const uint64_t* s, uint64_t y2, const PBlock& B, uint64_t& r, uint64_t& c) {
  using namespace gl::ax;
  uint64_t al, ah, c0;
  prow<mds_coeff(I, 0), 0>(s, nullptr, y2, B.cf[2 + I], B.dlo[4 + I], B.dhi[4 + I], al, ah);
  const uint64_t tt = madm1_co((uint32_t)(ah >> 32), al, c0);   // < 2^49: no carry
  const uint32_t rh = add_co((uint32_t)(tt >> 32), (uint32_t)ah, c);
  r = ((uint64_t)rh << 32) | (uint32_t)tt;
}
template <int I>
__device__ __forceinline__ void pblock2_group(const uint64_t* s, uint64_t y2, uint64_t* t, const PBlock& B) {
  using namespace gl::ax;
  uint64_t r0, r1, r2, r3, c0, c1, c2, c3, d;
  prow2_unfixed<I>(s, y2, B, r0, c0);
  prow2_unfixed<I + 1>(s, y2, B, r1, c1);
  prow2_unfixed<I + 2>(s, y2, B, r2, c2);
  prow2_unfixed<I + 3>(s, y2, B, r3, c3);
  if (__builtin_expect((c0 | c1 | c2 | c3) != 0, 0)) {
    r0 = madm1_co(mask_1(c0), r0, d);
    r1 = madm1_co(mask_1(c1), r1, d);
    r2 = madm1_co(mask_1(c2), r2, d);
    r3 = madm1_co(mask_1(c3), r3, d);
  }
  t[I] = r0; t[I + 1] = r1; t[I + 2] = r2; t[I + 3] = r3;
}
#endif
// D partial rounds: s = the state entering the block's first round (its constants included),
// t = the state entering the round after the block.  s is clobbered.
template <int D>
__device__ __forceinline__ void pblock(uint64_t* s, uint64_t* t, const PBlock& B) {
  uint64_t y[D + 1];
  s[0] = sbox_one(s[0]);   // y1, word 0 of s'
  {   // chain row 1 (row 0 of M s' + d1): inline MDS entries
    uint64_t al = madk_s<mds_coeff(0, 0)>((uint32_t)s[0], B.dlo[0]);
    uint64_t ah = madk_s<mds_coeff(0, 0)>((uint32_t)(s[0] >> 32), B.dhi[0]);
    mds_acc<0, 1>(s, al, ah);
    y[2] = sbox_one(reduce_rows(al, ah));
  }
  if constexpr (D >= 3) {   // chain row 2: row sums < 2^16, the branch form of the fix-up
    uint64_t al, ah;
    prow<mds_coeff(0, 0), 0>(s, nullptr, y[2], B.cf[0], B.dlo[1], B.dhi[1], al, ah);
    y[3] = sbox_one(reduce_rows(al, ah));
  }
  if constexpr (D >= 4) {   // chain row 3: row sums < 2^24
    uint64_t al, ah;
    prow<mds_coeff(0, 0), 1>(s, y + 2, y[3], B.cf[1], B.dlo[2], B.dhi[2], al, ah);
    y[4] = sbox_one(reduce_t(al, ah));
  }
#if P2V_MDS_BRANCH == 2
  if constexpr (D == 2) {
    pblock2_group<0>(s, y[2], t, B);
    pblock2_group<4>(s, y[2], t, B);
    pblock2_group<8>(s, y[2], t, B);
    return;
  }
#endif
  pblock_rows<D, 0>(s, y, t, B);
}
}  // namespace dv

// Device permutation, one per lane.  zh: state words 8..11 are 0 on entry (2-to-1 compression,
// first sponge block).  gm: groups of 4 output words the caller reads (bit k = words
// 4k..4k+3); the others are left undefined.  Both wave-uniform.  Same function as
// Hash/Poseidon.hs:42-101, restructured for the gfx950 VALU:
//  * the round constant of round r+1 is folded into round r's MDS: each row's two 32-bit-half
//    accumulators START at the constant's halves (the first v_mad_u64_u32's addend), so
//    rounds 1..29 spend no instruction on constant addition;
//  * every MDS multiply-add is an explicit v_mad_u64_u32 with the matrix entry as an inline
//    constant;
//  * rounds alternate between two register sets (s -> t -> s), so no copies are needed at
//    loop edges; full rounds run as 4 pairs, the 22 partial rounds as merged blocks (PBlock,
//    P2V_PMERGE; 11 pairs of single rounds with P2V_PMERGE=0).
// FOLD: compile the peeled zh round 0 (P2V_ZH_FOLD) into this call site; false leaves it out where zh
// is never set (the leaf sponge's second block of a trip: with both of its call sites folded,
// k_phase1 spilled 8 B)
template <bool FOLD = true>
__device__ __forceinline__ void permute_dev(uint64_t s[12], bool zh = false, int gm = 7) {
  uint64_t t[12];
  // keep zh / gm run-time uniform values (uniform branches); as compile-time constants the
  // compiler peels loop iterations and the extra code raises register pressure
  int fl = __builtin_amdgcn_readfirstlane((zh ? 8 : 0) | gm);
  asm("" : "+s"(fl));
  zh = fl & 8;
  gm = fl & 7;
  // round 0's constants through an opaque pointer: a caller's loop must not hoist their loads
  // (with the merged partial rounds' table loads the SGPRs are full, and the hoisted values
  // would be spilled to VGPR lanes and read back with a VALU op each)
  const uint64_t* rc0 = c_round_constants;
  asm volatile("" : "+s"(rc0));
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = add_nc(s[i], rc0[i]);
  int k0 = 0;
#if P2V_MDS_BRANCH == 2 && P2V_ZH_FOLD
  // zh: rounds 0 and 1 peeled before the loop, round 0 over words 0..7 only (c_zrc); the loop body
  // stays the one generic full-round pair (a second round-0 form inside it spilled, round 5)
  if constexpr (FOLD) if (zh) {
    dv::round0_zh(s, t);
    dv::round_pp<true>(t, s, 1, false, 7);
    k0 = 1;
  }
#endif
  if (!zh) {
#pragma unroll
    for (int i = 8; i < 12; i++) s[i] = add_nc(s[i], rc0[i]);
  }
#pragma unroll 1
  for (int k = k0; k < 4; k++) {   // full-round pairs (0,1) (2,3) (26,27) (28,29)
    const int r = k < 2 ? 2 * k : 22 + 2 * k;
    dv::round_pp<true>(s, t, r, zh && k == 0, 7);   // (k == 0 with zh: only when not peeled)
    dv::round_pp<true>(t, s, r + 1, false, k == 3 ? gm : 7);
    if (k == 1) {
#if P2V_PMERGE == 4
      // blocks of 4, 4, 4, 4, 4, 2 merged partial rounds; each loop trip reads its own table
      // copies, so the coefficient loads stay inside the loop (no SGPR spills)
#pragma unroll 1
      for (int b = 0; b < 4; b += 2) {
        dv::pblock<4>(s, t, c_pm.b[b]);
        dv::pblock<4>(t, s, c_pm.b[b + 1]);
      }
      dv::pblock<4>(s, t, c_pm.b[4]);
      dv::pblock<2>(t, s, c_pm.b[5]);
#elif P2V_PMERGE == 3
#pragma unroll 1
      for (int b = 0; b < 6; b += 2) {
        dv::pblock<3>(s, t, c_pm.b[b]);
        dv::pblock<3>(t, s, c_pm.b[b + 1]);
      }
      dv::pblock<3>(s, t, c_pm.b[6]);
      dv::round_pp<false>(t, s, 25, false, 7);
#elif P2V_PMERGE == 2
#pragma unroll 1
      for (int b = 0; b < 10; b += 2) {
        dv::pblock<2>(s, t, c_pm.b[b]);
        dv::pblock<2>(t, s, c_pm.b[b + 1]);
      }
      dv::round_pp<false>(s, t, 24, false, 7);
      dv::round_pp<false>(t, s, 25, false, 7);
#else
#pragma unroll 1
      for (int q = 4; q < 26; q += 2) {   // partial-round pairs
        dv::round_pp<false>(s, t, q, false, 7);
        dv::round_pp<false>(t, s, q + 1, false, 7);
      }
#endif
    }
  }
  // canonical outputs for the groups the caller reads (the others are undefined: their last MDS
  // rows were not formed); a compression's 8 unread words no longer pay ~5 VALU each (round 6)
  if (gm & 1) {
#pragma unroll
    for (int i = 0; i < 4; i++) s[i] = gl::canon(s[i]);
  }
  if (gm & 2) {
#pragma unroll
    for (int i = 4; i < 8; i++) s[i] = gl::canon(s[i]);
  }
  if (gm & 4) {
#pragma unroll
    for (int i = 8; i < 12; i++) s[i] = gl::canon(s[i]);
  }
}
#elif defined(__HIPCC__)
template <bool FOLD = true>
__device__ void permute_dev(uint64_t s[12], bool zh = false, int gm = 7);   // device-only
namespace dv { template <uint32_t C> __device__ uint64_t madk(uint32_t a, uint64_t acc); }
#endif

// Hash/Poseidon.hs:42-46.  Inputs may be any value < 2^64; outputs are canonical.
__host__ __device__ __forceinline__ void permute(uint64_t s[12]) {
#if defined(__HIP_DEVICE_COMPILE__)
  permute_dev(s);
#else
  for (int r = 0; r < 4; r++) full_round(s, r);
  for (int r = 4; r < 26; r++) partial_round(s, r);
  for (int r = 26; r < 30; r++) full_round(s, r);
  P2_UNROLL
  for (int i = 0; i < 12; i++) s[i] = gl::canon(s[i]);
#endif
}

}  // namespace p2
