// gl.h — Goldilocks field p = 2^64 - 2^32 + 1 and its quadratic extension F[X]/(X^2-7),
// shared by host C++ and the gfx950 device code.
//
// Semantics follow the reference (src/Algebra/Goldilocks.hs:126-175,
// src/Algebra/GoldilocksExt.hs:54-100): every public operation returns the canonical
// representative in [0, p); inv(0) = 0 (the reference computes inv as x^(p-2)).
//
// Device multiply: a 64x64 product is built from 32x32->64 partial products
// (v_mad_u64_u32) and reduced with 2^64 = 2^32 - 1 (mod p), 2^96 = -1 (mod p).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GL_HD __host__ __device__ __forceinline__
#else
#define GL_HD static inline
#ifndef __host__
#define __host__
#define __device__
#define __forceinline__ inline __attribute__((always_inline))
#endif
#endif

namespace gl {

static constexpr uint64_t P = 0xFFFFFFFF00000001ULL;
static constexpr uint64_t EPS = 0xFFFFFFFFULL;           // 2^64 mod p
static constexpr uint64_t MULT_GEN = 0xc65c18b67785d900ULL;      // Goldilocks.hs:51-52
static constexpr uint64_t TWO_ADIC_GEN = 0x64fdd1a46201e246ULL;  // Goldilocks.hs:55-56

GL_HD uint64_t canon(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return x >= P ? x - P : x;
#else
  uint64_t y; bool b = __builtin_sub_overflow(x, P, &y);
  return b ? x : y;
#endif
}

// (hi:lo) 128-bit value -> [0, 2^64) congruent mod p (not necessarily canonical)
GL_HD uint64_t reduce128_nc(uint64_t hi, uint64_t lo) {
  uint64_t hi_hi = hi >> 32;
  uint64_t hi_lo = hi & EPS;
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t t0 = lo - hi_hi;
  if (lo < hi_hi) t0 -= EPS;
  uint64_t t1 = (hi_lo << 32) - hi_lo;
  uint64_t r = t0 + t1;
  if (r < t1) r += EPS;
#else
  uint64_t t0, r;
  bool br = __builtin_sub_overflow(lo, hi_hi, &t0);
  t0 -= EPS & (0 - (uint64_t)br);
  uint64_t t1 = (hi_lo << 32) - hi_lo;
  bool cy = __builtin_add_overflow(t0, t1, &r);
  r += EPS & (0 - (uint64_t)cy);
#endif
  return r;
}
GL_HD uint64_t reduce128(uint64_t hi, uint64_t lo) { return canon(reduce128_nc(hi, lo)); }

// hi < 2^32: value hi*2^64 + lo
GL_HD uint64_t reduce96_nc(uint64_t hi, uint64_t lo) {
  uint64_t t1 = (hi << 32) - hi;
  uint64_t r = lo + t1;
  if (r < t1) r += EPS;
  return r;
}

#ifndef P2V_MUL_CMAD
#define P2V_MUL_CMAD 1   // the product's carry-free MADs in plain C (no inline-asm SGPR outputs)
#endif
#ifndef P2V_MUL_PRODUCT
#define P2V_MUL_PRODUCT 1   // device multiply's partial products: 1 = chained MAD addends (round 4), 0 = carry adds
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// gfx950 carry-chain primitives.  The compiler does not use the carry-out of
// v_mad_u64_u32 / v_add_co_u32 and re-derives every carry with a 64-bit compare; these
// wrappers expose the hardware carry (an SGPR-pair lane mask).  They are plain (non-volatile)
// asm, so the scheduler still interleaves them, and it inserts the SGPR write->read hazard
// waits between them itself.
namespace ax {
__device__ __forceinline__ uint64_t mad0(uint32_t a, uint32_t b) { uint64_t d, c; asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(d), "=s"(c) : "v"(a), "v"(b)); return d; }
__device__ __forceinline__ uint64_t mad_co(uint32_t a, uint32_t b, uint64_t x, uint64_t& co) { uint64_t d; asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(co) : "v"(a), "v"(b), "v"(x)); return d; }
// a b + x where the caller guarantees no carry out of 64 bits
__device__ __forceinline__ uint64_t mad_nc(uint32_t a, uint32_t b, uint64_t x) { uint64_t co; return mad_co(a, b, x, co); }
__device__ __forceinline__ uint64_t madm1_co(uint32_t a, uint64_t x, uint64_t& co) { uint64_t d; asm("v_mad_u64_u32 %0, %1, %2, -1, %3" : "=v"(d), "=s"(co) : "v"(a), "v"(x)); return d; }
__device__ __forceinline__ uint32_t add_co(uint32_t a, uint32_t b, uint64_t& co) { uint32_t d; asm("v_add_co_u32_e64 %0, %1, %2, %3" : "=v"(d), "=s"(co) : "v"(a), "v"(b)); return d; }
__device__ __forceinline__ uint32_t addc_co(uint32_t a, uint32_t b, uint64_t ci, uint64_t& co) { uint32_t d; asm("v_addc_co_u32_e64 %0, %1, %2, %3, %4" : "=v"(d), "=s"(co) : "v"(a), "v"(b), "s"(ci)); return d; }
__device__ __forceinline__ uint32_t addc0(uint32_t a, uint64_t ci) { uint32_t d; uint64_t co; asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(d), "=s"(co) : "v"(a), "s"(ci)); return d; }
__device__ __forceinline__ uint32_t sub_co(uint32_t a, uint32_t b, uint64_t& co) { uint32_t d; asm("v_sub_co_u32_e64 %0, %1, %2, %3" : "=v"(d), "=s"(co) : "v"(a), "v"(b)); return d; }
__device__ __forceinline__ uint32_t subb_co(uint32_t a, uint32_t b, uint64_t ci, uint64_t& co) { uint32_t d; asm("v_subb_co_u32_e64 %0, %1, %2, %3, %4" : "=v"(d), "=s"(co) : "v"(a), "v"(b), "s"(ci)); return d; }
__device__ __forceinline__ uint32_t subb0_co(uint32_t a, uint64_t ci, uint64_t& co) { uint32_t d; asm("v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(d), "=s"(co) : "v"(a), "s"(ci)); return d; }
__device__ __forceinline__ uint32_t mask_m1(uint64_t m) { uint32_t d; asm("v_cndmask_b32_e64 %0, 0, -1, %1" : "=v"(d) : "s"(m)); return d; }
__device__ __forceinline__ uint32_t sel(uint32_t a, uint32_t b, uint64_t m) { uint32_t d; asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(m)); return d; }
__device__ __forceinline__ uint64_t add64(uint64_t a, uint64_t b) { uint64_t d; asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(d) : "v"(a), "v"(b)); return d; }
__device__ __forceinline__ uint32_t mask_1(uint64_t m) { uint32_t d; asm("v_cndmask_b32_e64 %0, 0, 1, %1" : "=v"(d) : "s"(m)); return d; }
}  // namespace ax

// a * b (mod p) for any a, b < 2^64, result in [0, 2^64) (not necessarily canonical).
// 4 partial products; the 128-bit product lo + h0 2^64 + h1 2^96 through the carry chain,
// where the carry cm of the middle sum a0 b1 + a1 b0 (weight 2^96) is not added into h1 but
// enters the subtraction of h1 as its borrow-in; then lo + h0 (2^32 - 1) - h1
// (2^64 == 2^32 - 1, 2^96 == -1 mod p) and the wrap fix-ups.  V selects the fix-up form:
//   V = 1: one fix-up for the net wrap (14 VALU), branch-free: the general multiply;
//   V = 2: the common +2^64 wrap by one MAD, the rare -2^64 wrap in a wave-uniform branch
//          (12 VALU when not taken): the Poseidon S-box (p2::mul_nc);
//   V = 0: one fix-up per wrap (16 VALU), the first form, kept for measurement.
template <int V = 1>
__device__ __forceinline__ uint64_t mul_nc_dev_v(uint64_t a, uint64_t b, uint64_t& negm) {
  using namespace ax;
  const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  uint64_t cm, c1, c2, ct, c4, bw1, bw2, bw3, bw4;
#if P2V_MUL_PRODUCT == 1
  // the partial products chained through the MADs' 64-bit addends: every carry between the
  // 32-bit columns is absorbed by the next MAD, so no add-with-carry is needed
  //   x = a0 b1 + hi(a0 b0)          <= (2^32-1)^2 + 2^32 - 2 < 2^64
  //   y = a1 b0 + x = y + cm 2^64    (the column of weight 2^32; cm has weight 2^96)
  //   h = a1 b1 + hi(y)              <= (2^32-1)^2 + 2^32 - 1 < 2^64
  // product = lo(a0 b0) + lo(y) 2^32 + h 2^64 + cm 2^96: 4 MADs and 2 zero-extensions against
  // 4 MADs and 3 carry adds (round 4)
  (void)c1; (void)c2;
#if P2V_MUL_CMAD
  // the MADs whose carry-out is not needed in plain C: the compiler emits the same
  // v_mad_u64_u32 and, unlike after an inline-asm SGPR output, knows no wait state is needed
  const uint64_t p00 = (uint64_t)a0 * b0;
  const uint64_t x = (uint64_t)a0 * b1 + (p00 >> 32);
  const uint64_t y = mad_co(a1, b0, x, cm);
  const uint64_t hh = (uint64_t)a1 * b1 + (y >> 32);
#else
  const uint64_t p00 = mad0(a0, b0);
  const uint64_t x = mad_nc(a0, b1, p00 >> 32);
  const uint64_t y = mad_co(a1, b0, x, cm);
  const uint64_t hh = mad_nc(a1, b1, y >> 32);
#endif
  const uint32_t h0 = (uint32_t)hh, h1 = (uint32_t)(hh >> 32);          // + cm: below
  const uint64_t lo = ((uint64_t)(uint32_t)y << 32) | (uint32_t)p00;
#else
  const uint64_t p00 = mad0(a0, b0);
  const uint64_t p01 = mad0(a0, b1);
  const uint64_t m = mad_co(a1, b0, p01, cm);   // a0 b1 + a1 b0 = m + cm 2^64
  const uint64_t p11 = mad0(a1, b1);
  const uint32_t lo1 = add_co((uint32_t)(p00 >> 32), (uint32_t)m, c1);
  const uint32_t h0 = addc_co((uint32_t)p11, (uint32_t)(m >> 32), c1, c2);
  const uint32_t h1 = addc0((uint32_t)(p11 >> 32), c2);                 // + cm: below
  const uint64_t lo = ((uint64_t)lo1 << 32) | (uint32_t)p00;
#endif
  if constexpr (V == 2 || V == 3) {
  // as below, but the -2^64 case (only when the product has bits 64..95 zero and bits 0..63
  // below 2^32, e.g. powers of two) is a wave-uniform branch that is almost never taken.
  // V = 3: no branch here; the caller receives the lanes that still need it (mul_nc_part)
  (void)c4; (void)bw3; (void)bw4;
  const uint64_t t = madm1_co(h0, lo, ct);
  const uint32_t ul = subb_co((uint32_t)t, h1, cm, bw1);
  const uint32_t uh = subb0_co((uint32_t)(t >> 32), bw1, bw2);
  const uint64_t pos = ct & ~bw2, neg = bw2 & ~ct;
  uint64_t r = madm1_co(mask_1(pos), ((uint64_t)uh << 32) | ul, c4);
  if constexpr (V == 3) { negm = neg; return r; }
  if (__builtin_expect(neg != 0, 0)) r = add64(r, ((uint64_t)mask_m1(neg) << 32) | sel(0u, 1u, neg));
  return r;
  } else if constexpr (V == 1) {
  // lo + h0 (2^32 - 1) - (h1 + cm) = u + (c - b) 2^64 with the carry c of the MAD and the
  // borrow b of the subtraction; one fix-up for the net wrap: +2^64 == + (2^32 - 1), and
  // -2^64 == + p (mod 2^64 arithmetic), both without a second wrap.
  (void)c4; (void)bw2; (void)bw3; (void)bw4;
  const uint64_t t = madm1_co(h0, lo, ct);
  const uint32_t ul = subb_co((uint32_t)t, h1, cm, bw1);
  const uint32_t uh = subb0_co((uint32_t)(t >> 32), bw1, bw2);
  const uint64_t pos = ct & ~bw2, neg = bw2 & ~ct;
  const uint32_t kl = sel(sel(0u, 1u, neg), 0xFFFFFFFFu, pos);
  const uint32_t kh = mask_m1(neg);
  return add64(((uint64_t)uh << 32) | ul, ((uint64_t)kh << 32) | kl);
  } else {
  const uint64_t t = madm1_co(h0, lo, ct);                              // lo + h0 (2^32 - 1)
  const uint32_t tl = add_co((uint32_t)t, mask_m1(ct), c4);             // wrapped: + 2^32 - 1
  const uint32_t th = addc0((uint32_t)(t >> 32), c4);
  const uint32_t rl = subb_co(tl, h1, cm, bw1);                         // - (h1 + cm) < 2^32
  const uint32_t rh = subb0_co(th, bw1, bw2);
  const uint32_t rl2 = sub_co(rl, mask_m1(bw2), bw3);                   // wrapped: - (2^32 - 1)
  const uint32_t rh2 = subb0_co(rh, bw3, bw4);
  return ((uint64_t)rh2 << 32) | rl2;
  }
}
template <int V = 1>
__device__ __forceinline__ uint64_t mul_nc_dev_v(uint64_t a, uint64_t b) { uint64_t n; return mul_nc_dev_v<V>(a, b, n); }
// the S-box form without its rare branch: r, and in `neg` the lanes whose product wrapped below
// 0 (r is then 2^64 too small); mul_fix_neg adds it back (+2^64 == +(2^32 - 1) mod p, as
// 2^64 - 2^32 + 1 mod 2^64).  A caller merges the branches of independent products into one.
__device__ __forceinline__ uint64_t mul_nc_part(uint64_t a, uint64_t b, uint64_t& neg) { return mul_nc_dev_v<3>(a, b, neg); }
__device__ __forceinline__ uint64_t mul_fix_neg(uint64_t r, uint64_t neg) {
  using namespace ax;
  return add64(r, ((uint64_t)mask_m1(neg) << 32) | sel(0u, 1u, neg));
}
// the general-purpose multiply (FRI, vanishing, gates): the branch-free one-fix-up form.  (The
// round-1 build option that put the branch form V = 2 here is gone: it was slower, and the one
// fault seen under it was never reproduced; V = 2 stays the S-box's form)
__device__ __forceinline__ uint64_t mul_nc_dev(uint64_t a, uint64_t b) { return mul_nc_dev_v<1>(a, b); }
#endif

GL_HD void mul128(uint64_t a, uint64_t b, uint64_t& hi, uint64_t& lo) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  uint64_t p00 = (uint64_t)a0 * b0;
  uint64_t p01 = (uint64_t)a0 * b1 + (p00 >> 32);          // < 2^64
  uint64_t p10 = (uint64_t)a1 * b0 + (uint32_t)p01;        // < 2^64
  lo = (p10 << 32) | (uint32_t)p00;
  hi = (uint64_t)a1 * b1 + (p01 >> 32) + (p10 >> 32);
#else
  unsigned __int128 t = (unsigned __int128)a * b;
  lo = (uint64_t)t; hi = (uint64_t)(t >> 64);
#endif
}

GL_HD uint64_t add(uint64_t a, uint64_t b) {   // a, b canonical
  uint64_t s = a + b;
  uint64_t r = s + ((s < a) ? EPS : 0);          // wrapped: +2^64 == +EPS
  return canon(r);
}
GL_HD uint64_t sub(uint64_t a, uint64_t b) {   // a, b canonical
  uint64_t d = a - b;
  return (a < b) ? d + P : d;
}
GL_HD uint64_t neg(uint64_t a) { return a ? P - a : 0; }
GL_HD uint64_t mul(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return canon(mul_nc_dev(a, b));
#else
  uint64_t hi, lo; mul128(a, b, hi, lo); return reduce128(hi, lo);
#endif
}
GL_HD uint64_t sqr(uint64_t a) { return mul(a, a); }
// multiply by a small constant c < 2^32
GL_HD uint64_t mul_small(uint64_t a, uint32_t c) {
  uint64_t lo = (uint64_t)(uint32_t)a * c;
  uint64_t hi = (a >> 32) * (uint64_t)c;           // < 2^64
  uint64_t l = lo + (hi << 32);
  uint64_t h = (hi >> 32) + (l < lo ? 1 : 0);
  return canon(reduce96_nc(h, l));
}
GL_HD uint64_t pow(uint64_t x, uint64_t e) {
  uint64_t acc = 1, s = x;
  while (e) { if (e & 1) acc = mul(acc, s); s = mul(s, s); e >>= 1; }
  return acc;
}
GL_HD uint64_t inv(uint64_t x) { return pow(x, P - 2); }   // inv(0) = 0, as the reference

// rootsOfUnity!k, Goldilocks.hs:68-74
GL_HD uint64_t subgroup_gen(int k) {
  uint64_t x = TWO_ADIC_GEN;
  for (int i = 0; i < 32 - k; i++) x = mul(x, x);
  return x;
}

GL_HD uint32_t rev_bits(int n, uint32_t w) {
#if defined(__HIP_DEVICE_COMPILE__)
  return n ? (__brev(w) >> (32 - n)) : 0;
#else
  uint32_t r = 0;
  for (int k = 0; k < n; k++) r |= ((w >> k) & 1u) << (n - k - 1);
  return r;
#endif
}

// ---------------------------------------------------------------- F^2 = F[X]/(X^2-7)
struct E { uint64_t a, b; };
GL_HD E e0() { return E{0, 0}; }
GL_HD E eb(uint64_t x) { return E{x, 0}; }
GL_HD E eadd(E x, E y) { return E{add(x.a, y.a), add(x.b, y.b)}; }
GL_HD E esub(E x, E y) { return E{sub(x.a, y.a), sub(x.b, y.b)}; }
GL_HD E eneg(E x) { return E{neg(x.a), neg(x.b)}; }
GL_HD E escale(uint64_t s, E x) { return E{mul(s, x.a), mul(s, x.b)}; }
GL_HD bool eeq(E x, E y) { return x.a == y.a && x.b == y.b; }
GL_HD E emul(E x, E y) {
  // (a + bX)(c + dX) = (ac + 7bd) + (ad + bc)X, lazily reduced: one reduction per limb
  uint64_t h0, l0, h1, l1, h2, l2, h3, l3;
  mul128(x.a, y.a, h0, l0);
  mul128(x.b, y.b, h1, l1);
  uint64_t bd = reduce128_nc(h1, l1);            // < 2^64
  // ac + 7*bd as 128-bit
  uint64_t s7l = (uint64_t)(uint32_t)bd * 7, s7h = (bd >> 32) * 7;
  uint64_t t7 = s7l + (s7h << 32); uint64_t c7 = (s7h >> 32) + (t7 < s7l ? 1 : 0);
  uint64_t ra = l0 + t7; uint64_t rh = h0 + c7 + (ra < l0 ? 1 : 0);
  mul128(x.a, y.b, h2, l2);
  mul128(x.b, y.a, h3, l3);
  uint64_t rb = l2 + l3; uint64_t rbh = h2 + h3 + (rb < l2 ? 1 : 0);   // h2+h3 < 2^64 since hi < 2^64-1 each... see note
  // note: h2,h3 <= 2^64-2 each; their sum may wrap.  Keep a third word.
  uint64_t rbhh = (rbh < h2) ? 1 : 0;
  if (rbhh) { // 2^128 = (2^64)^2 = EPS^2 mod p ; fold: add EPS^2 mod p = 0xfffffffe00000001 (2^64-2^33+1)
    uint64_t f = 0xFFFFFFFE00000001ULL;
    uint64_t r2 = rb + f; rbh += (r2 < rb ? 1 : 0); rb = r2;
  }
  return E{reduce128(rh, ra), reduce128(rbh, rb)};
}
GL_HD E esqr(E x) { return emul(x, x); }
GL_HD E einv(E x) {   // invExt: conj / norm, norm = a^2 - 7b^2; 0 -> 0
  uint64_t n = sub(mul(x.a, x.a), mul_small(mul(x.b, x.b), 7));
  uint64_t d = inv(n);
  return E{mul(x.a, d), mul(neg(x.b), d)};
}
GL_HD E ediv(E u, E v) { return emul(u, einv(v)); }
GL_HD E epow(E x, uint64_t e) {
  E acc = eb(1), s = x;
  while (e) { if (e & 1) acc = emul(acc, s); s = emul(s, s); e >>= 1; }
  return acc;
}

}  // namespace gl
