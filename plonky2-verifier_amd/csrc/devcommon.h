// devcommon.h — device helpers shared by the verifier kernels.
#pragma once
#include "gl.h"
#include "poseidon.h"
#include "dev.h"

namespace p2d {

using gl::E;

// Proof word w of lane p.  P2V_PROOF_MAJOR = 1 (default): the caller's proof-major batch
// [n][words] read in place, lanes past n re-reading the last proof; every lane streams its own
// proof's contiguous words, so the lines a load brings in serve the lane's next loads (measured:
// +3 % proofs/s against 0, the transposed batch [word][B] written by an extra k_transpose pass
// of 2 x 0.52 GB per 4 096 proofs, whose loads were coalesced 512-B rows)
#ifndef P2V_PROOF_MAJOR
#define P2V_PROOF_MAJOR 1
#endif
//
// c.tiled (P2V_FLAG_INPUT_TILED, wave-uniform): the caller's batch in 64-proof tiles
// [n/64][words][64], so the 64 lanes of a wave read one 512-B row per word: the same kernels with
// coalesced loads and no transpose pass, and HBM traffic at the algorithmic bytes.
// Both forms are affine in w, addr = base(p) + w * c.wstride (wstride 1 or 64, wave-uniform), so
// a kernel keeps one per-lane base and a scalar step, as the proof-major form alone did.
__device__ __forceinline__ uint64_t ld(const DevCircuit& c, int64_t w, int p) {
#if P2V_PROOF_MAJOR
  const int64_t q = min(p, c.n - 1);
  const int64_t base = c.tiled ? (((q >> 6) * c.words) << 6) + (q & 63) : q * c.words;
  return c.soa[base + w * c.wstride];
#else
  return c.soa[w * c.B + p];
#endif
}
__device__ __forceinline__ E lde(const DevCircuit& c, int64_t w, int p) { return E{ld(c, w, p), ld(c, w + 1, p)}; }
__device__ __forceinline__ uint64_t& chal(const DevCircuit& c, int64_t w, int p) { return c.chal[w * c.B + p]; }
__device__ __forceinline__ E chal_e(const DevCircuit& c, int64_t w, int p) { return E{c.chal[w * c.B + p], c.chal[(w + 1) * c.B + p]}; }

// subgroup_gen(k)^e  (Goldilocks.hs:68-74): product of the precomputed 2^j-th powers.
// e may differ per lane: multiply by 1 where the bit is clear (no divergence).
__device__ __forceinline__ uint64_t pow_root(const DevCircuit& c, int k, uint32_t e) {
  uint64_t acc = 1;
  for (int j = 0; j < k; j++) {
    uint64_t f = ((e >> j) & 1u) ? c.root_pow2[32 - k + j] : 1ULL;
    acc = gl::mul(acc, f);
  }
  return acc;
}

// x^(p-2) by an addition chain (64 squarings + 9 multiplies); inv(0) = 0 like the
// reference's pow-based inverse (Goldilocks.hs:155-156).
__device__ __forceinline__ uint64_t sqn(uint64_t v, int n) { for (int i = 0; i < n; i++) v = gl::mul(v, v); return v; }
__device__ __forceinline__ uint64_t inv_chain(uint64_t x) {
  uint64_t e2 = gl::mul(gl::mul(x, x), x);
  uint64_t e3 = gl::mul(gl::mul(e2, e2), x);
  uint64_t e6 = gl::mul(sqn(e3, 3), e3);
  uint64_t e12 = gl::mul(sqn(e6, 6), e6);
  uint64_t e24 = gl::mul(sqn(e12, 12), e12);
  uint64_t e30 = gl::mul(sqn(e24, 6), e6);
  uint64_t e31 = gl::mul(gl::mul(e30, e30), x);
  uint64_t z = gl::mul(gl::mul(e31, e31), x);
  return gl::mul(sqn(e31, 33), z);
}
__device__ __forceinline__ uint64_t norm(E x) { return gl::sub(gl::mul(x.a, x.a), gl::mul_small(gl::mul(x.b, x.b), 7)); }
__device__ __forceinline__ E einv(E x) {   // invExt, GoldilocksExt.hs:76-80
  uint64_t d = inv_chain(norm(x));
  return E{gl::mul(x.a, d), gl::mul(gl::neg(x.b), d)};
}
// 1/u and 1/v with one base-field inversion; exact inv(0)=0 semantics kept by a fallback
__device__ __forceinline__ void einv2(E u, E v, E& iu, E& iv) {
  uint64_t nu = norm(u), nv = norm(v);
  uint64_t nuv = gl::mul(nu, nv);
  if (nuv != 0) {
    uint64_t t = inv_chain(nuv);
    uint64_t inu = gl::mul(t, nv), inv_ = gl::mul(t, nu);
    iu = E{gl::mul(u.a, inu), gl::mul(gl::neg(u.b), inu)};
    iv = E{gl::mul(v.a, inv_), gl::mul(gl::neg(v.b), inv_)};
  } else {
    iu = einv(u); iv = einv(v);
  }
}
__device__ __forceinline__ E epow_u(E x, uint32_t e) {   // uniform small exponent
  E acc = gl::eb(1), s = x;
  while (e) { if (e & 1) acc = gl::emul(acc, s); s = gl::emul(s, s); e >>= 1; }
  return acc;
}
__device__ __forceinline__ E epow2n(E x, int n) { for (int i = 0; i < n; i++) x = gl::emul(x, x); return x; }

}  // namespace p2d
