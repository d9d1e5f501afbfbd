// vanish.hip — the Plonk-identity kernels other than the PoseidonGate parts (those are in
// vanish_poseidon.hip): the lookup-table pieces, the coset-interpolation and misc item classes,
// and the final sum with the quotient check.  The device programs are in vanish.h.
#include "vanish.h"

using namespace p2d;
using gl::E;

// evalFinalRE pieces: one wave = (challenge round j, piece, 64 proofs)
extern "C" __global__ void __launch_bounds__(256) k_lut(DevCircuit c) {
  const int lane = threadIdx.x & 63;
  const int unit = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int NPB = c.B >> 6;
  if (unit >= c.r * c.n_lut_pieces * NPB) return;
  __builtin_amdgcn_s_setprio(2);   // side stream, concurrent with k_merkle (see k_vanish)
  const int jp = unit / NPB, p = (unit % NPB) * 64 + lane;
  const int j = jp / c.n_lut_pieces, pi = jp % c.n_lut_pieces;
  int k = 0;
  while (c.lut_pbase[k + 1] <= pi) k++;
  const int s2 = pi - c.lut_pbase[k];
  const int c0 = s2 * P2V_LUT_PIECE, c1 = min(c0 + P2V_LUT_PIECE, (int)c.lut_rchunks[k]);
  const uint64_t dB = chal(c, CH_DELTA(c) + 4 * j + 1, p), dde = chal(c, CH_DELTA(c) + 4 * j + 3, p);
  c.lutpart[(int64_t)jp * c.B + p] = lut_piece(c, k, c0, c1, dde, dB);
}

// the vanishing kernels of the coset and misc classes, for r = 2 (_r2) and generic r <= P2V_MAX_R
// (the host picks by the circuit's r); one-wave work-groups.  They run beside k_merkle (6 waves
// per SIMD at 80 VGPRs): a wave of theirs fits where one k_merkle wave retired only at <= 112
// VGPRs, and the register budgets a build can request are 128 (4 waves) or 96 (5), so 5
// (P2V_SIDE_WAVES; the programs' own register fences, vanish.h pin/pinm, bring them near that
// budget).  The lookup items have a kernel of their own, launched only for circuits with lookup
// tables.
#ifndef P2V_SIDE_WAVES
#define P2V_SIDE_WAVES 5
#endif
#define P2V_SIDE_ATTR __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(P2V_SIDE_WAVES)))
extern "C" __global__ void P2V_SIDE_ATTR k_vanish_coset_r2(DevCircuit c) { vanish_body<VK_COSET, P2V_R_STD>(c); }
extern "C" __global__ void P2V_SIDE_ATTR k_vanish_coset_rn(DevCircuit c) { vanish_body<VK_COSET, P2V_MAX_R>(c); }
extern "C" __global__ void P2V_SIDE_ATTR k_vanish_r2(DevCircuit c) { vanish_body<VK_MISC, P2V_R_STD>(c); }
extern "C" __global__ void P2V_SIDE_ATTR k_vanish_rn(DevCircuit c) { vanish_body<VK_MISC, P2V_MAX_R>(c); }
// the lookup items (lookup circuits only) under the same cap (round 4, VERDICT r3 item 3: at the
// compiler's 154 VGPRs their waves could not start beside k_merkle); P2V_LOOKUP_WAVES=0 lifts it
#ifndef P2V_LOOKUP_WAVES
#define P2V_LOOKUP_WAVES P2V_SIDE_WAVES
#endif
#if P2V_LOOKUP_WAVES > 0
#define P2V_LOOKUP_ATTR __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(P2V_LOOKUP_WAVES)))
#else
#define P2V_LOOKUP_ATTR __launch_bounds__(64)
#endif
extern "C" __global__ void P2V_LOOKUP_ATTR k_vanish_lookup_r2(DevCircuit c) { vanish_body<VK_LOOKUP, P2V_R_STD>(c); }
extern "C" __global__ void P2V_LOOKUP_ATTR k_vanish_lookup_rn(DevCircuit c) { vanish_body<VK_LOOKUP, P2V_MAX_R>(c); }

// sum of the item partials, then Q(zeta)(zeta^n - 1) == C(zeta), Plonk/Verifier.hs:35-51
// (one-wave work-groups, like the other side-stream kernels: a wave fits where one k_merkle wave retired)
extern "C" __global__ void __launch_bounds__(256) k_vanish_final(DevCircuit c) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= c.B) return;
  const int r = c.r;
  const E one = gl::eb(1);
  const E zeta_n = epow2n(chal_e(c, CH_ZETA(c), p), c.degree_bits);
  const E zn1 = gl::esub(zeta_n, one);
  bool ok = true;
  for (int i = 0; i < r; i++) {
    E h = gl::e0();
    for (int it = 0; it < c.n_vitems; it++) {
      const uint64_t* src = c.vparts + ((int64_t)it * 2 * r + 2 * i) * c.B + p;
      h = gl::eadd(h, E{src[0], src[c.B]});
    }
    E q = gl::e0();
    for (int k = c.qdf - 1; k >= 0; k--) q = gl::eadd(gl::emul(q, zeta_n), lde(c, c.o_quot + 2 * ((int64_t)i * c.qdf + k), p));
    ok = ok && gl::eeq(gl::emul(q, zn1), h);
    c.van[(int64_t)(1 + 2 * i) * c.B + p] = h.a;
    c.van[(int64_t)(2 + 2 * i) * c.B + p] = h.b;
    c.van[(int64_t)(1 + 2 * r + 2 * i) * c.B + p] = q.a;
    c.van[(int64_t)(2 + 2 * r + 2 * i) * c.B + p] = q.b;
  }
  c.van[p] = ok ? 1 : 0;
}
