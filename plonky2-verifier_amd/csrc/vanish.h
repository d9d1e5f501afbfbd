// vanish.h — the Plonk-identity kernels (vanish.hip, vanish_poseidon.hip): one lane per proof evaluates every vanishing term
// at zeta (Plonk/Vanishing.hs:48-137): Z(1) boundary terms, partial-product transitions,
// lookup terms (Plonk/Lookups.hs:45-132) and the filtered gate constraints of every gate
// in the circuit (Gate/Constraints.hs:40-128, Gate/Custom/*), combined with powers of the
// base-field alphas, then checks Q(zeta)(zeta^n - 1) = C(zeta) (Plonk/Verifier.hs:35-51).
//
// The gate list is uniform across the batch (all proofs share the circuit), so the gate
// loop is a wave-uniform interpreter at gate granularity: each gate kind is hand-written
// device code with its (runtime, uniform) parameters.  Instead of materialising the
// vertically-summed constraint vector (Vanishing.hs:124-125) each gate's constraints are
// folded into the running alpha-combination directly: sum_k a^(G0+k) sum_g s_g c_gk ==
// sum_g s_g a^G0 sum_k a^k c_gk — the same field element, exact arithmetic.
#pragma once
#include "devcommon.h"

using namespace p2d;
using gl::E;

namespace {

// "doubly extended" values: Ext over Expr evaluated in F^2 (Gate/Vars.hs:56-57); the 7 of
// X^2 = 7 is the literal LitE 7 (GoldilocksExt.hs:54-61).
struct EE { E re, im; };
__device__ __forceinline__ EE ee_add(EE x, EE y) { return EE{gl::eadd(x.re, y.re), gl::eadd(x.im, y.im)}; }
__device__ __forceinline__ EE ee_sub(EE x, EE y) { return EE{gl::esub(x.re, y.re), gl::esub(x.im, y.im)}; }
__device__ __forceinline__ E e_mul7(E x) { return E{gl::mul_small(x.a, 7), gl::mul_small(x.b, 7)}; }
__device__ __forceinline__ EE ee_mul(EE x, EE y) {
  return EE{gl::eadd(gl::emul(x.re, y.re), e_mul7(gl::emul(x.im, y.im))), gl::eadd(gl::emul(x.re, y.im), gl::emul(y.re, x.im))};
}
__device__ __forceinline__ EE ee_scale(E s, EE x) { return EE{gl::emul(s, x.re), gl::emul(s, x.im)}; }
__device__ __forceinline__ EE ee_base(E x) { return EE{x, gl::e0()}; }
__device__ __forceinline__ E lit(uint64_t x) { return gl::eb(x); }

// compile-time loop: f(integral_constant<int, I>) for I in [B, N).  The PoseidonGate programs
// index their 12-word states only through these, so every index is a constant and the state
// stays in registers (a partially unrolled `for` left them in scratch memory).
template <int B, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < N) { f(std::integral_constant<int, B>{}); sfor<B + 1, N>(f); }
}

// running sum_k alpha_i^k t_k for every challenge round i < r.  R = P2V_MAX_R is the generic
// form (r <= R at run time); R < P2V_MAX_R holds exactly R rounds, known at compile time (the
// kernels for the standard r = 2), so that only R accumulators occupy registers.
template <int R>
struct Acc {
  E h[R];
  uint64_t pw[R];
  uint64_t al[R];
  int r;
  __device__ __forceinline__ bool on(int i) const { return R < P2V_MAX_R || i < r; }
  __device__ __forceinline__ void push(E t) {
#pragma unroll
    for (int i = 0; i < R; i++)
      if (on(i)) { h[i] = gl::eadd(h[i], gl::escale(pw[i], t)); pw[i] = gl::mul(pw[i], al[i]); }
  }
  __device__ __forceinline__ void pushx(EE t) { push(t.re); push(t.im); }   // commitExt
};

struct Vars {
  const DevCircuit* c;
  int p;
  __device__ __forceinline__ E w(int64_t i) const { return lde(*c, c->o_wires + 2 * i, p); }
  __device__ __forceinline__ EE wx(int64_t i) const { return EE{w(i), w(i + 1)}; }
  __device__ __forceinline__ E k(int64_t i) const { return lde(*c, c->o_const + 2 * (c->ngroups + c->nls + i), p); }
};

// register-pressure fences.  pin: a value computed before it stays computed before it (IR passes
// may not sink it past the asm; the scheduler may not move work across the barrier).  pinm: the
// same, and memory operations stay on their side too (later loads are not hoisted above it).
// The side-stream kernels must fit where one k_merkle wave retired (<= 112 VGPRs, vanish.hip).
__device__ __forceinline__ void pin(E& x) {
  asm volatile("" : "+v"(x.a), "+v"(x.b));
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void pinm(E& x) {
  asm volatile("" : "+v"(x.a), "+v"(x.b) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void pinm64(uint64_t& x) {
  asm volatile("" : "+v"(x) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void pinm2(E& x, E& y) {
  asm volatile("" : "+v"(x.a), "+v"(x.b), "+v"(y.a), "+v"(y.b) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ E esbox(E x) { E x2 = gl::emul(x, x); E x3 = gl::emul(x, x2); E x4 = gl::emul(x2, x2); return gl::emul(x3, x4); }

// PoseidonGate (Gate/Custom/Poseidon.hs:63-150), part `part` of 8: defined in
// vanish_poseidon.hip, the only translation unit that instantiates the Poseidon class
template <int R>
__device__ void gate_poseidon(const Vars& V, Acc<R>& A, int part);

// CosetInterpolationGate, Gate/Custom/CosetInterp.hs:51-121
template <class A_>
__device__ __forceinline__ void gate_coset(const DevCircuit& c, const Vars& V, A_& A, int bits, int64_t degree, const uint64_t* weights, int nweights,
                                           int part) {
  // one chunk ci = part (dev.h p2v_coset_parts): its terms, and the gate's first / last terms in
  // the first / last part
  const int64_t npts = (int64_t)1 << bits;
  const int64_t nint = (npts - 2) / (degree - 1);
  const uint64_t gen = c.root_pow2[32 - bits];
  const EE shifted = V.wx(1 + 2 * (npts + 2) + 4 * nint);
  if (part == 0) {
    const E shift = V.w(0);
    const EE eval_loc = V.wx(1 + 2 * npts);
    A.pushx(ee_sub(eval_loc, ee_scale(shift, shifted)));
  }
  // chunk xs = take degree xs : partition (degree-1) (drop degree xs)
  const int64_t first = degree < npts ? degree : npts;
  const int64_t nst = p2v_coset_parts(bits, degree, nweights);   // zipWith worker initials chunks
  const int64_t ci = part;
  EE ev, pr;
  if (ci == 0) { ev = EE{gl::e0(), gl::e0()}; pr = EE{gl::eb(1), gl::e0()}; }
  else { ev = V.wx(1 + 2 * (npts + 2) + 2 * (ci - 1)); pr = V.wx(1 + 2 * (npts + 2) + 2 * (nint + ci - 1)); }
  const int64_t cs = ci == 0 ? 0 : first + (ci - 1) * (degree - 1);
  int64_t ce = ci == 0 ? first : cs + (degree - 1);
  if (ce > npts) ce = npts;
  uint64_t x = 1;   // gen^cs: the domain position of the chunk's first point
  for (uint64_t b = gen, e = (uint64_t)cs; e; e >>= 1) { if (e & 1) x = gl::mul(x, b); b = gl::mul(b, b); }
  for (int64_t k = cs; k < ce; k++) {
    if (k >= nweights) break;
    // one product at a time (the fences keep the five F^2-over-F^2 products from being
    // interleaved into registers): ev' = term ev + val pr, pr' = term pr
    const EE term = ee_sub(shifted, ee_base(gl::eb(x)));
    EE t1 = ee_mul(term, ev);
    pin(t1.re); pin(t1.im);
    EE val = ee_scale(gl::eb(weights[k]), V.wx(1 + 2 * k));
    pinm2(val.re, val.im);
    EE t2 = ee_mul(val, pr);
    pin(t2.re); pin(t2.im);
    pr = ee_mul(term, pr); ev = ee_add(t1, t2);
    x = gl::mul(x, gen);
    pinm2(pr.re, pr.im); pin(ev.re); pin(ev.im);
  }
  if (ci + 1 < nst) {
    A.pushx(ee_sub(V.wx(1 + 2 * (npts + 2) + 2 * ci), ev));
    A.pushx(ee_sub(V.wx(1 + 2 * (npts + 2) + 2 * (nint + ci)), pr));
  } else {
    const EE eval_result = V.wx(1 + 2 * npts + 2);
    A.pushx(ee_sub(eval_result, ev));
  }
}

// the level-L node of lookup_eq's pairwise reduction over inputs [k 2^L, (k+1) 2^L): level j
// combines a[2t], a[2t+1] with bit b_j as a[2t] + b_j (a[2t+1] - a[2t]).  Evaluated depth-first
// (the same node values as the level-by-level form, a stack of NB values instead of 2^NB)
template <int L>
__device__ __forceinline__ E leq_node(const Vars& V, int64_t in0, int64_t b0, int64_t k) {
  if constexpr (L == 0) return V.w(in0 + k);
  else {
    E lo = leq_node<L - 1>(V, in0, b0, 2 * k);
    pinm(lo);
    const E hi = leq_node<L - 1>(V, in0, b0, 2 * k + 1);
    const E b = V.w(b0 + L - 1);
    return gl::eadd(lo, gl::emul(b, gl::esub(hi, lo)));
  }
}
template <int NB>
__device__ __forceinline__ E lookup_eq_fixed(const Vars& V, int64_t in0, int64_t b0) { return leq_node<NB>(V, in0, b0, 0); }

// RandomAccessGate, Gate/Custom/RandomAccess.hs:47-88.  lookup_eq is the multilinear
// interpolation sum_i v_i prod_j (bit_j(i) ? b_j : 1 - b_j); it is evaluated by the same
// pairwise reduction as the reference (exactly the same field element).
template <class A_>
__device__ __forceinline__ void gate_random_access(const Vars& V, A_& A, int nbits, int64_t copies, int64_t extra) {
  const int64_t veclen = (int64_t)1 << nbits, width = 2 + veclen;
  const int64_t bstart = width * copies + extra;
  const E one = gl::eb(1);
  for (int64_t k = 0; k < copies; k++) {
    for (int j = 0; j < nbits; j++) { E b = V.w(bstart + k * nbits + j); A.push(gl::emul(b, gl::esub(b, one))); }
    E rec = gl::e0();
    for (int j = nbits - 1; j >= 0; j--) rec = gl::eadd(gl::eadd(rec, rec), V.w(bstart + k * nbits + j));
    A.push(gl::esub(rec, V.w(k * width)));
    // lookup_eq: level-by-level pairwise reduction (registers for up to 2^4 inputs)
    E val;
    switch (nbits) {
      case 0: val = V.w(k * width + 2); break;
      case 1: val = lookup_eq_fixed<1>(V, k * width + 2, bstart + k * nbits); break;
      case 2: val = lookup_eq_fixed<2>(V, k * width + 2, bstart + k * nbits); break;
      case 3: val = lookup_eq_fixed<3>(V, k * width + 2, bstart + k * nbits); break;
      case 4: val = lookup_eq_fixed<4>(V, k * width + 2, bstart + k * nbits); break;
      default: {   // same element via the multilinear form sum_i v_i prod_j (b_j or 1-b_j)
        val = gl::e0();
        for (int64_t i = 0; i < veclen; i++) {
          E wgt = gl::eb(1);
          for (int j = 0; j < nbits; j++) { E b = V.w(bstart + k * nbits + j); wgt = gl::emul(wgt, ((i >> j) & 1) ? b : gl::esub(one, b)); }
          val = gl::eadd(val, gl::emul(wgt, V.w(k * width + 2 + i)));
        }
      }
    }
    A.push(gl::esub(val, V.w(k * width + 1)));
  }
  for (int64_t j = 0; j < extra; j++) A.push(gl::esub(V.k(j), V.w(copies * width + j)));
}

// Gate items are split by kernel class so that each kernel is register-allocated for its
// own programs (one kernel holding all of them needed 256 VGPRs and still spilled):
// VK_POSEIDON: PoseidonGate parts; VK_COSET: CosetInterpolationGate; VK_MISC: everything else.
// VK_LOOKUP: the lookup-argument items (Plonk/Lookups.hs:45-132), a class of their own so that
// their register demand does not set the misc kernel's.
enum { VK_POSEIDON = 0, VK_COSET = 1, VK_MISC = 2, VK_LOOKUP = 3 };

template <int CLS, class A_>
__device__ __forceinline__ void eval_gate(const DevCircuit& c, const Vars& V, A_& A, int g, int part) {
  const int64_t p0 = c.gate_par[3 * g], p1 = c.gate_par[3 * g + 1], p2 = c.gate_par[3 * g + 2];
  if constexpr (CLS == VK_POSEIDON) { (void)p0; (void)p1; (void)p2; gate_poseidon(V, A, part); return; }
  if constexpr (CLS == VK_COSET) { gate_coset(c, V, A, (int)p0, p1, c.weights + c.gate_woff[g], c.gate_woff[g + 1] - c.gate_woff[g], part); return; }
  const int kind = c.gate_kind[g];
  const E one = gl::eb(1);
  switch (kind) {
    case 0:   // ArithmeticGate, Constraints.hs:45-46
      for (int64_t i = 0; i < p0; i++) {
        const int64_t j = 4 * i;
        A.push(gl::esub(gl::esub(V.w(j + 3), gl::emul(gl::emul(V.k(0), V.w(j)), V.w(j + 1))), gl::emul(V.k(1), V.w(j + 2))));
      }
      break;
    case 1:   // ArithmeticExtensionGate, :49-54
      for (int64_t i = 0; i < p0; i++) {
        const int64_t j = 8 * i;
        const EE c0 = ee_base(V.k(0)), c1 = ee_base(V.k(1));
        A.pushx(ee_sub(ee_sub(V.wx(j + 6), ee_mul(ee_mul(c0, V.wx(j)), V.wx(j + 2))), ee_mul(c1, V.wx(j + 4))));
      }
      break;
    case 2: {  // BaseSumGate, :57-62
      const E base = gl::eb((uint64_t)p1 % gl::P);
      E h;
      if (0 < p0 - 1) { h = V.w(p0); for (int64_t t = p0 - 2; t >= 0; t--) h = gl::eadd(V.w(t + 1), gl::emul(base, h)); }
      else h = V.w(1);
      A.push(gl::esub(h, V.w(0)));
      for (int64_t i = 0; i < p0; i++) {
        E pr = one; const E l = V.w(i + 1);
        for (int64_t t = 0; t < p1; t++) pr = gl::emul(pr, gl::esub(l, gl::eb((uint64_t)t)));
        A.push(pr);
      }
      break; }
    case 4: for (int64_t i = 0; i < p0; i++) A.push(gl::esub(V.k(i), V.w(i))); break;   // ConstantGate
    case 5: {  // ExponentiationGate, :114-128
      const int64_t n = p0;
      const E base = V.w(0);
      for (int64_t i = 0; i < n; i++) {
        E prev = one;
        if (i != 0) { E tv = V.w(n + 2 + i - 1); prev = gl::emul(tv, tv); }
        const E bit = V.w((n - 1 - i) + 1);
        const E comp = gl::emul(prev, gl::eadd(gl::emul(bit, base), gl::esub(one, bit)));
        A.push(gl::esub(comp, V.w(n + 2 + i)));
      }
      A.push(gl::esub(V.w(n + 1), V.w(n + 2 + n - 1)));
      break; }
    case 8:   // MulExtensionGate, :80-83
      for (int64_t i = 0; i < p0; i++) {
        const int64_t j = 6 * i;
        A.pushx(ee_sub(V.wx(j + 4), ee_mul(ee_mul(ee_base(V.k(0)), V.wx(j)), V.wx(j + 2))));
      }
      break;
    case 10:   // PublicInputGate, :88-89
      for (int i = 0; i < 4; i++) A.push(gl::esub(V.w(i), gl::eb(chal(c, CH_PI(c) + i, V.p))));
      break;
    case 12:   // PoseidonMdsGate, Custom/Poseidon.hs:49-59
#pragma unroll 1
      for (int i = 0; i < 12; i++) {
        asm volatile("" : : : "memory");   // the 12 inputs are re-read per row, not held in 96 VGPRs
        EE acc = EE{gl::e0(), gl::e0()};
        for (int j = 0; j < 12; j++) {
          const uint32_t m = p2::mds_coeff(i, j);
          const EE x = V.wx(2 * j);
          acc = ee_add(acc, EE{E{gl::mul_small(x.re.a, m), gl::mul_small(x.re.b, m)}, E{gl::mul_small(x.im.a, m), gl::mul_small(x.im.b, m)}});
        }
        A.pushx(ee_sub(V.wx(2 * (i + 12)), acc));
      }
      break;
    case 13: gate_random_access(V, A, (int)p0, p1, p2); break;
    case 14:   // ReducingGate, Custom/Reducing.hs:28-41
      for (int64_t i = 0; i < p0; i++) {
        const EE prev = i == 0 ? V.wx(4) : V.wx(6 + p0 + 2 * (i - 1));
        const EE acc = i < p0 - 1 ? V.wx(6 + p0 + 2 * i) : V.wx(0);
        A.pushx(ee_sub(ee_add(ee_mul(prev, V.wx(2)), ee_base(V.w(6 + i))), acc));
      }
      break;
    case 15:   // ReducingExtensionGate, Custom/Reducing.hs:45-60
      for (int64_t i = 0; i < p0; i++) {
        const EE prev = i == 0 ? V.wx(4) : V.wx(6 + 2 * p0 + 2 * (i - 1));
        const EE acc = i < p0 - 1 ? V.wx(6 + 2 * p0 + 2 * i) : V.wx(0);
        A.pushx(ee_sub(ee_add(ee_mul(prev, V.wx(2)), V.wx(6 + 2 * i)), acc));
      }
      break;
    default: break;   // Lookup / LookupTable / Noop: no constraints
  }
}

__device__ __forceinline__ uint64_t pow_u(uint64_t x, uint32_t e) {   // uniform exponent
  uint64_t acc = 1;
  for (; e; e >>= 1) { if (e & 1) acc = gl::mul(acc, x); x = gl::mul(x, x); }
  return acc;
}

// Z(1) boundary terms: L0(zeta)(Z_i(zeta) - 1), Vanishing.hs:86-95, Algebra/Poly.hs:14-16
template <class A_>
__device__ __forceinline__ void item_zs1(const DevCircuit& c, A_& T, int p) {
  const E zeta = chal_e(c, CH_ZETA(c), p), one = gl::eb(1);
  const E zeta_n = epow2n(zeta, c.degree_bits);
  E L0;
  if (gl::eeq(zeta, one)) L0 = one;
  else L0 = gl::emul(gl::esub(zeta_n, one), einv(gl::escale((1ULL << c.degree_bits) % gl::P, gl::esub(zeta, one))));
  for (int i = 0; i < c.r; i++) T.push(gl::emul(L0, gl::esub(lde(c, c.o_zs + 2 * i, p), one)));
}

// partial-product transitions of challenge round j, Vanishing.hs:97-111
template <class A_>
__device__ __forceinline__ void item_pp(const DevCircuit& c, A_& T, int j, int p) {
  const E zeta = chal_e(c, CH_ZETA(c), p), one = gl::eb(1);
  const uint64_t beta = chal(c, CH_BETA(c) + j, p), gamma = chal(c, CH_GAMMA(c) + j, p);
  const int nnum = c.num_routed < c.num_wires ? c.num_routed : c.num_wires;
  for (int ch = 0; ch < c.n_pp_terms; ch++) {
    const E prev = ch == 0 ? lde(c, c.o_zs + 2 * j, p) : lde(c, c.o_pp + 2 * ((int64_t)j * c.npp + ch - 1), p);
    const E next = ch == c.npp ? lde(c, c.o_zs_next + 2 * j, p) : lde(c, c.o_pp + 2 * ((int64_t)j * c.npp + ch), p);
    E pn = one, pd = one;
    for (int t = ch * c.qdf; t < nnum && t < (ch + 1) * c.qdf; t++) {
      const E w = lde(c, c.o_wires + 2 * t, p);
      pn = gl::emul(pn, gl::eadd(gl::eadd(w, gl::escale(gl::mul(beta, c.k_is[t]), zeta)), gl::eb(gamma)));
      pd = gl::emul(pd, gl::eadd(gl::eadd(w, gl::escale(beta, lde(c, c.o_sig + 2 * t, p))), gl::eb(gamma)));
      pinm2(pn, pd);
    }
    T.push(gl::esub(gl::emul(prev, pn), gl::emul(next, pd)));
  }
}

// lookup terms of challenge round j, Plonk/Lookups.hs:45-132
// evalFinalRE (Lookups.hs:103-109) as Ain(delta) + B Aout(delta), where Ain / Aout have the
// table's (padded, reversed) inputs / outputs as coefficients (exactly the reference's Horner
// sum, reassociated).  Baby steps: delta^0..15 per lane; each 16-entry chunk is a dot product
// of u24 wave-uniform coefficients (scalar loads) with the powers' 32-bit halves, accumulated
// exactly in 64 bits (< 16 2^24 2^32 = 2^60) and reduced once; giant steps: Horner in
// delta^16 over the chunks.  ~8 VALU per table entry instead of ~50.  k_lut evaluates pieces
// of P2V_LUT_PIECE chunks, P_s = sum_{c in piece s} delta^(16 (c - c0_s)) (Cin_c + B Cout_c),
// on many waves; item_lookup combines them by Horner in delta^(16 P2V_LUT_PIECE).
__device__ __forceinline__ uint64_t lut_piece(const DevCircuit& c, int k, int c0, int c1, uint64_t dde, uint64_t dB) {
  constexpr int M = P2V_LUT_CHUNK;
  uint64_t pw[M];
  pw[0] = 1;
#pragma unroll
  for (int j = 1; j < M; j++) pw[j] = gl::mul(pw[j - 1], dde);
  const uint64_t dM = gl::mul(pw[M - 1], dde);
  const uint32_t* ri = c.lut_rin + c.lut_roff[k];
  const uint32_t* ro = c.lut_rout + c.lut_roff[k];
  uint64_t ai = 0, ao = 0;
  for (int ch = c1 - 1; ch >= c0; ch--) {
    uint64_t il = 0, ih = 0, ol = 0, oh = 0;
#pragma unroll
    for (int j = 0; j < M; j++) {
      const uint64_t ci = ri[M * ch + j], co = ro[M * ch + j];
      il += ci * (uint32_t)pw[j]; ih += ci * (uint32_t)(pw[j] >> 32);
      ol += co * (uint32_t)pw[j]; oh += co * (uint32_t)(pw[j] >> 32);
    }
    ai = gl::add(gl::mul(ai, dM), gl::canon(p2::mds_reduce(il, ih)));
    ao = gl::add(gl::mul(ao, dM), gl::canon(p2::mds_reduce(ol, oh)));
  }
  return gl::add(ai, gl::mul(dB, ao));
}

template <class A_>
__device__ __forceinline__ void item_lookup(const DevCircuit& c, A_& T, int j, int p) {
  const E one = gl::eb(1);
  const int nlp = c.nlp, nsldc = nlp - 1;
  const int nlu = c.num_routed / 2 < c.num_wires / 2 ? c.num_routed / 2 : c.num_wires / 2;
  const int slots3 = c.num_routed / 3;
  const int nlut = slots3 < c.num_wires / 3 ? slots3 : c.num_wires / 3;
  const int lu_degree = c.qdf - 1, lut_degree = (slots3 + nsldc - 1) / nsldc;
  const int nclu = (nlu + lu_degree - 1) / lu_degree, nclut = (nlut + lut_degree - 1) / lut_degree, ncm = (slots3 + lut_degree - 1) / lut_degree;
  int nz = nclu < nclut ? nclu : nclut; nz = nz < ncm ? nz : ncm; nz = nz < nsldc ? nz : nsldc;
  const int64_t ls = c.o_const + 2 * (int64_t)c.ngroups;   // lookup selectors
  auto sel = [&](int k) { return c.unit_filters ? gl::eb(1) : lde(c, ls + 2 * k, p); };
  auto wv = [&](int t) { return lde(c, c.o_wires + 2 * (int64_t)t, p); };
  const uint64_t dA = chal(c, CH_DELTA(c) + 4 * j, p), dB = chal(c, CH_DELTA(c) + 4 * j + 1, p);
  const uint64_t dal = chal(c, CH_DELTA(c) + 4 * j + 2, p), dde = chal(c, CH_DELTA(c) + 4 * j + 3, p);
  const int64_t zoff = c.o_lzs + 2 * (int64_t)j * nlp, znoff = c.o_lzs_next + 2 * (int64_t)j * nlp;
  const E re = lde(c, zoff, p), re_next = lde(c, znoff, p);
  auto sldc = [&](int k) { return lde(c, zoff + 2 * (1 + k), p); };
  auto sldc_next = [&](int k) { return lde(c, znoff + 2 * (1 + k), p); };
  T.push(gl::emul(sel(3), sldc(nsldc - 1)));
  T.push(gl::emul(sel(2), sldc(0)));
  T.push(gl::emul(sel(2), re));
  for (int k = 0; k < c.nluts; k++) {   // evalFinalRE, :103-109
    uint64_t cur;
    if (c.lut_rchunks[k] > 0) {   // combine the k_lut pieces
      const int pb = c.lut_pbase[k], np = c.lut_pbase[k + 1] - pb;
      uint64_t dL = dde;
      for (int e = 1; e < P2V_LUT_CHUNK * P2V_LUT_PIECE; e <<= 1) dL = gl::mul(dL, dL);   // delta^(16 * 256)
      const uint64_t* part = c.lutpart + ((int64_t)j * c.n_lut_pieces + pb) * c.B + p;
      cur = part[(int64_t)(np - 1) * c.B];
      for (int s2 = np - 2; s2 >= 0; s2--) { cur = gl::add(gl::mul(cur, dL), part[(int64_t)s2 * c.B]); pinm64(cur); }
    } else {
      const int64_t len = c.lut_len[k], off = c.lut_off[k];
      const int64_t padded = ((len + slots3 - 1) / slots3) * slots3;
      cur = 0;
      for (int64_t i = 0; i < padded; i++) {
        const int64_t jj = i < len ? i : 0;
        cur = gl::add(gl::mul(dde, cur), gl::add(c.lut_in[off + jj], gl::mul(dB, c.lut_out[off + jj])));
        pinm64(cur);
      }
    }
    c.lutre[((int64_t)j * c.nluts + k) * c.B + p] = cur;
    T.push(gl::emul(sel(4 + k), gl::esub(re, gl::eb(cur))));
  }
  {
    E cs = re_next;
    for (int t = 0; t < nlut; t++) { cs = gl::eadd(gl::escale(dde, cs), gl::eadd(wv(3 * t), gl::escale(dB, wv(3 * t + 1)))); pinm(cs); }
    T.push(gl::emul(sel(0), gl::esub(re, cs)));
  }
  const E alpha = gl::eb(dal);
  for (int ch = 0; ch < nz; ch++) {
    const E prev = ch == 0 ? sldc_next(nsldc - 1) : sldc(ch - 1);
    const E curv = sldc(ch);
    E Plu = one, Slu = gl::e0(), Plut = one, Slut = gl::e0();
    const int lus = ch * lu_degree, lue = (lus + lu_degree < nlu) ? lus + lu_degree : nlu;
    for (int t = lus; t < lue; t++) {
      const E x = gl::esub(alpha, gl::eadd(wv(2 * t), gl::escale(dA, wv(2 * t + 1))));
      Slu = gl::eadd(gl::emul(Slu, x), Plu); Plu = gl::emul(Plu, x);
      pinm2(Slu, Plu);
    }
    const int tts = ch * lut_degree, tte = (tts + lut_degree < nlut) ? tts + lut_degree : nlut;
    const int mte = (tts + lut_degree < slots3) ? tts + lut_degree : slots3;
    const int nmz = (tte - tts) < (mte - tts) ? (tte - tts) : (mte - tts);
    for (int t = tts; t < tte; t++) {
      const E y = gl::esub(alpha, gl::eadd(wv(3 * t), gl::escale(dA, wv(3 * t + 1))));
      const E m = (t - tts) < nmz ? wv(3 * t + 2) : gl::e0();
      Slut = gl::eadd(gl::emul(Slut, y), gl::emul(m, Plut)); Plut = gl::emul(Plut, y);
      pinm2(Slut, Plut);
    }
    const E diff = gl::esub(curv, prev);
    T.push(gl::emul(sel(0), gl::esub(gl::emul(Plut, diff), Slut)));   // eq_sum_trans
    T.push(gl::emul(sel(1), gl::eadd(gl::emul(Plu, diff), Slu)));     // eq_ldc_trans
  }
}

// One vanishing work item for proof p: a contiguous run of terms of the combined sequence
// sum_k alpha_i^k t_k (Vanishing.hs:48-137).  Item `it` = {type, a, b, first_term}; its
// partial sums (one F^2 per challenge round) go to vparts[it][2r][B].  R: see Acc.
template <int CLS, int R>
__device__ __forceinline__ void vanish_item(const DevCircuit& c, int it, int p) {
  const int type = c.vitems[4 * it], a = c.vitems[4 * it + 1], b = c.vitems[4 * it + 2];
  const uint32_t first = (uint32_t)c.vitems[4 * it + 3];
  const int r = c.r;
  Acc<R> T;
  T.r = r;
#pragma unroll
  for (int i = 0; i < R; i++) {
    T.h[i] = gl::e0();
    T.al[i] = T.on(i) ? chal(c, CH_ALPHA(c) + i, p) : 0;
    T.pw[i] = T.on(i) ? pow_u(T.al[i], first) : 0;
  }
  if constexpr (CLS == VK_LOOKUP) { (void)b; item_lookup(c, T, a, p); }
  else if (CLS == VK_MISC && type == VI_ZS1) item_zs1(c, T, p);
  else if (CLS == VK_MISC && type == VI_PP) item_pp(c, T, a, p);
  else {   // gate a (part b): alpha^G0 * S_g(zeta) * sum_k alpha^k c_gk, Vanishing.hs:113-125
    Vars V{&c, p};
    eval_gate<CLS>(c, V, T, a, b);
    // the filter after the program (same element; nothing of it is live during the gate's terms)
    const int grp = c.gate_grp[a];
    const E x = lde(c, c.o_const + 2 * grp, p);   // S_grp(zeta)
    const E one = gl::eb(1);
    const E unused = gl::eb(0xFFFFFFFFULL);
    E s = c.ngroups > 1 ? gl::esub(unused, x) : one;   // Gate/Selector.hs:83-89
    for (int j = c.grp_start[grp]; j < c.grp_end[grp]; j++) if (j != a) s = gl::emul(s, gl::esub(gl::eb((uint64_t)j), x));
    if (c.unit_filters) s = one;
#pragma unroll
    for (int i = 0; i < R; i++)
      if (T.on(i)) T.h[i] = gl::escale(pow_u(T.al[i], (uint32_t)c.alpha_base_gates), gl::emul(s, T.h[i]));
  }
  uint64_t* dst = c.vparts + (int64_t)it * 2 * r * c.B + p;
#pragma unroll
  for (int i = 0; i < R; i++)   // constant indices: T stays in registers
    if (T.on(i)) { dst[(int64_t)(2 * i) * c.B] = T.h[i].a; dst[(int64_t)(2 * i + 1) * c.B] = T.h[i].b; }
}

// one wave = (item, 64 proofs); items are wave-uniform, heaviest first (host order); the
// items of kernel class CLS are c.vcls[CLS] .. c.vcls[CLS + 1].  Work-groups of one wave, so a
// wave can be dispatched wherever one k_merkle wave has retired.
template <int CLS, int R>
__device__ __forceinline__ void vanish_body(const DevCircuit& c) {
  const int lane = threadIdx.x & 63;
  const int unit = blockIdx.x;
  const int NPB = c.B >> 6;
  const int i0 = c.vcls[CLS], ni = c.vcls[CLS + 1] - i0;
  if (unit >= ni * NPB) return;
  const int it = i0 + unit / NPB, p = (unit % NPB) * 64 + lane;
  // runs concurrently with k_merkle (VALU-bound, many waves): raise the priority of these
  // few latency-bound waves so they do not end up on the critical path
  __builtin_amdgcn_s_setprio(2);
  vanish_item<CLS, R>(c, it, p);
}

// the standard number of challenge rounds (plonky2's default num_challenges)
#define P2V_R_STD 2

}  // namespace
