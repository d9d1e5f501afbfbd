// gen/gates.hpp — the proof generator's own statement of the gate kinds (workload and
// fixture infrastructure, NOT on the verifier path; libp2v never includes it).
//
// Two halves per gate kind:
//   * eval():  the constraint program of Gate/Constraints.hs:40-128 and Gate/Custom/*.hs,
//              in the reference's constraint order and sign, evaluated at one point of the
//              base field (the prover evaluates it on a coset to build the quotient);
//   * fill():  a witness row with plonky2's semantics, derived WITHOUT the constraint
//              program wherever the gate has an independent meaning: the Poseidon output and
//              every S-box input come from the naive permutation (Hash/Poseidon.hs:42-101,
//              KAT-pinned), the CosetInterpolation result from Lagrange interpolation, the
//              Exponentiation output from base^e, the Reducing outputs from Horner sums, the
//              RandomAccess output from list[index].
// A row from fill() must make every eval() term zero; the prover asserts it (its quotient is
// low-degree only if it does), so a misreading of a gate's wire layout or formula in either
// half shows up as a generator error, and the verifier must then agree with eval() at zeta.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>
#include "../gl.h"
#include "../poseidon.h"

namespace gg {

using u64 = uint64_t;
using gl::E;

enum Kind { ARITH, ARITH_EXT, BASESUM, COSET, CONST, EXP, LOOKUP, LOOKUPTABLE, MULEXT, NOOP, PI,
            POSEIDON, POSEIDON_MDS, RANDACC, REDUCING, REDUCING_EXT };

struct Gate {
  Kind kind = NOOP;
  int64_t p0 = 0, p1 = 0, p2 = 0;
  std::vector<u64> weights;   // CosetInterpolationGate barycentric weights
  std::string str;            // the Rust Debug string (Gate/Parser.hs grammar)
  int degree = 0;             // measured total degree of the constraints (prover)
};

static const u64 FAST_FIRST_RC[12] = P2V_FAST_PARTIAL_FIRST_ROUND_CONSTANT_INIT;
static const u64 FAST_RC[22] = P2V_FAST_PARTIAL_ROUND_CONSTANTS_INIT;
static const u64 FAST_VS[22 * 11] = P2V_FAST_PARTIAL_ROUND_VS_INIT;
static const u64 FAST_W_HATS[22 * 11] = P2V_FAST_PARTIAL_ROUND_W_HATS_INIT;
static const u64 FAST_INIT_MATRIX[11 * 11] = P2V_FAST_PARTIAL_ROUND_INITIAL_MATRIX_INIT;
static const u64 ROUND_CONSTANTS[360] = P2V_ALL_ROUND_CONSTANTS_INIT;

inline u64 f(u64 x) { return x % gl::P; }
inline u64 add(u64 a, u64 b) { return gl::add(a, b); }
inline u64 sub(u64 a, u64 b) { return gl::sub(a, b); }
inline u64 mul(u64 a, u64 b) { return gl::mul(a, b); }
inline u64 sbox(u64 x) { u64 x2 = mul(x, x), x3 = mul(x, x2), x4 = mul(x2, x2); return mul(x3, x4); }

// ---------------------------------------------------------------- layouts
struct CosetLayout {   // Gate/Custom/CosetInterp.hs:91-98
  int64_t npts, nint, degree;
  int64_t val(int64_t k) const { return 1 + 2 * k; }
  int64_t eval_loc() const { return 1 + 2 * npts; }
  int64_t eval_result() const { return 1 + 2 * npts + 2; }
  int64_t tmp_eval(int64_t i) const { return 1 + 2 * (npts + 2) + 2 * i; }
  int64_t tmp_prod(int64_t i) const { return 1 + 2 * (npts + 2) + 2 * (nint + i); }
  int64_t shifted() const { return 1 + 2 * (npts + 2) + 4 * nint; }
  // chunk xs = take degree xs : partition (degree-1) (drop degree xs)
  std::vector<std::pair<int64_t, int64_t>> chunks() const {
    std::vector<std::pair<int64_t, int64_t>> c;
    int64_t first = degree < npts ? degree : npts;
    c.push_back({0, first});
    for (int64_t s = first; s < npts; s += degree - 1) c.push_back({s, std::min(npts, s + degree - 1)});
    return c;
  }
};
inline CosetLayout coset_layout(const Gate& g) {
  CosetLayout L;
  L.npts = (int64_t)1 << g.p0; L.degree = g.p1;
  if (L.degree < 2) throw std::runtime_error("gen: coset gate degree < 2");
  L.nint = (L.npts - 2) / (L.degree - 1);
  return L;
}

// Poseidon gate wires, Gate/Custom/Poseidon.hs:143-150
constexpr int PW_SWAP = 24, PW_DELTA = 25, PW_ISB = 29, PW_PSB = 29 + 36, PW_FSB = 29 + 36 + 22;

// ---------------------------------------------------------------- constraint programs
// The evaluation point's wire / constant values are base-field elements; `wireExt i` is the
// F^2 element (w_i, w_{i+1}) and commitExt pushes its two coordinates (Gate/Computation.hs:75-76).
struct Ctx {
  const u64* w; int nw; const u64* k; int nk; const u64* pih;
  std::vector<u64>* out;
  u64 W(int64_t i) const { if (i < 0 || i >= nw) throw std::runtime_error("gen: wire index out of range"); return w[i]; }
  u64 K(int64_t i) const { if (i < 0 || i >= nk) throw std::runtime_error("gen: constant index out of range"); return k[i]; }
  E WX(int64_t i) const { return E{W(i), W(i + 1)}; }
  void push(u64 x) const { out->push_back(x); }
  void pushx(E x) const { out->push_back(x.a); out->push_back(x.b); }
};

inline void eval_poseidon(const Ctx& c) {   // Custom/Poseidon.hs:63-150
  const u64 swap = c.W(PW_SWAP);
  c.push(mul(swap, sub(swap, 1)));
  for (int i = 0; i < 4; i++) c.push(sub(mul(swap, sub(c.W(i + 4), c.W(i))), c.W(PW_DELTA + i)));
  u64 st[12], t[12];
  for (int i = 0; i < 4; i++) st[i] = add(c.W(i), c.W(PW_DELTA + i));
  for (int i = 4; i < 8; i++) st[i] = sub(c.W(i), c.W(PW_DELTA + i - 4));
  for (int i = 8; i < 12; i++) st[i] = c.W(i);
  auto mds = [&](u64* s) {
    for (int i = 0; i < 12; i++) { u64 a = 0; for (int j = 0; j < 12; j++) a = add(a, mul(p2::mds_coeff(i, j), s[j])); t[i] = a; }
    memcpy(s, t, sizeof t);
  };
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 12; i++) st[i] = add(st[i], ROUND_CONSTANTS[12 * r + i]);
    if (r != 0) {
      for (int i = 0; i < 12; i++) c.push(sub(st[i], c.W(PW_ISB + 12 * (r - 1) + i)));
      for (int i = 0; i < 12; i++) st[i] = c.W(PW_ISB + 12 * (r - 1) + i);
    }
    for (int i = 0; i < 12; i++) st[i] = sbox(st[i]);
    mds(st);
  }
  for (int i = 0; i < 12; i++) st[i] = add(st[i], FAST_FIRST_RC[i]);
  // mdsInitPartial: row i of the 11x11 block is sum_j partialMdsMatrixCoeff i j * rest_j,
  // partialMdsMatrixCoeff i j = FAST_PARTIAL_ROUND_INITIAL_MATRIX ! (j, i)
  t[0] = st[0];
  for (int i = 0; i < 11; i++) { u64 a = 0; for (int j = 0; j < 11; j++) a = add(a, mul(FAST_INIT_MATRIX[11 * j + i], st[1 + j])); t[1 + i] = a; }
  memcpy(st, t, sizeof t);
  for (int r = 0; r < 22; r++) {
    const u64 sb = c.W(PW_PSB + r);
    c.push(sub(st[0], sb));
    u64 z = sbox(sb);
    if (r < 21) z = add(z, FAST_RC[r]);
    st[0] = z;
    u64 d = mul(st[0], p2::mds_coeff(0, 0));   // cs = m00 : w_hats r
    for (int j = 0; j < 11; j++) d = add(d, mul(st[1 + j], FAST_W_HATS[11 * r + j]));
    for (int j = 0; j < 11; j++) st[1 + j] = add(st[1 + j], mul(z, FAST_VS[11 * r + j]));
    st[0] = d;
  }
  for (int r = 0; r < 4; r++) {
    for (int i = 0; i < 12; i++) st[i] = add(st[i], ROUND_CONSTANTS[12 * (r + 26) + i]);
    for (int i = 0; i < 12; i++) c.push(sub(st[i], c.W(PW_FSB + 12 * r + i)));
    for (int i = 0; i < 12; i++) st[i] = sbox(c.W(PW_FSB + 12 * r + i));
    mds(st);
  }
  for (int i = 0; i < 12; i++) c.push(sub(st[i], c.W(12 + i)));
}

inline void eval_coset(const Gate& g, const Ctx& c) {   // Custom/CosetInterp.hs:51-121
  const CosetLayout L = coset_layout(g);
  const u64 gen = gl::subgroup_gen((int)g.p0);
  const E shifted = c.WX(L.shifted());
  c.pushx(gl::esub(c.WX(L.eval_loc()), gl::escale(c.W(0), shifted)));
  auto ch = L.chunks();
  size_t nst = std::min((size_t)L.nint + 1, ch.size());
  E ev = gl::e0(), pr = gl::eb(1);
  u64 xk = 1;   // domain point g^k; the chunks cover k = 0, 1, ... in order
  for (size_t ci = 0; ci < nst; ci++) {
    if (ci > 0) { ev = c.WX(L.tmp_eval(ci - 1)); pr = c.WX(L.tmp_prod(ci - 1)); }
    for (int64_t k = ch[ci].first; k < ch[ci].second && k < (int64_t)g.weights.size(); k++, xk = mul(xk, gen)) {
      const E val = gl::escale(g.weights[k], c.WX(L.val(k)));
      const E term = gl::esub(shifted, gl::eb(xk));
      const E ne = gl::eadd(gl::emul(term, ev), gl::emul(val, pr));
      pr = gl::emul(term, pr); ev = ne;
    }
    if (ci + 1 < nst) { c.pushx(gl::esub(c.WX(L.tmp_eval(ci)), ev)); c.pushx(gl::esub(c.WX(L.tmp_prod(ci)), pr)); }
  }
  c.pushx(gl::esub(c.WX(L.eval_result()), ev));
}

inline void eval_random_access(const Gate& g, const Ctx& c) {   // Custom/RandomAccess.hs:47-88
  const int nb = (int)g.p0; const int64_t copies = g.p1, extra = g.p2;
  const int64_t veclen = (int64_t)1 << nb, width = 2 + veclen, bstart = width * copies + extra;
  for (int64_t k = 0; k < copies; k++) {
    for (int j = 0; j < nb; j++) { u64 b = c.W(bstart + k * nb + j); c.push(mul(b, sub(b, 1))); }
    u64 rec = 0;
    for (int j = nb - 1; j >= 0; j--) rec = add(add(rec, rec), c.W(bstart + k * nb + j));   // foldr (\b acc -> 2acc+b) 0
    c.push(sub(rec, c.W(k * width)));
    std::vector<u64> v(veclen);
    for (int64_t i = 0; i < veclen; i++) v[i] = c.W(k * width + 2 + i);
    for (int j = 0; j < nb; j++) {   // lookup_eq: pairs (x, y) -> x + b (y - x)
      const u64 b = c.W(bstart + k * nb + j);
      for (size_t t = 0; t < v.size() / 2; t++) v[t] = add(v[2 * t], mul(b, sub(v[2 * t + 1], v[2 * t])));
      v.resize(v.size() / 2);
    }
    c.push(sub(v[0], c.W(k * width + 1)));
  }
  for (int64_t j = 0; j < extra; j++) c.push(sub(c.K(j), c.W(copies * width + j)));
}

inline void eval(const Gate& g, const u64* w, int nw, const u64* k, int nk, const u64* pih, std::vector<u64>& out) {
  Ctx c{w, nw, k, nk, pih, &out};
  switch (g.kind) {
    case ARITH:   // Constraints.hs:45-46
      for (int64_t i = 0; i < g.p0; i++) { int64_t j = 4 * i;
        c.push(sub(sub(c.W(j + 3), mul(mul(c.K(0), c.W(j)), c.W(j + 1))), mul(c.K(1), c.W(j + 2)))); }
      break;
    case ARITH_EXT:   // :49-54
      for (int64_t i = 0; i < g.p0; i++) { int64_t j = 8 * i;
        c.pushx(gl::esub(gl::esub(c.WX(j + 6), gl::emul(gl::escale(c.K(0), c.WX(j)), c.WX(j + 2))), gl::escale(c.K(1), c.WX(j + 4)))); }
      break;
    case BASESUM: {   // :57-62
      const int64_t nl = g.p0; const u64 base = f((u64)g.p1);
      u64 h = c.W(nl);
      for (int64_t t = nl - 2; t >= 0; t--) h = add(c.W(t + 1), mul(base, h));
      c.push(sub(h, c.W(0)));
      for (int64_t i = 0; i < nl; i++) { u64 pr = 1; for (int64_t t = 0; t < g.p1; t++) pr = mul(pr, sub(c.W(i + 1), f((u64)t))); c.push(pr); }
      break; }
    case COSET: eval_coset(g, c); break;
    case CONST: for (int64_t i = 0; i < g.p0; i++) c.push(sub(c.K(i), c.W(i))); break;   // :68-69
    case EXP: {   // :114-128
      const int64_t n = g.p0;
      for (int64_t i = 0; i < n; i++) {
        const u64 prev = i == 0 ? 1 : mul(c.W(n + 2 + i - 1), c.W(n + 2 + i - 1));
        const u64 bit = c.W((n - 1 - i) + 1);
        c.push(sub(mul(prev, add(mul(bit, c.W(0)), sub(1, bit))), c.W(n + 2 + i)));
      }
      c.push(sub(c.W(n + 1), c.W(n + 2 + n - 1)));
      break; }
    case MULEXT:   // :80-83
      for (int64_t i = 0; i < g.p0; i++) { int64_t j = 6 * i;
        c.pushx(gl::esub(c.WX(j + 4), gl::emul(gl::escale(c.K(0), c.WX(j)), c.WX(j + 2)))); }
      break;
    case PI: for (int i = 0; i < 4; i++) c.push(sub(c.W(i), pih[i])); break;   // :88-89
    case POSEIDON: eval_poseidon(c); break;
    case POSEIDON_MDS:   // Custom/Poseidon.hs:49-59
      for (int i = 0; i < 12; i++) {
        E a = gl::e0();
        for (int j = 0; j < 12; j++) a = gl::eadd(a, gl::escale(p2::mds_coeff(i, j), c.WX(2 * j)));
        c.pushx(gl::esub(c.WX(2 * (i + 12)), a));
      }
      break;
    case RANDACC: eval_random_access(g, c); break;
    case REDUCING: case REDUCING_EXT: {   // Custom/Reducing.hs:28-60
      const int64_t n = g.p0; const bool ext = g.kind == REDUCING_EXT;
      const int64_t acc0 = ext ? 6 + 2 * n : 6 + n;
      auto accum = [&](int64_t i) { return i < n - 1 ? c.WX(acc0 + 2 * i) : c.WX(0); };
      for (int64_t i = 0; i < n; i++) {
        const E prev = i == 0 ? c.WX(4) : accum(i - 1);
        const E co = ext ? c.WX(6 + 2 * i) : gl::eb(c.W(6 + i));
        c.pushx(gl::esub(gl::eadd(gl::emul(prev, c.WX(2)), co), accum(i)));
      }
      break; }
    case LOOKUP: case LOOKUPTABLE: case NOOP: break;
  }
}

// ---------------------------------------------------------------- witness semantics
struct Rng {
  u64 s;
  explicit Rng(u64 seed) : s(seed ^ 0x9E3779B97F4A7C15ULL) {}
  u64 next() { u64 z = (s += 0x9E3779B97F4A7C15ULL); z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL; z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL; return z ^ (z >> 31); }
  u64 field() { for (;;) { u64 x = next(); if (x < gl::P) return x; } }
};

// wires a copy constraint may feed: inputs whose every value satisfies the gate
inline std::vector<int> free_inputs(const Gate& g, int nw) {
  std::vector<int> v;
  auto rng = [&](int a, int b) { for (int i = a; i < b; i++) v.push_back(i); };
  switch (g.kind) {
    case ARITH: for (int i = 0; i < g.p0; i++) rng(4 * i, 4 * i + 3); break;
    case ARITH_EXT: for (int i = 0; i < g.p0; i++) rng(8 * i, 8 * i + 6); break;
    case MULEXT: for (int i = 0; i < g.p0; i++) rng(6 * i, 6 * i + 4); break;
    case EXP: v.push_back(0); break;
    case POSEIDON: rng(0, 12); break;
    case POSEIDON_MDS: rng(0, 24); break;
    case RANDACC: { int64_t width = 2 + ((int64_t)1 << g.p0); for (int k = 0; k < g.p1; k++) rng((int)(k * width + 2), (int)(k * width + width)); break; }
    case REDUCING: rng(2, 6 + (int)g.p0); break;
    case REDUCING_EXT: rng(2, 6 + 2 * (int)g.p0); break;
    case COSET: rng(1, (int)(1 + 2 * ((int64_t)1 << g.p0) + 2)); break;   // values and eval_loc (not the shift: nonzero)
    case NOOP: rng(0, nw); break;   // every wire
    default: break;
  }
  return v;
}

// constants a row of this gate reads (the rest of the row's constant columns are 0)
inline int num_row_constants(const Gate& g) {
  switch (g.kind) {
    case ARITH: case ARITH_EXT: return 2;
    case MULEXT: return 1;
    case CONST: return (int)g.p0;
    case RANDACC: return (int)g.p2;
    default: return 0;
  }
}

// Lagrange interpolation through (shift g^k, v_k) evaluated at z (F^2), straight from the
// definition (no barycentric form): the CosetInterpolation result's meaning
inline E lagrange_eval(u64 shift, u64 gen, const std::vector<E>& v, E z) {
  const size_t n = v.size();
  std::vector<u64> xs(n);
  for (size_t k = 0; k < n; k++) xs[k] = mul(shift, gl::pow(gen, k));
  E acc = gl::e0();
  for (size_t k = 0; k < n; k++) {
    E num = gl::eb(1); u64 den = 1;
    for (size_t j = 0; j < n; j++) if (j != k) { num = gl::emul(num, gl::esub(z, gl::eb(xs[j]))); den = mul(den, sub(xs[k], xs[j])); }
    acc = gl::eadd(acc, gl::emul(v[k], gl::escale(gl::inv(den), num)));
  }
  return acc;
}

// Fill the row `w` (nw wires) of a gate instance.  pre[i] != 0: w[i] was fixed by a copy
// constraint (only ever a free input); everything else is written here.  Unused wires get
// random values (randomize_unused_wires).  k: the row's gate constants.
inline void fill(const Gate& g, u64* w, const uint8_t* pre, int nw, const u64* k, const u64* pih, Rng& rg) {
  std::vector<uint8_t> set(nw, 0);
  auto put = [&](int64_t i, u64 x) {
    if (i < 0 || i >= nw) throw std::runtime_error("gen: fill wire out of range");
    if (pre[i]) throw std::runtime_error("gen: a copy constraint feeds a computed wire");
    w[i] = x; set[i] = 1;
  };
  auto in = [&](int64_t i) -> u64 {   // a free input: the copied value or a fresh random one
    if (i < 0 || i >= nw) throw std::runtime_error("gen: fill wire out of range");
    if (!pre[i] && !set[i]) { w[i] = rg.field(); }
    set[i] = 1; return w[i];
  };
  auto inx = [&](int64_t i) { E e; e.a = in(i); e.b = in(i + 1); return e; };
  auto putx = [&](int64_t i, E x) { put(i, x.a); put(i + 1, x.b); };
  switch (g.kind) {
    case ARITH:
      for (int64_t i = 0; i < g.p0; i++) { int64_t j = 4 * i; u64 x = in(j), y = in(j + 1), z = in(j + 2);
        put(j + 3, add(mul(mul(k[0], x), y), mul(k[1], z))); }
      break;
    case ARITH_EXT:
      for (int64_t i = 0; i < g.p0; i++) { int64_t j = 8 * i; E x = inx(j), y = inx(j + 2), z = inx(j + 4);
        putx(j + 6, gl::eadd(gl::escale(k[0], gl::emul(x, y)), gl::escale(k[1], z))); }
      break;
    case MULEXT:
      for (int64_t i = 0; i < g.p0; i++) { int64_t j = 6 * i; E x = inx(j), y = inx(j + 2);
        putx(j + 4, gl::escale(k[0], gl::emul(x, y))); }
      break;
    case BASESUM: {   // limbs in [0, B), sum = sum_i limb_i B^i
      u64 s = 0, bp = 1;
      for (int64_t i = 0; i < g.p0; i++) { u64 l = rg.next() % (u64)g.p1; put(i + 1, l); s = add(s, mul(l, bp)); bp = mul(bp, f((u64)g.p1)); }
      put(0, s);
      break; }
    case CONST: for (int64_t i = 0; i < g.p0; i++) put(i, k[i]); break;
    case PI: for (int i = 0; i < 4; i++) put(i, pih[i]); break;
    case EXP: {   // [base, e_0..e_{n-1}, out, t_0..t_{n-1}], out = base^(sum e_i 2^i)
      const int64_t n = g.p0;
      const u64 base = in(0);
      std::vector<int> bits(n);
      unsigned __int128 e = 0;
      int any = 0;
      for (int64_t i = 0; i < n; i++) { bits[i] = (int)(rg.next() & 1); any |= bits[i]; put(i + 1, (u64)bits[i]); }
      for (int64_t i = n - 1; i >= 0; i--) e = ((e << 1) | (unsigned)bits[i]) % (gl::P - 1);   // Fermat: exponents mod p-1 (base != 0)
      const u64 out = base == 0 ? (any ? 0 : 1) : gl::pow(base, (u64)e);
      put(n + 1, out);
      u64 t = 1;   // the square-and-multiply chain, most significant bit first
      for (int64_t i = 0; i < n; i++) { const int b = bits[n - 1 - i]; t = mul(i == 0 ? 1 : mul(t, t), b ? base : 1); put(n + 2 + i, t); }
      break; }
    case POSEIDON: {
      const u64 swap = rg.next() & 1;
      u64 inp[12];
      for (int i = 0; i < 12; i++) inp[i] = in(i);
      put(PW_SWAP, swap);
      for (int i = 0; i < 4; i++) put(PW_DELTA + i, swap ? sub(inp[i + 4], inp[i]) : 0);
      u64 s[12];
      for (int i = 0; i < 12; i++) s[i] = inp[i];
      if (swap) for (int i = 0; i < 4; i++) std::swap(s[i], s[i + 4]);
      // the naive permutation, recording every S-box input (Hash/Poseidon.hs:50-101)
      auto mds = [&]() { u64 t[12]; for (int i = 0; i < 12; i++) { u64 a = 0; for (int j = 0; j < 12; j++) a = add(a, mul(p2::mds_coeff(i, j), s[j])); t[i] = a; } memcpy(s, t, sizeof t); };
      for (int r = 0; r < 30; r++) {
        for (int i = 0; i < 12; i++) s[i] = add(s[i], ROUND_CONSTANTS[12 * r + i]);
        const bool full = r < 4 || r >= 26;
        if (r >= 1 && r < 4) for (int i = 0; i < 12; i++) put(PW_ISB + 12 * (r - 1) + i, s[i]);
        if (r >= 26) for (int i = 0; i < 12; i++) put(PW_FSB + 12 * (r - 26) + i, s[i]);
        if (!full) put(PW_PSB + (r - 4), s[0]);
        if (full) for (int i = 0; i < 12; i++) s[i] = sbox(s[i]); else s[0] = sbox(s[0]);
        mds();
      }
      u64 chk[12]; memcpy(chk, inp, sizeof chk);
      if (swap) for (int i = 0; i < 4; i++) std::swap(chk[i], chk[i + 4]);
      p2::permute(chk);   // the hashing permutation (KAT-pinned) must agree with the recorded run
      for (int i = 0; i < 12; i++) { if (gl::canon(chk[i]) != s[i]) throw std::runtime_error("gen: poseidon witness mismatch"); put(12 + i, s[i]); }
      break; }
    case POSEIDON_MDS:
      for (int i = 0; i < 12; i++) {
        E a = gl::e0();
        for (int j = 0; j < 12; j++) a = gl::eadd(a, gl::escale(p2::mds_coeff(i, j), inx(2 * j)));
        putx(2 * (i + 12), a);
      }
      break;
    case RANDACC: {
      const int nb = (int)g.p0; const int64_t copies = g.p1, extra = g.p2;
      const int64_t veclen = (int64_t)1 << nb, width = 2 + veclen, bstart = width * copies + extra;
      for (int64_t kk = 0; kk < copies; kk++) {
        const u64 idx = rg.next() & (u64)(veclen - 1);
        put(kk * width, idx);
        for (int64_t i = 0; i < veclen; i++) in(kk * width + 2 + i);
        put(kk * width + 1, w[kk * width + 2 + idx]);
        for (int j = 0; j < nb; j++) put(bstart + kk * nb + j, (idx >> j) & 1);
      }
      for (int64_t j = 0; j < extra; j++) put(copies * width + j, k[j]);
      break; }
    case REDUCING: case REDUCING_EXT: {   // output = old alpha^n + sum_i c_i alpha^(n-1-i)
      const int64_t n = g.p0; const bool ext = g.kind == REDUCING_EXT;
      const int64_t acc0 = ext ? 6 + 2 * n : 6 + n;
      const E alpha = inx(2), old = inx(4);
      std::vector<E> co(n);
      for (int64_t i = 0; i < n; i++) co[i] = ext ? inx(6 + 2 * i) : gl::eb(in(6 + i));
      E out = old; for (int64_t i = 0; i < n; i++) out = gl::emul(out, alpha);
      E ap = gl::eb(1);
      for (int64_t i = n - 1; i >= 0; i--) { out = gl::eadd(out, gl::emul(co[i], ap)); ap = gl::emul(ap, alpha); }
      E acc = old;
      for (int64_t i = 0; i < n - 1; i++) { acc = gl::eadd(gl::emul(acc, alpha), co[i]); putx(acc0 + 2 * i, acc); }
      putx(0, out);
      break; }
    case COSET: {
      const CosetLayout L = coset_layout(g);
      const u64 gen = gl::subgroup_gen((int)g.p0);
      u64 shift; do { shift = rg.field(); } while (shift == 0);
      put(0, shift);
      std::vector<E> v(L.npts);
      for (int64_t kk = 0; kk < L.npts; kk++) v[kk] = inx(L.val(kk));
      const E loc = inx(L.eval_loc());
      putx(L.eval_result(), lagrange_eval(shift, gen, v, loc));
      const E shifted = gl::escale(gl::inv(shift), loc);
      putx(L.shifted(), shifted);
      auto ch = L.chunks();   // intermediate running (eval, prod) pairs of the chunked barycentric sum
      E ev = gl::e0(), pr = gl::eb(1);
      for (size_t ci = 0; ci + 1 < std::min((size_t)L.nint + 1, ch.size()); ci++) {
        for (int64_t kk = ch[ci].first; kk < ch[ci].second; kk++) {
          const E term = gl::esub(shifted, gl::eb(gl::pow(gen, (u64)kk)));
          ev = gl::eadd(gl::emul(term, ev), gl::emul(gl::escale(g.weights[kk], v[kk]), pr)); pr = gl::emul(term, pr);
        }
        putx(L.tmp_eval(ci), ev); putx(L.tmp_prod(ci), pr);
      }
      break; }
    case NOOP: case LOOKUP: case LOOKUPTABLE: break;
  }
  for (int i = 0; i < nw; i++) if (!set[i] && !pre[i]) w[i] = rg.field();   // unused wires
}

}  // namespace gg
