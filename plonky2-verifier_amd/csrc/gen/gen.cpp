// gen.cpp — synthetic valid-proof generator (workload + fixture source, NOT part of the
// verifier path).  A degenerate-circuit Plonky2 prover:
//
//   * every gate-selector constant column is the constant UNUSED = 2^32-1 and there are
//     >= 2 selector groups, so every gate filter (Gate/Selector.hs:83-89) is 0 at zeta;
//   * lookup-selector columns are 0 (every lookup term carries a selector, Lookups.hs:78-132);
//   * sigma_j(X) = k_j X, so the permutation numerators equal the denominators
//     (Vanishing.hs:99-111) with Z == partial products == 1;
//   * quotient polynomials are 0.
// Hence C(zeta) = 0 = Q(zeta)(zeta^n - 1) and the Plonk identity holds, while the verifier
// still evaluates every gate program, lookup argument and the whole FRI proof.  Wires,
// gate constants and lookup_zs are random polynomials of degree < n, so proofs differ.
// The FRI part is a real prover: LDE on g*H in bit-reversed order, Merkle trees with caps,
// openings at zeta / omega*zeta, the combined quotient codeword, arity-2^k folding with
// commit-phase trees, final polynomial, proof-of-work grinding and query openings, all
// following the verifier conventions of Plonk/FRI.hs and Challenge/*.hs.
//
// A second mode ("real", p2v_gen_circuit_new2) proves a genuine circuit instead: every gate
// of the recursion gate set placed on rows, selector polynomials that pick each row's gate
// (Gate/Selector.hs:83-95), gate constants per row, copy constraints with a real sigma
// permutation, the running product Z and its partial products (Vanishing.hs:97-111), and the
// quotient C(X)/Z_H(X) computed on a 16n-point coset and split into qdf chunks
// (Verifier.hs:43-51).  Witness rows follow plonky2's gate semantics (gates.hpp), so every
// vanishing term of a valid proof is a non-zero value at zeta.
//
// Exposed as a C ABI (libp2v_gen.so) for tests/ and bench.py.
#include <algorithm>
#include <thread>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <string>
#include <vector>
#include <memory>
#include <stdexcept>
#include "../gl.h"
#include "../poseidon.h"
#include "gates.hpp"

using gl::E;
using u64 = uint64_t;

namespace {

// ------------------------------------------------------------------------ rng
struct Rng {
  u64 s;
  explicit Rng(u64 seed) : s(seed ^ 0x9E3779B97F4A7C15ULL) {}
  u64 next() {  // splitmix64
    u64 z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
  }
  u64 field() { for (;;) { u64 x = next(); if (x < gl::P) return x; } }
};

// ------------------------------------------------------------------ hashing
void sponge(const u64* xs, size_t n, u64 out[4]) {
  u64 st[12] = {0};
  for (size_t i = 0; i < n; i += 8) {
    size_t k = n - i < 8 ? n - i : 8;
    for (size_t j = 0; j < k; j++) st[j] = xs[i + j];
    p2::permute(st);
  }
  memcpy(out, st, 32);
}
// a Merkle leaf's digest: the sponge (Hash/Merkle.hs:27-28), or under the hash_or_noop
// extension (P2V_EXT_HASH_OR_NOOP) a leaf of <= 4 elements zero-padded (plonky2 hash_or_noop)
void leaf_digest(const u64* xs, size_t n, bool noop, u64 out[4]) {
  if (noop && n <= 4) { memset(out, 0, 32); memcpy(out, xs, n * 8); return; }
  sponge(xs, n, out);
}
void compress(const u64* a, const u64* b, u64 out[4]) {
  u64 st[12] = {0};
  memcpy(st, a, 32); memcpy(st + 4, b, 32);
  p2::permute(st);
  memcpy(out, st, 32);
}

struct Digest { u64 e[4]; };

// Merkle tree over n = 2^lg leaves (leaf digests given), cap of 2^cap_h nodes.
struct Tree {
  int lg = 0, cap_h = 0;
  std::vector<std::vector<Digest>> layers;   // layers[0] = leaf digests
  void build(std::vector<Digest>&& leaves, int lg_, int cap_h_) {
    lg = lg_; cap_h = cap_h_;
    layers.clear(); layers.push_back(std::move(leaves));
    for (int l = lg; l > cap_h; l--) {
      const auto& prev = layers.back();
      std::vector<Digest> nx(prev.size() / 2);
      for (size_t i = 0; i < nx.size(); i++) compress(prev[2 * i].e, prev[2 * i + 1].e, nx[i].e);
      layers.push_back(std::move(nx));
    }
  }
  const std::vector<Digest>& cap() const { return layers.back(); }
  std::vector<Digest> path(size_t idx) const {
    std::vector<Digest> sib;
    for (size_t l = 0; l + 1 < layers.size(); l++) { sib.push_back(layers[l][idx ^ 1]); idx >>= 1; }
    return sib;
  }
};

// ------------------------------------------------------------------ FFT
// in-place radix-2 DIT FFT of size 2^lg with generator w (natural order in / out)
void fft(std::vector<u64>& a, int lg, u64 w) {
  size_t n = (size_t)1 << lg;
  for (size_t i = 1, j = 0; i < n; i++) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) std::swap(a[i], a[j]);
  }
  std::vector<u64> tw(n / 2);
  for (size_t len = 2; len <= n; len <<= 1) {
    u64 wl = w;
    for (size_t t = len; t < n; t <<= 1) wl = gl::mul(wl, wl);   // w^(n/len)
    tw[0] = 1;
    for (size_t k = 1; k < len / 2; k++) tw[k] = gl::mul(tw[k - 1], wl);
    for (size_t i = 0; i < n; i += len)
      for (size_t k = 0; k < len / 2; k++) {
        u64 u = a[i + k], v = gl::mul(a[i + k + len / 2], tw[k]);
        a[i + k] = gl::add(u, v); a[i + k + len / 2] = gl::sub(u, v);
      }
  }
}
void efft(std::vector<E>& a, int lg, u64 w) {
  std::vector<u64> re(a.size()), im(a.size());
  for (size_t i = 0; i < a.size(); i++) { re[i] = a[i].a; im[i] = a[i].b; }
  fft(re, lg, w); fft(im, lg, w);
  for (size_t i = 0; i < a.size(); i++) a[i] = E{re[i], im[i]};
}

// LDE of a coefficient vector (length N) onto g*<eta> of size 2^lde, natural order
std::vector<u64> lde(const std::vector<u64>& coeffs, int lde_bits) {
  size_t M = (size_t)1 << lde_bits;
  std::vector<u64> a(M, 0);
  u64 gp = 1;
  for (size_t k = 0; k < coeffs.size(); k++) { a[k] = gl::mul(coeffs[k], gp); gp = gl::mul(gp, gl::MULT_GEN); }
  fft(a, lde_bits, gl::subgroup_gen(lde_bits));
  return a;
}

E eval_at(const std::vector<u64>& coeffs, E x) {   // Horner, base coefficients at F^2 point
  E acc = gl::e0();
  for (size_t k = coeffs.size(); k-- > 0;) acc = gl::eadd(gl::emul(acc, x), gl::eb(coeffs[k]));
  return acc;
}

void batch_inv(std::vector<E>& v) {   // Montgomery trick (no zeros expected)
  size_t n = v.size();
  std::vector<E> pre(n);
  E acc = gl::eb(1);
  for (size_t i = 0; i < n; i++) { pre[i] = acc; acc = gl::emul(acc, v[i]); }
  E inv = gl::einv(acc);
  for (size_t i = n; i-- > 0;) { E t = gl::emul(inv, pre[i]); inv = gl::emul(inv, v[i]); v[i] = t; }
}

// ------------------------------------------------------------------ duplex (Challenge/Pure.hs)
struct Duplex {
  u64 st[12] = {0};
  bool absorbing = true;
  u64 buf[8]; int nbuf = 0;
  u64 out[8]; int nout = 0, pos = 0;
  void dup() { for (int i = 0; i < nbuf; i++) st[i] = buf[i]; p2::permute(st); }
  void fresh() { absorbing = false; for (int i = 0; i < 8; i++) out[i] = st[7 - i]; nout = 8; pos = 0; }
  void absorb(u64 x) {
    if (!absorbing) { absorbing = true; nbuf = 0; }
    if (nbuf < 8) { buf[nbuf++] = x; return; }
    dup(); nbuf = 0; buf[nbuf++] = x;
  }
  u64 squeeze() {
    if (absorbing) { dup(); nbuf = 0; fresh(); }
    else if (pos == nout) { p2::permute(st); fresh(); }
    return out[pos++];
  }
  E squeeze_e() { E r; r.a = squeeze(); r.b = squeeze(); return r; }
  void absorb_digests(const std::vector<Digest>& ds) { for (auto& d : ds) for (int i = 0; i < 4; i++) absorb(d.e[i]); }
  void absorb_e(const std::vector<E>& v) { for (auto& x : v) { absorb(x.a); absorb(x.b); } }
};

// ------------------------------------------------------------------ JSON helpers
struct J {
  std::string s;
  void raw(const char* t) { s += t; }
  void u(u64 x) { char b[32]; snprintf(b, sizeof b, "%llu", (unsigned long long)x); s += b; }
  void i(long long x) { char b[32]; snprintf(b, sizeof b, "%lld", x); s += b; }
  void digest(const Digest& d) { raw("{\"elements\":["); for (int k = 0; k < 4; k++) { if (k) raw(","); u(d.e[k]); } raw("]}"); }
  void cap(const std::vector<Digest>& c) { raw("["); for (size_t k = 0; k < c.size(); k++) { if (k) raw(","); digest(c[k]); } raw("]"); }
  void fs(const u64* v, size_t n) { raw("["); for (size_t k = 0; k < n; k++) { if (k) raw(","); u(v[k]); } raw("]"); }
  void es(const std::vector<E>& v) { raw("["); for (size_t k = 0; k < v.size(); k++) { if (k) raw(","); raw("["); u(v[k].a); raw(","); u(v[k].b); raw("]"); } raw("]"); }
};

// ------------------------------------------------------------------ circuit
struct Circuit {
  int degree_bits = 12, rate_bits = 3, cap_height = 4, pow_bits = 16, num_queries = 28;
  int arity_bits = 4, final_poly_bits = 5;
  // opt-in plonky2 conventions (include/p2v.h P2V_EXT_*): 1 the steps are `arity_seq` written as
  // fri_params.reduction_arity_bits under a MinSize strategy; 2 hiding (4 salts per wires / zs /
  // quotient leaf); 4 hash_or_noop leaves.  arity_seq without bit 1: a Fixed strategy.
  unsigned ext = 0;
  std::vector<int> arity_seq;
  int num_wires = 135, num_routed = 80, num_gate_consts = 2, r = 2, qdf = 8;
  int num_pis = 4;
  int ngroups = 3;
  std::vector<int> grp_s, grp_e;   // selector groups [start, end) (SelectorsInfo, Types.hs:90-101)
  u64 sel_fill = 0xFFFFFFFFULL;    // degenerate mode: the constant selector column value
  int nlp = 0;                 // num_lookup_polys (0 = no lookups)
  std::vector<std::vector<std::pair<u64, u64>>> luts;
  std::vector<std::string> gates;
  std::vector<int> sel_idx;
  std::vector<u64> k_is;
  int npp = 9;                 // num_partial_products
  int num_gate_constraints = 123;
  u64 circuit_seed = 1;
  // derived
  int N = 0, lde_bits = 0, nls = 0, num_constants = 0;
  std::vector<int> arities;
  std::vector<std::vector<u64>> gate_const_coeffs;   // random polys
  std::vector<u64> const_lde;                         // [M][85] bit-reversed rows of the constants oracle
  int const_width = 0;
  Tree const_tree;
  Digest circuit_digest;
  std::string common_json, vkey_json;
  // ---- real mode
  bool real = false;
  int gate_set = 0;                                   // 0: recursion set, 1: small set (one selector group)
  std::vector<gg::Gate> G;                            // gates in circuit order (ascending degree)
  std::vector<int> row_gate;                          // [N]
  std::vector<u64> row_consts;                        // [N][num_gate_consts]
  std::vector<std::pair<int64_t, int64_t>> links;     // (dst, src) wire positions row*num_wires+wire, dst rows ascending
  std::vector<std::vector<u64>> const_coeffs;         // constants-oracle columns as coefficient vectors
  std::vector<std::vector<u64>> const_q;              // the same columns on the quotient coset (16N points)
  std::vector<std::vector<u64>> const_h;              // the same columns on H (natural order)
  int q_bits = 0;                                     // log2 of the quotient coset size
  int max_constraints = 0;
  // real mode with lookup tables (commentary/Lookups.md "Layout"): one block of rows per table,
  // in row order [LookupGate rows | LookupTableGate rows | NoopGate row].  The running sums read
  // the block bottom-up (Plonk/Lookups.hs:112-132: RE and SLDC at x take their "next" at omega x).
  struct LkBlock { int table, lu0, nlu, lut0, nlut, noop; };
  std::vector<LkBlock> lblocks;
  std::vector<int8_t> row_lk;                         // [N]: 0 none, 1 LookupGate, 2 LookupTableGate, 3 the block's Noop
  std::vector<int> row_block;                         // [N]: the block of a lookup row (-1 none)
};

// lookup geometry of a circuit (Plonk/Lookups.hs:64-68)
struct LkGeom {
  int lu_slots, lut_slots, nsl, lu_deg, lut_deg;
  explicit LkGeom(const Circuit& C)
      : lu_slots(C.num_routed / 2), lut_slots(C.num_routed / 3), nsl(C.nlp - 1), lu_deg(C.qdf - 1),
        lut_deg(C.nlp > 1 ? (C.num_routed / 3 + C.nlp - 2) / (C.nlp - 1) : 1) {}
  // zip truncation of prevThisPairs with the three chunk lists (:115-116)
  int npairs() const {
    const int clu = (lu_slots + lu_deg - 1) / lu_deg, clut = (lut_slots + lut_deg - 1) / lut_deg;
    return std::min(nsl, std::min(clu, clut));
  }
};

std::string coset_gate_string(int bits) {
  // CosetInterpolationGate with barycentric weights of the subgroup (CosetInterp.hs:36-49)
  int n = 1 << bits;
  u64 g = gl::subgroup_gen(bits);
  std::vector<u64> pts(n); pts[0] = 1; for (int i = 1; i < n; i++) pts[i] = gl::mul(pts[i - 1], g);
  std::string w = "[";
  for (int i = 0; i < n; i++) {
    u64 prod = 1;
    for (int j = 0; j < n; j++) if (j != i) prod = gl::mul(prod, gl::sub(pts[i], pts[j]));
    if (i) w += ", ";
    w += std::to_string((unsigned long long)gl::inv(prod));
  }
  w += "]";
  int max_degree = 8;
  int n_int_guess = (n - 2) / (max_degree - 1);
  int degree = (n - 2) / (n_int_guess + 1) + 2;
  return "CosetInterpolationGate { subgroup_bits: " + std::to_string(bits) + ", degree: " + std::to_string(degree) +
         ", barycentric_weights: " + w + ", _phantom: PhantomData<plonky2_field::goldilocks_field::GoldilocksField> }<D=2>";
}

std::string keccak_str(u64 seed) {
  Rng rg(seed); std::string s = "[";
  for (int i = 0; i < 32; i++) { if (i) s += ", "; s += std::to_string((unsigned)(rg.next() & 255)); }
  return s + "]";
}

// values on H = <omega> (natural order) -> coefficients
std::vector<u64> interpolate(std::vector<u64> v, int lg) {
  fft(v, lg, gl::inv(gl::subgroup_gen(lg)));
  const u64 inv_n = gl::inv((u64)v.size());
  for (auto& x : v) x = gl::mul(x, inv_n);
  return v;
}

// rows of an oracle on the LDE coset g<eta>, bit-reversed order: rows[idx][col]
std::vector<u64> oracle_rows(const std::vector<std::vector<u64>>& cols, int lde_bits) {
  const size_t M = (size_t)1 << lde_bits, W = cols.size();
  std::vector<u64> rows(M * W);
  for (size_t c = 0; c < W; c++) {
    auto l = lde(cols[c], lde_bits);
    for (size_t idx = 0; idx < M; idx++) rows[idx * W + c] = l[gl::rev_bits(lde_bits, (uint32_t)idx)];
  }
  return rows;
}

template <class Fn> void parallel_for(size_t n, Fn fn) {
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (n < 64) nt = 1;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; t++) th.emplace_back([&, t] { for (size_t i = t; i < n; i += nt) fn(i); });
  for (auto& x : th) x.join();
}

gg::Gate mkgate(gg::Kind k, int64_t p0, int64_t p1, int64_t p2, std::string str) {
  gg::Gate g; g.kind = k; g.p0 = p0; g.p1 = p1; g.p2 = p2; g.str = std::move(str); return g;
}

// total degree of a gate's constraints in the wires and constants: evaluate along a random
// line (w = a + t b) and read off the degree in t from forward differences
int measure_degree(const gg::Gate& g, int nw, int nk, Rng& rg) {
  const int D = 12;
  std::vector<u64> a(nw), b(nw), ka(nk), kb(nk), pih(4);
  for (auto& x : a) x = rg.field();
  for (auto& x : b) x = rg.field();
  for (auto& x : ka) x = rg.field();
  for (auto& x : kb) x = rg.field();
  for (auto& x : pih) x = rg.field();
  std::vector<std::vector<u64>> vals;
  std::vector<u64> w(nw), k(nk);
  for (int t = 0; t < D; t++) {
    for (int i = 0; i < nw; i++) w[i] = gl::add(a[i], gl::mul((u64)t, b[i]));
    for (int i = 0; i < nk; i++) k[i] = gl::add(ka[i], gl::mul((u64)t, kb[i]));
    std::vector<u64> out;
    gg::eval(g, w.data(), nw, k.data(), nk, pih.data(), out);
    vals.push_back(std::move(out));
  }
  int deg = 0;
  for (size_t c = 0; c < vals[0].size(); c++) {
    std::vector<u64> d(D);
    for (int t = 0; t < D; t++) d[t] = vals[t][c];
    int dc = -1;
    for (int m = 0; m < D; m++) {   // d holds the m-th differences
      for (int t = 0; t + m < D; t++) if (d[t] != 0) { dc = m; break; }
      for (int t = 0; t + m + 1 < D; t++) d[t] = gl::sub(d[t + 1], d[t]);
    }
    if (dc >= D - 2) throw std::runtime_error("gen: constraint degree too high to measure");
    deg = std::max(deg, dc);
  }
  return deg;
}

void build_real(Circuit& C) {
  const int N = C.N, NW = C.num_wires, NR = C.num_routed, NK = C.num_gate_consts;
  Rng rg(C.circuit_seed * 7919 + 17);
  for (int i = 0; i < 4; i++) C.circuit_digest.e[i] = rg.field();
  const std::string PH = "_phantom: PhantomData<plonky2_field::goldilocks_field::GoldilocksField>";
  using namespace gg;
  if (C.gate_set == 1) {
    C.G = { mkgate(NOOP, 0, 0, 0, "NoopGate"), mkgate(CONST, 2, 0, 0, "ConstantGate { num_consts: 2 }"),
            mkgate(PI, 0, 0, 0, "PublicInputGate"), mkgate(ARITH, 20, 0, 0, "ArithmeticGate { num_ops: 20 }") };
  } else {
    C.G = {
      mkgate(NOOP, 0, 0, 0, "NoopGate"),
      mkgate(CONST, 2, 0, 0, "ConstantGate { num_consts: 2 }"),
      mkgate(POSEIDON_MDS, 12, 0, 0, "PoseidonMdsGate(PhantomData<plonky2_field::goldilocks_field::GoldilocksField>)<WIDTH=12>"),
      mkgate(PI, 0, 0, 0, "PublicInputGate"),
      mkgate(BASESUM, 63, 2, 0, "BaseSumGate { num_limbs: 63 } + Base: 2"),
      mkgate(REDUCING_EXT, 32, 0, 0, "ReducingExtensionGate { num_coeffs: 32 }"),
      mkgate(REDUCING, 43, 0, 0, "ReducingGate { num_coeffs: 43 }"),
      mkgate(ARITH_EXT, 10, 0, 0, "ArithmeticExtensionGate { num_ops: 10 }"),
      mkgate(ARITH, 20, 0, 0, "ArithmeticGate { num_ops: 20 }"),
      mkgate(MULEXT, 13, 0, 0, "MulExtensionGate { num_ops: 13 }"),
      mkgate(RANDACC, 4, 4, 2, "RandomAccessGate { bits: 4, num_copies: 4, num_extra_constants: 2, " + PH + " }<D=2>"),
      mkgate(EXP, 66, 0, 0, "ExponentiationGate { num_power_bits: 66 }"),
      mkgate(COSET, 4, 6, 0, coset_gate_string(4)),
      mkgate(POSEIDON, 12, 0, 0, "PoseidonGate(PhantomData<plonky2_field::goldilocks_field::GoldilocksField>)<WIDTH=12>"),
    };
    auto& cg = C.G[12];   // the barycentric weights, as the gate string carries them
    const int n = 16; const u64 gsub = gl::subgroup_gen(4);
    std::vector<u64> pts(n); pts[0] = 1; for (int i = 1; i < n; i++) pts[i] = gl::mul(pts[i - 1], gsub);
    for (int i = 0; i < n; i++) { u64 pr = 1; for (int j = 0; j < n; j++) if (j != i) pr = gl::mul(pr, gl::sub(pts[i], pts[j])); cg.weights.push_back(gl::inv(pr)); }
  }
  // lookup tables: one block per table at the end of the rows, [LU | LUT | Noop] in row order;
  // a LUT row holds 26 (inp, out, mult) slots, a LU row 40 (inp, out) pairs (Lookups.hs:64-65).
  // Table entries fill the LUT rows from the bottom up (Lookups.md "Layout"): RE(x) = delta^26
  // RE(omega x) + row(x) then equals evalFinalRE's Horner over the table at the top LUT row.
  C.lblocks.clear();
  C.row_lk.assign(N, 0);
  C.row_block.assign(N, -1);
  if (!C.luts.empty()) {
    const LkGeom lg(C);
    std::vector<Circuit::LkBlock> bl;
    int total = 0;
    for (size_t t = 0; t < C.luts.size(); t++) {
      Circuit::LkBlock b{};
      b.table = (int)t;
      b.nlut = (int)((C.luts[t].size() + lg.lut_slots - 1) / lg.lut_slots);
      b.nlu = 1 + b.nlut / 32;
      total += b.nlu + b.nlut + 1;
      bl.push_back(b);
    }
    int row = N - total;
    if (row < (int)C.G.size()) throw std::runtime_error("gen: the lookup tables do not fit in 2^degree_bits rows");
    for (auto& b : bl) {
      b.lu0 = row; b.lut0 = b.lu0 + b.nlu; b.noop = b.lut0 + b.nlut; row = b.noop + 1;
      for (int i = b.lu0; i < b.lut0; i++) C.row_lk[i] = 1;
      for (int i = b.lut0; i < b.noop; i++) C.row_lk[i] = 2;
      C.row_lk[b.noop] = 3;
      for (int i = b.lu0; i <= b.noop; i++) C.row_block[i] = (int)C.lblocks.size();
      C.lblocks.push_back(b);
      const std::string h = keccak_str(100 + b.table);
      C.G.push_back(mkgate(LOOKUP, lg.lu_slots, b.table, 0, "LookupGate { num_slots: " + std::to_string(lg.lu_slots) + ", lut_hash: " + h + " }"));
      C.G.push_back(mkgate(LOOKUPTABLE, lg.lut_slots, b.table, 0, "LookupTableGate { num_slots: " + std::to_string(lg.lut_slots) +
                                                                   ", lut_hash: " + h + ", last_lut_row: " + std::to_string(b.noop - 1) + " }"));
    }
  }
  // degrees, sorted ascending (plonky2 orders a circuit's gates by degree), selector groups:
  // one group if max_deg + #gates - 1 <= qdf, else greedy ranges with size + degree <= qdf
  Rng drg(99);
  for (auto& g : C.G) g.degree = measure_degree(g, NW, NK, drg);
  std::stable_sort(C.G.begin(), C.G.end(), [](const gg::Gate& x, const gg::Gate& y) { return x.degree < y.degree; });
  const int NG = (int)C.G.size();
  C.gates.clear();
  for (auto& g : C.G) C.gates.push_back(g.str);
  C.grp_s.clear(); C.grp_e.clear();
  if (C.G.back().degree + NG - 1 <= C.qdf) { C.grp_s = {0}; C.grp_e = {NG}; }
  else {
    for (int st = 0; st < NG;) {
      int sz = 0;
      while (st + sz < NG && sz + C.G[st + sz].degree < C.qdf) sz++;
      if (sz == 0) throw std::runtime_error("gen: a gate's degree exceeds the quotient degree");
      C.grp_s.push_back(st); C.grp_e.push_back(st + sz); st += sz;
    }
  }
  C.ngroups = (int)C.grp_s.size();
  C.sel_idx.assign(NG, 0);
  for (int g = 0; g < C.ngroups; g++) for (int k = C.grp_s[g]; k < C.grp_e[g]; k++) C.sel_idx[k] = g;
  C.num_constants = C.ngroups + C.nls + NK;
  C.max_constraints = 0;
  {
    std::vector<u64> w(NW, 1), k(NK, 1), pih(4, 0), out;
    for (auto& g : C.G) { out.clear(); gg::eval(g, w.data(), NW, k.data(), NK, pih.data(), out); C.max_constraints = std::max(C.max_constraints, (int)out.size()); }
  }
  C.num_gate_constraints = C.max_constraints;
  // rows: every gate once, then random gates; row constants random where the gate reads them.
  // Lookup gates appear only in their tables' blocks (with the blocks' Noop rows).
  std::vector<int> plain;
  int noop_idx = -1;
  for (int k = 0; k < NG; k++) {
    if (C.G[k].kind == gg::NOOP) noop_idx = k;
    if (C.G[k].kind != gg::LOOKUP && C.G[k].kind != gg::LOOKUPTABLE) plain.push_back(k);
  }
  C.row_gate.assign(N, 0);
  for (int i = 0; i < N; i++) {
    if (C.row_lk[i]) {
      const auto& b = C.lblocks[C.row_block[i]];
      int k = noop_idx;
      for (int m = 0; m < NG && C.row_lk[i] != 3; m++)
        if (C.G[m].p1 == b.table && C.G[m].kind == (C.row_lk[i] == 1 ? gg::LOOKUP : gg::LOOKUPTABLE)) k = m;
      if (k < 0) throw std::runtime_error("gen: a lookup block needs a NoopGate");
      C.row_gate[i] = k;
    } else {
      C.row_gate[i] = i < (int)plain.size() ? plain[i] : plain[rg.next() % (u64)plain.size()];
    }
  }
  C.row_consts.assign((size_t)N * NK, 0);
  for (int i = 0; i < N; i++) {
    int nc = gg::num_row_constants(C.G[C.row_gate[i]]);
    if (nc > NK) throw std::runtime_error("gen: gate needs more constants than the config has");
    for (int c = 0; c < nc; c++) C.row_consts[(size_t)i * NK + c] = rg.field();
  }
  // copy constraints: a free routed input of a later row copies any routed wire of an earlier row
  C.links.clear();
  for (int i = 1; i < N; i++)
    for (int wi : gg::free_inputs(C.G[C.row_gate[i]], NW)) {
      if (wi >= NR || rg.next() % 6 != 0) continue;
      const int64_t src = (int64_t)(rg.next() % (u64)i) * NW + (int64_t)(rg.next() % (u64)NR);
      C.links.push_back({(int64_t)i * NW + wi, src});
    }
  // sigma: the copy classes (union-find over routed positions j*N + i) as cycles in position order
  const size_t NP = (size_t)NR * N;
  std::vector<uint32_t> par(NP);
  for (size_t p = 0; p < NP; p++) par[p] = (uint32_t)p;
  auto find = [&](uint32_t x) { while (par[x] != x) { par[x] = par[par[x]]; x = par[x]; } return x; };
  auto rpos = [&](int64_t wp) { return (uint32_t)((wp % NW) * N + wp / NW); };
  for (auto& l : C.links) { uint32_t a = find(rpos(l.first)), b = find(rpos(l.second)); if (a != b) par[std::max(a, b)] = std::min(a, b); }
  std::vector<uint32_t> sigma(NP), last(NP, UINT32_MAX), first(NP, UINT32_MAX);
  for (size_t p = 0; p < NP; p++) {
    uint32_t r = find((uint32_t)p);
    if (first[r] == UINT32_MAX) first[r] = (uint32_t)p; else sigma[last[r]] = (uint32_t)p;
    last[r] = (uint32_t)p;
  }
  for (size_t p = 0; p < NP; p++) if (find((uint32_t)p) == p) sigma[last[p]] = first[p];
  // constant columns on H: [selectors | gate constants | sigmas]
  const u64 omega = gl::subgroup_gen(C.degree_bits);
  std::vector<u64> om(N); om[0] = 1; for (int i = 1; i < N; i++) om[i] = gl::mul(om[i - 1], omega);
  std::vector<std::vector<u64>> cols;
  for (int g = 0; g < C.ngroups; g++) {
    std::vector<u64> v(N);
    for (int i = 0; i < N; i++) { int k = C.row_gate[i]; v[i] = C.sel_idx[k] == g ? (u64)k : 0xFFFFFFFFULL; }
    cols.push_back(std::move(v));
  }
  // lookup selectors (commentary/Lookups.md "Lookup selectors"; Lookups.hs:27-41): TransSre on
  // the LUT rows, TransLdc on the LU rows, InitSre on each block's Noop row, LastLdc on each
  // block's first LU row, StartEnd_t on the first LUT row of table t
  for (int s = 0; s < C.nls; s++) {
    std::vector<u64> v(N, 0);
    for (const auto& b : C.lblocks) {
      if (s == 0) for (int i = b.lut0; i < b.noop; i++) v[i] = 1;
      if (s == 1) for (int i = b.lu0; i < b.lut0; i++) v[i] = 1;
      if (s == 2) v[b.noop] = 1;
      if (s == 3) v[b.lu0] = 1;
      if (s == 4 + b.table) v[b.lut0] = 1;
    }
    cols.push_back(std::move(v));
  }
  for (int c = 0; c < NK; c++) { std::vector<u64> v(N); for (int i = 0; i < N; i++) v[i] = C.row_consts[(size_t)i * NK + c]; cols.push_back(std::move(v)); }
  for (int j = 0; j < NR; j++) {
    std::vector<u64> v(N);
    for (int i = 0; i < N; i++) { uint32_t t = sigma[(size_t)j * N + i]; v[i] = gl::mul(C.k_is[t / N], om[t % N]); }
    cols.push_back(std::move(v));
  }
  C.const_width = (int)cols.size();
  C.const_h = cols;
  C.const_coeffs.resize(cols.size());
  parallel_for(cols.size(), [&](size_t c) { C.const_coeffs[c] = interpolate(cols[c], C.degree_bits); });
  C.const_lde = oracle_rows(C.const_coeffs, C.lde_bits);
  C.q_bits = C.degree_bits + 4;   // >= (qdf + 1) n points
  C.const_q.resize(cols.size());
  parallel_for(cols.size(), [&](size_t c) { C.const_q[c] = lde(C.const_coeffs[c], C.q_bits); });
}

void build_circuit(Circuit& C) {
  C.N = 1 << C.degree_bits;
  C.lde_bits = C.degree_bits + C.rate_bits;
  C.nls = C.luts.empty() ? 0 : 4 + (int)C.luts.size();
  C.num_constants = C.ngroups + C.nls + C.num_gate_consts;
  C.npp = (C.num_routed + C.qdf - 1) / C.qdf - 1;
  C.arities.clear();
  if (!C.arity_seq.empty()) C.arities = C.arity_seq;
  else for (int logn = C.degree_bits; logn > C.final_poly_bits; logn -= C.arity_bits) C.arities.push_back(C.arity_bits);
  { int sa = 0; for (int a : C.arities) sa += a; if (sa > C.degree_bits) throw std::runtime_error("gen: FRI arities fold below degree 1"); }
  C.k_is.resize(C.num_routed);
  { u64 k = 1; for (int i = 0; i < C.num_routed; i++) { C.k_is[i] = k; k = gl::mul(k, gl::MULT_GEN); } }
  size_t M = (size_t)1 << C.lde_bits;
  if (C.real) build_real(C);
  else {
    if (C.gates.empty()) {
      C.gates = {
        "NoopGate",
        "ConstantGate { num_consts: 2 }",
        "PoseidonMdsGate(PhantomData<plonky2_field::goldilocks_field::GoldilocksField>)<WIDTH=12>",
        "PublicInputGate",
        "BaseSumGate { num_limbs: 63 } + Base: 2",
        "ReducingExtensionGate { num_coeffs: 32 }",
        "ReducingGate { num_coeffs: 43 }",
        "ArithmeticExtensionGate { num_ops: 10 }",
        "ArithmeticGate { num_ops: 20 }",
        "MulExtensionGate { num_ops: 13 }",
        "RandomAccessGate { bits: 4, num_copies: 4, num_extra_constants: 2, _phantom: PhantomData<plonky2_field::goldilocks_field::GoldilocksField> }<D=2>",
        "ExponentiationGate { num_power_bits: 66 }",
        coset_gate_string(4),
        "PoseidonGate(PhantomData<plonky2_field::goldilocks_field::GoldilocksField>)<WIDTH=12>",
      };
      if (!C.luts.empty()) {
        for (size_t t = 0; t < C.luts.size(); t++) {
          C.gates.insert(C.gates.begin() + 1, "LookupTableGate { num_slots: 26, lut_hash: " + keccak_str(100 + t) +
                                                 ", last_lut_row: " + std::to_string((C.luts[t].size() + 25) / 26) + " }");
          C.gates.insert(C.gates.begin() + 1, "LookupGate { num_slots: 40, lut_hash: " + keccak_str(100 + t) + " }");
        }
      }
    }
    C.sel_idx.assign(C.gates.size(), 0);
    {  // split gates into ngroups contiguous groups
      size_t per = (C.gates.size() + C.ngroups - 1) / C.ngroups;
      for (size_t g = 0; g < C.gates.size(); g++) C.sel_idx[g] = (int)(g / per);
      C.ngroups = C.sel_idx.back() + 1;
      C.num_constants = C.ngroups + C.nls + C.num_gate_consts;
      C.grp_s.clear(); C.grp_e.clear();
      for (int g = 0; g < C.ngroups; g++) { C.grp_s.push_back((int)(g * per)); C.grp_e.push_back((int)std::min(C.gates.size(), (size_t)(g + 1) * per)); }
    }
    // every gate filter must be 0 at every point: with several groups the UNUSED factor does
    // it; with one group the selector column is NoopGate's index (its filter is the only
    // non-zero one, and NoopGate has no constraints)
    C.sel_fill = 0xFFFFFFFFULL;
    if (C.ngroups == 1) {
      auto it = std::find(C.gates.begin(), C.gates.end(), std::string("NoopGate"));
      if (it == C.gates.end()) throw std::runtime_error("gen: one selector group needs a NoopGate");
      C.sel_fill = (u64)(it - C.gates.begin());
    }
    Rng rg(C.circuit_seed * 7919 + 17);
    C.gate_const_coeffs.assign(C.num_gate_consts, std::vector<u64>(C.N));
    for (auto& p : C.gate_const_coeffs) for (auto& c : p) c = rg.field();
    for (int i = 0; i < 4; i++) C.circuit_digest.e[i] = rg.field();

    // constants oracle: [selectors (UNUSED) | lookup selectors (0) | gate constants | sigmas]
    C.const_width = C.num_constants + C.num_routed;
    C.const_lde.assign(M * C.const_width, 0);
    std::vector<std::vector<u64>> gc_lde;
    for (auto& p : C.gate_const_coeffs) gc_lde.push_back(lde(p, C.lde_bits));
    u64 eta = gl::subgroup_gen(C.lde_bits);
    std::vector<u64> xs(M); { u64 x = gl::MULT_GEN; for (size_t i = 0; i < M; i++) { xs[i] = x; x = gl::mul(x, eta); } }
    for (size_t idx = 0; idx < M; idx++) {
      size_t nat = gl::rev_bits(C.lde_bits, (uint32_t)idx);
      u64* row = &C.const_lde[idx * C.const_width];
      int c = 0;
      for (int g = 0; g < C.ngroups; g++) row[c++] = C.sel_fill;
      for (int g = 0; g < C.nls; g++) row[c++] = 0;
      for (int g = 0; g < C.num_gate_consts; g++) row[c++] = gc_lde[g][nat];
      for (int j = 0; j < C.num_routed; j++) row[c++] = gl::mul(C.k_is[j], xs[nat]);
    }
  }
  std::vector<Digest> leaves(M);
  for (size_t idx = 0; idx < M; idx++) leaf_digest(&C.const_lde[idx * C.const_width], C.const_width, C.ext & 4, leaves[idx].e);
  C.const_tree.build(std::move(leaves), C.lde_bits, C.cap_height);

  // ---------------------------------------------------------- JSON (Types.hs field names)
  J j;
  auto fri_config = [&](J& o) {
    o.raw("{\"rate_bits\":"); o.i(C.rate_bits); o.raw(",\"cap_height\":"); o.i(C.cap_height);
    o.raw(",\"proof_of_work_bits\":"); o.i(C.pow_bits);
    if (C.ext & 1) o.raw(",\"reduction_strategy\":{\"MinSize\":null}");
    else if (!C.arity_seq.empty()) {
      o.raw(",\"reduction_strategy\":{\"Fixed\":[");
      for (size_t k = 0; k < C.arity_seq.size(); k++) { if (k) o.raw(","); o.i(C.arity_seq[k]); }
      o.raw("]}");
    } else { o.raw(",\"reduction_strategy\":{\"ConstantArityBits\":["); o.i(C.arity_bits); o.raw(","); o.i(C.final_poly_bits); o.raw("]}"); }
    o.raw(",\"num_query_rounds\":"); o.i(C.num_queries); o.raw("}");
  };
  j.raw("{\"config\":{\"num_wires\":"); j.i(C.num_wires); j.raw(",\"num_routed_wires\":"); j.i(C.num_routed);
  j.raw(",\"num_constants\":"); j.i(C.num_gate_consts); j.raw(",\"use_base_arithmetic_gate\":true,\"security_bits\":100");
  j.raw(",\"num_challenges\":"); j.i(C.r); j.raw((C.ext & 2) ? ",\"zero_knowledge\":true" : ",\"zero_knowledge\":false"); j.raw(",\"randomize_unused_wires\":true");
  j.raw(",\"max_quotient_degree_factor\":"); j.i(C.qdf); j.raw(",\"fri_config\":"); fri_config(j); j.raw("}");
  j.raw(",\"fri_params\":{\"config\":"); fri_config(j); j.raw((C.ext & 2) ? ",\"hiding\":true" : ",\"hiding\":false"); j.raw(",\"degree_bits\":"); j.i(C.degree_bits);
  j.raw(",\"reduction_arity_bits\":["); for (size_t k = 0; k < C.arities.size(); k++) { if (k) j.raw(","); j.i(C.arities[k]); } j.raw("]}");
  j.raw(",\"gates\":[");
  for (size_t g = 0; g < C.gates.size(); g++) { if (g) j.raw(","); j.raw("\""); j.raw(C.gates[g].c_str()); j.raw("\""); }
  j.raw("],\"selectors_info\":{\"selector_indices\":[");
  for (size_t g = 0; g < C.sel_idx.size(); g++) { if (g) j.raw(","); j.i(C.sel_idx[g]); }
  j.raw("],\"groups\":[");
  for (int g = 0; g < C.ngroups; g++) {
    if (g) j.raw(",");
    j.raw("{\"start\":"); j.i(C.grp_s[g]); j.raw(",\"end\":"); j.i(C.grp_e[g]); j.raw("}");
  }
  j.raw("]},\"quotient_degree_factor\":"); j.i(C.qdf);
  j.raw(",\"num_gate_constraints\":"); j.i(C.num_gate_constraints);
  j.raw(",\"num_constants\":"); j.i(C.num_constants);
  j.raw(",\"num_public_inputs\":"); j.i(C.num_pis - ((C.ext & 16) ? 1 : 0));   // ext 16: declares one PI fewer than proofs carry
  j.raw(",\"k_is\":"); j.fs(C.k_is.data(), C.k_is.size());
  j.raw(",\"num_partial_products\":"); j.i(C.npp);
  j.raw(",\"num_lookup_polys\":"); j.i(C.nlp);
  j.raw(",\"num_lookup_selectors\":"); j.i(C.nls);
  j.raw(",\"luts\":[");
  for (size_t t = 0; t < C.luts.size(); t++) {
    if (t) j.raw(",");
    j.raw("[");
    for (size_t k = 0; k < C.luts[t].size(); k++) { if (k) j.raw(","); j.raw("["); j.u(C.luts[t][k].first); j.raw(","); j.u(C.luts[t][k].second); j.raw("]"); }
    j.raw("]");
  }
  j.raw("]}");
  C.common_json = std::move(j.s);
  J v;
  v.raw("{\"constants_sigmas_cap\":"); v.cap(C.const_tree.cap()); v.raw(",\"circuit_digest\":"); v.digest(C.circuit_digest); v.raw("}");
  C.vkey_json = std::move(v.s);
}

// ------------------------------------------------------------------ witness (wires + zs/pp oracle)
struct Witness {
  std::vector<std::vector<u64>> wire_coeffs;     // [W][N]
  std::vector<std::vector<u64>> lzs_coeffs;      // [r*nlp][N]
  std::vector<u64> wires_lde;                    // [M][W] bit-reversed rows
  std::vector<u64> zs_lde;                       // [M][r*(1+npp+nlp)]
  std::vector<u64> q_lde;                        // [M][r*qdf] (all zero)
  int zw = 0, qw = 0;
  Tree wires_tree, zs_tree, q_tree;
  std::vector<u64> salt[3];                      // hiding: [M][4] salts of the wires / zs / quotient leaves
  // real mode
  std::vector<u64> pis;                          // public inputs (fixed by the witness: PublicInputGate)
  std::vector<std::vector<u64>> zs_coeffs;       // [r*(1+npp)] Z_j, then the partial products
  std::vector<std::vector<u64>> q_coeffs;        // [r*qdf] quotient chunks
};

// the leaf row of position idx: the oracle's row, then its salts (hiding), as the proof carries it
void leaf_row(const u64* row, int width, const std::vector<u64>& salt, size_t idx, std::vector<u64>& out) {
  out.assign(row, row + width);
  if (!salt.empty()) out.insert(out.end(), salt.begin() + idx * 4, salt.begin() + idx * 4 + 4);
}
void tree_of_rows(const std::vector<u64>& rows, int width, int lde_bits, int cap_height, Tree& t,
                  const std::vector<u64>& salt = {}, bool noop = false) {
  const size_t M = (size_t)1 << lde_bits;
  std::vector<Digest> leaves(M);
  parallel_for(M, [&](size_t idx) {
    std::vector<u64> lr;
    leaf_row(&rows[idx * width], width, salt, idx, lr);
    leaf_digest(lr.data(), lr.size(), noop, leaves[idx].e);
  });
  t.build(std::move(leaves), lde_bits, cap_height);
}
void make_salts(const Circuit& C, Witness* W, u64 seed) {
  if (!(C.ext & 2)) return;
  Rng rg(seed * 31337 + 7);
  const size_t M = (size_t)1 << C.lde_bits;
  for (auto& s : W->salt) { s.resize(M * 4); for (auto& x : s) x = rg.field(); }
}

void batch_inv_base(std::vector<u64>& v) {   // Montgomery's trick over F (no zeros expected)
  const size_t n = v.size();
  std::vector<u64> pre(n);
  u64 acc = 1;
  for (size_t i = 0; i < n; i++) { pre[i] = acc; acc = gl::mul(acc, v[i]); }
  if (acc == 0) throw std::runtime_error("gen: zero in a batch inversion");
  u64 inv = gl::inv(acc);
  for (size_t i = n; i-- > 0;) { u64 t = gl::mul(inv, pre[i]); inv = gl::mul(inv, v[i]); v[i] = t; }
}

// A real witness and the prover's first three rounds (Plonky2's order: wires, then Z/partial
// products after beta/gamma, then the quotient after alpha), reproducing the verifier's
// transcript (Challenge/Verifier.hs:58-92).
Witness* make_witness_real(const Circuit& C, u64 seed) {
  auto* W = new Witness();
  Rng rg(seed * 1000003 + 11);
  make_salts(C, W, seed);
  const int N = C.N, NW = C.num_wires, NR = C.num_routed, NK = C.num_gate_consts, r = C.r, n = C.degree_bits;
  W->pis.resize(C.num_pis);
  for (auto& x : W->pis) x = rg.field();
  u64 pih[4] = {0, 0, 0, 0};
  if (!W->pis.empty()) sponge(W->pis.data(), W->pis.size(), pih);
  // ---- lookups: per block the looked-up table entries (witness-random, the last LU row padded
  // with the table's first entry as plonky2 pads) and each table slot's multiplicity; padded
  // table slots (copies of the head entry, Lookups.hs:107) carry multiplicity 0
  const LkGeom lg(C);
  std::vector<std::vector<uint32_t>> lk_ent(C.lblocks.size());   // [block][nlu * lu_slots] entry index
  std::vector<std::vector<u64>> lk_mult(C.lblocks.size());       // [block][nlut * lut_slots]
  for (size_t b = 0; b < C.lblocks.size(); b++) {
    const auto& B = C.lblocks[b];
    const auto& lut = C.luts[B.table];
    const int nslot = B.nlu * lg.lu_slots;
    const int nreal = std::max(1, nslot - (int)(rg.next() % (u64)(lg.lu_slots / 2 + 1)));
    lk_ent[b].assign(nslot, 0);
    for (int s = 0; s < nreal; s++) lk_ent[b][s] = (uint32_t)(rg.next() % (u64)lut.size());
    lk_mult[b].assign((size_t)B.nlut * lg.lut_slots, 0);
    for (uint32_t e : lk_ent[b]) lk_mult[b][e] = gl::add(lk_mult[b][e], 1);
  }
  // ---- wires: rows in order; a copy constraint presets its (free input) destination
  std::vector<u64> rows((size_t)N * NW);
  std::vector<uint8_t> pre(NW);
  gg::Rng wrg(seed * 7 + 3);
  size_t li = 0;
  std::vector<u64> out;
  for (int i = 0; i < N; i++) {
    std::fill(pre.begin(), pre.end(), 0);
    u64* w = &rows[(size_t)i * NW];
    for (; li < C.links.size() && C.links[li].first / NW == i; li++) {
      const int wi = (int)(C.links[li].first % NW);
      w[wi] = rows[C.links[li].second]; pre[wi] = 1;
    }
    const gg::Gate& g = C.G[C.row_gate[i]];
    const u64* k = &C.row_consts[(size_t)i * NK];
    gg::fill(g, w, pre.data(), NW, k, pih, wrg);
    if (C.row_lk[i] == 1 || C.row_lk[i] == 2) {   // the slots of a lookup row (the rest stay random)
      const int b = C.row_block[i];
      const auto& B = C.lblocks[b];
      const auto& lut = C.luts[B.table];
      if (C.row_lk[i] == 1)
        for (int s = 0; s < lg.lu_slots; s++) {
          const auto& e = lut[lk_ent[b][(size_t)(i - B.lu0) * lg.lu_slots + s]];
          w[2 * s] = e.first; w[2 * s + 1] = e.second;
        }
      else
        for (int s = 0; s < lg.lut_slots; s++) {
          const size_t slot = (size_t)(B.noop - 1 - i) * lg.lut_slots + s;   // entries fill bottom-up
          const auto& e = lut[slot < lut.size() ? slot : 0];
          w[3 * s] = e.first; w[3 * s + 1] = e.second; w[3 * s + 2] = lk_mult[b][slot];
        }
    }
    out.clear();
    gg::eval(g, w, NW, k, NK, pih, out);
    for (size_t t = 0; t < out.size(); t++)
      if (out[t]) throw std::runtime_error("gen: witness row " + std::to_string(i) + " violates constraint " + std::to_string(t) + " of " + g.str);
  }
  W->wire_coeffs.resize(NW);
  parallel_for(NW, [&](size_t c) {
    std::vector<u64> v(N);
    for (int i = 0; i < N; i++) v[i] = rows[(size_t)i * NW + c];
    W->wire_coeffs[c] = interpolate(std::move(v), n);
  });
  W->wires_lde = oracle_rows(W->wire_coeffs, C.lde_bits);
  tree_of_rows(W->wires_lde, NW, C.lde_bits, C.cap_height, W->wires_tree, W->salt[0], C.ext & 4);
  Duplex d;
  for (int i = 0; i < 4; i++) d.absorb(C.circuit_digest.e[i]);
  for (int i = 0; i < 4; i++) d.absorb(pih[i]);
  d.absorb_digests(W->wires_tree.cap());
  std::vector<u64> betas(r), gammas(r), alphas(r);
  for (auto& b : betas) b = d.squeeze();
  for (auto& g : gammas) g = d.squeeze();
  // lookup challenges: betas ++ gammas ++ 2r fresh, in chunks of 4 = (A, B, alpha, delta) per
  // challenge round (Challenge/Verifier.hs:29-40,82-86)
  std::vector<u64> deltas;
  if (C.nlp > 0) {
    deltas = betas; deltas.insert(deltas.end(), gammas.begin(), gammas.end());
    for (int i = 0; i < 2 * r; i++) deltas.push_back(d.squeeze());
  }
  // ---- Z and the partial products per challenge round (Vanishing.hs:97-111)
  const int nch = (NR + C.qdf - 1) / C.qdf;   // chunks; partial products = nch - 1 = npp
  const u64 omega = gl::subgroup_gen(n);
  std::vector<u64> om(N); om[0] = 1; for (int i = 1; i < N; i++) om[i] = gl::mul(om[i - 1], omega);
  const int LZ = r * (1 + C.npp);             // first lookup column: [Z | partial products | lookup zs]
  W->zw = LZ + r * C.nlp;
  std::vector<std::vector<u64>> zcols(W->zw, std::vector<u64>(N));
  // per round and table: evalFinalRE, Horner in delta over the padded table (Lookups.hs:103-109)
  std::vector<std::vector<u64>> final_re(C.nlp > 0 ? r : 0);
  for (int j = 0; j < (int)final_re.size(); j++)
    for (const auto& lut : C.luts) {
      const u64 Bc = deltas[4 * j + 1], de = deltas[4 * j + 3];
      const size_t padded = (lut.size() + lg.lut_slots - 1) / lg.lut_slots * lg.lut_slots;
      u64 acc = 0;
      for (size_t s = 0; s < padded; s++) {
        const auto& e = lut[s < lut.size() ? s : 0];
        acc = gl::add(gl::mul(de, acc), gl::add(e.first, gl::mul(Bc, e.second)));
      }
      final_re[j].push_back(acc);
    }
  // ---- lookup polynomials per round: RE (column 0) and the SLDC running sums (1..nsl), built
  // bottom-up through each block so that every Lookups.hs:94-132 term vanishes on H; rows outside
  // the blocks (and RE on the LU rows) are unconstrained and random
  for (int j = 0; j < (int)final_re.size(); j++) {
    const u64 Ac = deltas[4 * j], Bc = deltas[4 * j + 1], al = deltas[4 * j + 2], de = deltas[4 * j + 3];
    const int L = LZ + j * C.nlp;
    for (int c = L; c < L + C.nlp; c++) for (int i = 0; i < N; i++) zcols[c][i] = rg.field();
    for (const auto& B : C.lblocks) {
      for (int c = L; c < L + C.nlp; c++) zcols[c][B.noop] = 0;
      for (int i = B.noop - 1; i >= B.lu0; i--) {
        const u64* w = &rows[(size_t)i * NW];
        const bool is_lut = i >= B.lut0;
        u64 prev = zcols[L + lg.nsl][i + 1];
        for (int k = 0; k < lg.nsl; k++) {
          u64 sum = 0;
          if (k < lg.npairs()) {
            if (is_lut)
              for (int s = k * lg.lut_deg; s < std::min((k + 1) * lg.lut_deg, lg.lut_slots); s++)
                sum = gl::add(sum, gl::mul(w[3 * s + 2], gl::inv(gl::sub(al, gl::add(w[3 * s], gl::mul(Ac, w[3 * s + 1]))))));
            else
              for (int s = k * lg.lu_deg; s < std::min((k + 1) * lg.lu_deg, lg.lu_slots); s++)
                sum = gl::sub(sum, gl::inv(gl::sub(al, gl::add(w[2 * s], gl::mul(Ac, w[2 * s + 1])))));
          }
          prev = gl::add(prev, sum);
          zcols[L + 1 + k][i] = prev;
        }
        if (is_lut) {
          u64 re = zcols[L][i + 1];
          for (int s = 0; s < lg.lut_slots; s++) re = gl::add(gl::mul(de, re), gl::add(w[3 * s], gl::mul(Bc, w[3 * s + 1])));
          zcols[L][i] = re;
        }
      }
      if (zcols[L + lg.nsl][B.lu0] != 0) throw std::runtime_error("gen: the lookups' log-derivative sum is not zero");
      if (zcols[L][B.lut0] != final_re[j][B.table]) throw std::runtime_error("gen: the table's running evaluation is not evalFinalRE");
    }
  }
  for (int j = 0; j < r; j++) {
    std::vector<u64> num((size_t)N * nch), den((size_t)N * nch);
    parallel_for(N, [&](size_t i) {
      for (int c = 0; c < nch; c++) {
        u64 pn = 1, pd = 1;
        for (int t = c * C.qdf; t < NR && t < (c + 1) * C.qdf; t++) {
          const u64 w = rows[i * NW + t];
          pn = gl::mul(pn, gl::add(gl::add(w, gl::mul(betas[j], gl::mul(C.k_is[t], om[i]))), gammas[j]));
          pd = gl::mul(pd, gl::add(gl::add(w, gl::mul(betas[j], C.const_h[C.ngroups + C.nls + NK + t][i])), gammas[j]));
        }
        num[i * nch + c] = pn; den[i * nch + c] = pd;
      }
    });
    batch_inv_base(den);
    u64 z = 1;
    for (int i = 0; i < N; i++) {
      zcols[j][i] = z;
      u64 cur = z;
      for (int c = 0; c < nch; c++) {
        cur = gl::mul(cur, gl::mul(num[(size_t)i * nch + c], den[(size_t)i * nch + c]));
        if (c < nch - 1) zcols[r + j * C.npp + c][i] = cur;
      }
      z = cur;
    }
    if (z != 1) throw std::runtime_error("gen: the permutation product is not 1 (copy constraints violated)");
  }
  W->zs_coeffs.resize(W->zw);
  parallel_for(W->zw, [&](size_t c) { W->zs_coeffs[c] = interpolate(zcols[c], n); });
  W->lzs_coeffs.assign(W->zs_coeffs.begin() + LZ, W->zs_coeffs.end());
  W->zs_lde = oracle_rows(W->zs_coeffs, C.lde_bits);
  tree_of_rows(W->zs_lde, W->zw, C.lde_bits, C.cap_height, W->zs_tree, W->salt[1], C.ext & 4);
  d.absorb_digests(W->zs_tree.cap());
  for (auto& a : alphas) a = d.squeeze();
  // ---- the quotient: C_i(x) / (x^n - 1) on g<nu>, |<nu>| = 2^q_bits >= (qdf + 1) n
  const int qb = C.q_bits;
  const size_t MQ = (size_t)1 << qb, shift = MQ / (size_t)N;   // omega = nu^shift
  std::vector<std::vector<u64>> wq(NW), zq(W->zw);
  parallel_for(NW, [&](size_t c) { wq[c] = lde(W->wire_coeffs[c], qb); });
  parallel_for(W->zw, [&](size_t c) { zq[c] = lde(W->zs_coeffs[c], qb); });
  const u64 nu = gl::subgroup_gen(qb);
  const int NG = (int)C.G.size(), TG = C.max_constraints;
  std::vector<std::vector<u64>> qv(r, std::vector<u64>(MQ));
  parallel_for(MQ, [&](size_t t) {
    const u64 x = gl::mul(gl::MULT_GEN, gl::pow(nu, t));
    const u64 zh = gl::sub(gl::pow(x, (u64)N), 1);
    const u64 L0 = gl::mul(zh, gl::inv(gl::mul((u64)N % gl::P, gl::sub(x, 1))));
    std::vector<u64> terms;
    for (int j = 0; j < r; j++) terms.push_back(gl::mul(L0, gl::sub(zq[j][t], 1)));
    for (int j = 0; j < r; j++) {
      for (int c = 0; c < nch; c++) {
        const u64 prev = c == 0 ? zq[j][t] : zq[r + j * C.npp + c - 1][t];
        const u64 next = c == nch - 1 ? zq[j][(t + shift) % MQ] : zq[r + j * C.npp + c][t];
        u64 pn = 1, pd = 1;
        for (int s = c * C.qdf; s < NR && s < (c + 1) * C.qdf; s++) {
          pn = gl::mul(pn, gl::add(gl::add(wq[s][t], gl::mul(gl::mul(betas[j], C.k_is[s]), x)), gammas[j]));
          pd = gl::mul(pd, gl::add(gl::add(wq[s][t], gl::mul(betas[j], C.const_q[C.ngroups + C.nls + NK + s][t])), gammas[j]));
        }
        terms.push_back(gl::sub(gl::mul(prev, pn), gl::mul(next, pd)));
      }
    }
    // lookup terms per round (Plonk/Lookups.hs:89-132), in the reference's order
    for (int j = 0; j < (int)final_re.size(); j++) {
      const u64 Ac = deltas[4 * j], Bc = deltas[4 * j + 1], al = deltas[4 * j + 2], de = deltas[4 * j + 3];
      const int L = LZ + j * C.nlp;
      const size_t tn = (t + shift) % MQ;
      auto sel = [&](int s) { return C.const_q[C.ngroups + s][t]; };
      auto W_ = [&](int c) { return wq[c][t]; };
      terms.push_back(gl::mul(sel(3), zq[L + lg.nsl][t]));   // LastLdc: the final SLDC is 0
      terms.push_back(gl::mul(sel(2), zq[L + 1][t]));        // InitSre: SUM starts at 0
      terms.push_back(gl::mul(sel(2), zq[L][t]));            // InitSre: RE starts at 0
      for (size_t k = 0; k < C.luts.size(); k++) terms.push_back(gl::mul(sel(4 + (int)k), gl::sub(zq[L][t], final_re[j][k])));
      u64 cur = zq[L][tn];
      for (int s = 0; s < lg.lut_slots; s++) cur = gl::add(gl::mul(de, cur), gl::add(W_(3 * s), gl::mul(Bc, W_(3 * s + 1))));
      terms.push_back(gl::mul(sel(0), gl::sub(zq[L][t], cur)));
      // sum_i prod_{j != i} of a chunk's factors, and the full product
      auto prods = [&](const std::vector<u64>& f, const std::vector<u64>* mult, u64& full, u64& sum1) {
        full = 1; sum1 = 0;
        for (size_t i = 0; i < f.size(); i++) {
          full = gl::mul(full, f[i]);
          u64 p = mult ? (*mult)[i] : 1;
          for (size_t m = 0; m < f.size(); m++) if (m != i) p = gl::mul(p, f[m]);
          sum1 = gl::add(sum1, p);
        }
      };
      std::vector<u64> f, mu;
      for (int m = 0; m < lg.npairs(); m++) {
        const u64 prev = m == 0 ? zq[L + lg.nsl][tn] : zq[L + m][t], thiz = zq[L + 1 + m][t];
        const u64 dlt = gl::sub(thiz, prev);
        u64 lu_p, lu_s, lut_p, lut_s;
        f.clear();
        for (int s = m * lg.lu_deg; s < std::min((m + 1) * lg.lu_deg, lg.lu_slots); s++) f.push_back(gl::sub(al, gl::add(W_(2 * s), gl::mul(Ac, W_(2 * s + 1)))));
        prods(f, nullptr, lu_p, lu_s);
        f.clear(); mu.clear();
        for (int s = m * lg.lut_deg; s < std::min((m + 1) * lg.lut_deg, lg.lut_slots); s++) {
          f.push_back(gl::sub(al, gl::add(W_(3 * s), gl::mul(Ac, W_(3 * s + 1)))));
          mu.push_back(W_(3 * s + 2));
        }
        prods(f, &mu, lut_p, lut_s);
        terms.push_back(gl::mul(sel(0), gl::sub(gl::mul(lut_p, dlt), lut_s)));   // SUM transition
        terms.push_back(gl::mul(sel(1), gl::add(gl::mul(lu_p, dlt), lu_s)));     // LDC transition
      }
    }
    std::vector<u64> wv(NW), kv(NK), cons, vsum(TG, 0);
    for (int c = 0; c < NW; c++) wv[c] = wq[c][t];
    for (int c = 0; c < NK; c++) kv[c] = C.const_q[C.ngroups + C.nls + c][t];
    for (int k = 0; k < NG; k++) {
      const int g = C.sel_idx[k];
      const u64 S = C.const_q[g][t];
      u64 filt = C.ngroups > 1 ? gl::sub(0xFFFFFFFFULL, S) : 1;   // Gate/Selector.hs:83-89
      for (int m = C.grp_s[g]; m < C.grp_e[g]; m++) if (m != k) filt = gl::mul(filt, gl::sub((u64)m, S));
      cons.clear();
      gg::eval(C.G[k], wv.data(), NW, kv.data(), NK, pih, cons);
      for (size_t q = 0; q < cons.size(); q++) vsum[q] = gl::add(vsum[q], gl::mul(filt, cons[q]));
    }
    terms.insert(terms.end(), vsum.begin(), vsum.end());
    const u64 izh = gl::inv(zh);
    for (int i = 0; i < r; i++) {
      u64 acc = 0;   // sum_s alpha^s term_s (Vanishing.hs:54-56)
      for (size_t s = terms.size(); s-- > 0;) acc = gl::add(terms[s], gl::mul(alphas[i], acc));
      qv[i][t] = gl::mul(acc, izh);
    }
  });
  W->qw = r * C.qdf;
  W->q_coeffs.assign(W->qw, std::vector<u64>(N));
  const u64 ginv = gl::inv(gl::MULT_GEN);
  for (int i = 0; i < r; i++) {
    auto co = interpolate(qv[i], qb);   // coefficients of Q(g y); Q's m-th is co[m] g^-m
    u64 gp = 1;
    for (size_t m = 0; m < MQ; m++, gp = gl::mul(gp, ginv)) {
      const u64 qm = gl::mul(co[m], gp);
      if (m < (size_t)C.qdf * N) W->q_coeffs[i * C.qdf + m / N][m % N] = qm;
      else if (qm != 0) throw std::runtime_error("gen: the constraint polynomial does not vanish on H (quotient degree too high)");
    }
  }
  W->q_lde = oracle_rows(W->q_coeffs, C.lde_bits);
  tree_of_rows(W->q_lde, W->qw, C.lde_bits, C.cap_height, W->q_tree, W->salt[2], C.ext & 4);
  return W;
}

Witness* make_witness(const Circuit& C, u64 seed) {
  auto* W = new Witness();
  Rng rg(seed * 1000003 + 11);
  make_salts(C, W, seed);
  size_t M = (size_t)1 << C.lde_bits;
  W->wire_coeffs.assign(C.num_wires, std::vector<u64>(C.N));
  for (auto& p : W->wire_coeffs) for (auto& c : p) c = rg.field();
  int nl = C.r * C.nlp;
  W->lzs_coeffs.assign(nl, std::vector<u64>(C.N));
  for (auto& p : W->lzs_coeffs) for (auto& c : p) c = rg.field();
  W->wires_lde.assign(M * C.num_wires, 0);
  for (int w = 0; w < C.num_wires; w++) {
    auto l = lde(W->wire_coeffs[w], C.lde_bits);
    for (size_t idx = 0; idx < M; idx++) W->wires_lde[idx * C.num_wires + w] = l[gl::rev_bits(C.lde_bits, (uint32_t)idx)];
  }
  // zs/pp oracle columns: [zs (r) | partial products (r*npp) | lookup zs (r*nlp)] — Z == pp == 1
  W->zw = C.r * (1 + C.npp + C.nlp);
  W->zs_lde.assign(M * W->zw, 1);
  for (int k = 0; k < nl; k++) {
    auto l = lde(W->lzs_coeffs[k], C.lde_bits);
    int col = C.r * (1 + C.npp) + k;
    for (size_t idx = 0; idx < M; idx++) W->zs_lde[idx * W->zw + col] = l[gl::rev_bits(C.lde_bits, (uint32_t)idx)];
  }
  W->qw = C.r * C.qdf;
  W->q_lde.assign(M * W->qw, 0);
  tree_of_rows(W->wires_lde, C.num_wires, C.lde_bits, C.cap_height, W->wires_tree, W->salt[0], C.ext & 4);
  tree_of_rows(W->zs_lde, W->zw, C.lde_bits, C.cap_height, W->zs_tree, W->salt[1], C.ext & 4);
  tree_of_rows(W->q_lde, W->qw, C.lde_bits, C.cap_height, W->q_tree, W->salt[2], C.ext & 4);
  return W;
}

// ------------------------------------------------------------------ proof
// flags (malicious-prover modes for reject-path tests):
//   1: corrupt the first FRI layer before committing   -> step-0 evaluation mismatch
//   2: corrupt the last FRI layer (final poly truncated) -> final polynomial mismatch
//   4: corrupt a quotient opening                        -> Plonk identity fails
//   8: final polynomial with two trailing zero coefficients (a valid proof of another length)
std::string make_proof(const Circuit& C, const Witness& W, u64 pi_seed, unsigned flags = 0) {
  Rng rg(pi_seed * 104729 + 5);
  const size_t M = (size_t)1 << C.lde_bits;
  const int r = C.r;
  std::vector<u64> pis(C.num_pis);
  if (C.real) pis = W.pis;
  else for (auto& x : pis) x = rg.field();
  u64 pih[4]; sponge(pis.data(), pis.size(), pih);
  if (pis.empty()) memset(pih, 0, sizeof pih);

  Duplex d;
  for (int i = 0; i < 4; i++) d.absorb(C.circuit_digest.e[i]);
  for (int i = 0; i < 4; i++) d.absorb(pih[i]);
  d.absorb_digests(W.wires_tree.cap());
  std::vector<u64> betas(r), gammas(r);
  for (auto& b : betas) b = d.squeeze();
  for (auto& g : gammas) g = d.squeeze();
  if (C.nlp > 0) for (int i = 0; i < 2 * r; i++) (void)d.squeeze();
  d.absorb_digests(W.zs_tree.cap());
  for (int i = 0; i < r; i++) (void)d.squeeze();   // alphas
  d.absorb_digests(W.q_tree.cap());
  E zeta = d.squeeze_e();
  u64 omega = gl::subgroup_gen(C.degree_bits);
  E zeta_w = gl::escale(omega, zeta);

  // openings at zeta (OpeningSet order, Types.hs:265-279)
  std::vector<E> o_const, o_sig, o_wires, o_zs, o_zs_next, o_pp, o_quot, o_lzs, o_lzs_next;
  if (C.real) {
    for (int c = 0; c < C.num_constants; c++) o_const.push_back(eval_at(C.const_coeffs[c], zeta));
    for (int j = 0; j < C.num_routed; j++) o_sig.push_back(eval_at(C.const_coeffs[C.num_constants + j], zeta));
    for (int w = 0; w < C.num_wires; w++) o_wires.push_back(eval_at(W.wire_coeffs[w], zeta));
    for (int i = 0; i < r; i++) { o_zs.push_back(eval_at(W.zs_coeffs[i], zeta)); o_zs_next.push_back(eval_at(W.zs_coeffs[i], zeta_w)); }
    for (int i = 0; i < r * C.npp; i++) o_pp.push_back(eval_at(W.zs_coeffs[r + i], zeta));
    for (int i = 0; i < r * C.qdf; i++) o_quot.push_back(eval_at(W.q_coeffs[i], zeta));
    if (flags & 4) o_quot[0] = gl::eadd(o_quot[0], gl::eb(12345));
  } else {
    for (int g = 0; g < C.ngroups; g++) o_const.push_back(gl::eb(C.sel_fill));
    for (int g = 0; g < C.nls; g++) o_const.push_back(gl::e0());
    for (int g = 0; g < C.num_gate_consts; g++) o_const.push_back(eval_at(C.gate_const_coeffs[g], zeta));
    for (int j = 0; j < C.num_routed; j++) o_sig.push_back(gl::escale(C.k_is[j], zeta));
    for (int w = 0; w < C.num_wires; w++) o_wires.push_back(eval_at(W.wire_coeffs[w], zeta));
    for (int i = 0; i < r; i++) { o_zs.push_back(gl::eb(1)); o_zs_next.push_back(gl::eb(1)); }
    for (int i = 0; i < r * C.npp; i++) o_pp.push_back(gl::eb(1));
    for (int i = 0; i < r * C.qdf; i++) o_quot.push_back(gl::e0());
    if (flags & 4) o_quot[0] = gl::eb(12345);
  }
  for (int k = 0; k < r * C.nlp; k++) { o_lzs.push_back(eval_at(W.lzs_coeffs[k], zeta)); o_lzs_next.push_back(eval_at(W.lzs_coeffs[k], zeta_w)); }
  std::vector<E> b1, b2;
  for (auto* v : {&o_const, &o_sig, &o_wires, &o_zs, &o_pp, &o_quot, &o_lzs}) b1.insert(b1.end(), v->begin(), v->end());
  for (auto* v : {&o_zs_next, &o_lzs_next}) b2.insert(b2.end(), v->begin(), v->end());
  d.absorb_e(b1); d.absorb_e(b2);
  E alpha = d.squeeze_e();

  // combined codeword at every LDE position (bit-reversed order), Plonk/FRI.hs:151-207
  auto reduce = [&](const std::vector<E>& xs) { E acc = gl::e0(); for (size_t i = xs.size(); i-- > 0;) acc = gl::eadd(xs[i], gl::emul(alpha, acc)); return acc; };
  E y0 = reduce(b1), y1 = reduce(b2);
  int npp_all = (C.num_routed + C.qdf - 1) / C.qdf;   // zs + pps per challenge
  int len2 = r + r * C.nlp;
  E alpha_len2 = gl::epow(alpha, (u64)len2);
  u64 eta = gl::subgroup_gen(C.lde_bits);
  std::vector<E> den0(M), den1(M);
  std::vector<u64> px(M);
  for (size_t idx = 0; idx < M; idx++) {
    px[idx] = gl::mul(gl::MULT_GEN, gl::pow(eta, gl::rev_bits(C.lde_bits, (uint32_t)idx)));
    den0[idx] = gl::esub(gl::eb(px[idx]), zeta);
    den1[idx] = gl::esub(gl::eb(px[idx]), zeta_w);
  }
  batch_inv(den0); batch_inv(den1);
  std::vector<E> cw(M);
  std::vector<u64> row;
  for (size_t idx = 0; idx < M; idx++) {
    // firstBatch = consts|sigmas | wires | pp-part (r*npp_all) | quotient | lookup part
    const u64* rc = &C.const_lde[idx * C.const_width];
    const u64* rw = &W.wires_lde[idx * C.num_wires];
    const u64* rz = &W.zs_lde[idx * W.zw];
    const u64* rq = &W.q_lde[idx * W.qw];
    row.clear();
    row.insert(row.end(), rc, rc + C.const_width);
    row.insert(row.end(), rw, rw + C.num_wires);
    row.insert(row.end(), rz, rz + r * npp_all);
    row.insert(row.end(), rq, rq + W.qw);
    row.insert(row.end(), rz + r * npp_all, rz + W.zw);
    E g0 = gl::e0();
    for (size_t i = row.size(); i-- > 0;) g0 = gl::eadd(gl::eb(row[i]), gl::emul(alpha, g0));
    E g1 = gl::e0();
    std::vector<u64> sb(rz, rz + r); sb.insert(sb.end(), rz + r * npp_all, rz + W.zw);
    for (size_t i = sb.size(); i-- > 0;) g1 = gl::eadd(gl::eb(sb[i]), gl::emul(alpha, g1));
    E one = gl::emul(gl::esub(g0, y0), den0[idx]);
    E two = gl::emul(gl::esub(g1, y1), den1[idx]);
    cw[idx] = gl::eadd(gl::emul(alpha_len2, one), two);
  }

  // commit phase (folding), Plonk/FRI.hs:233-323 conventions
  std::vector<Tree> step_trees;
  std::vector<std::vector<E>> layers;   // values of each layer (bit-reversed order)
  std::vector<E> betas_fri;
  if (flags & 1) for (auto& x : cw) x = gl::eadd(x, gl::eb(1));   // not the committed polynomial's values
  layers.push_back(cw);
  u64 shift = gl::MULT_GEN; int logn = C.lde_bits;
  for (size_t s = 0; s < C.arities.size(); s++) {
    int ab = C.arities[s], ar = 1 << ab;
    const auto& v = layers.back();
    size_t nl = v.size() / ar;
    std::vector<Digest> leaves(nl);
    std::vector<u64> flat(2 * ar);
    for (size_t jj = 0; jj < nl; jj++) {
      for (int k = 0; k < ar; k++) { flat[2 * k] = v[jj * ar + k].a; flat[2 * k + 1] = v[jj * ar + k].b; }
      leaf_digest(flat.data(), flat.size(), C.ext & 4, leaves[jj].e);
    }
    Tree t; t.build(std::move(leaves), logn - ab, C.cap_height);
    d.absorb_digests(t.cap());
    E beta = d.squeeze_e();
    betas_fri.push_back(beta);
    // fold: new[j] = interpolant through coset j at beta
    u64 eta_b = gl::subgroup_gen(logn), om = gl::subgroup_gen(ab);
    u64 om_inv = gl::inv(om), inv_ar = gl::inv((u64)ar);
    std::vector<E> nv(nl);
    std::vector<E> vals(ar);
    for (size_t jj = 0; jj < nl; jj++) {
      u64 ofs = gl::mul(shift, gl::pow(eta_b, gl::rev_bits(logn, (uint32_t)(jj << ab))));
      for (int k = 0; k < ar; k++) vals[gl::rev_bits(ab, (uint32_t)k)] = v[jj * ar + k];
      // coefficients of P(ofs*Y): c_k = (1/ar) sum_j vals_j om^{-jk}
      std::vector<E> c(vals);
      efft(c, ab, om_inv);
      // P(beta) = sum_k c_k (beta/ofs)^k / ar
      E bo = gl::escale(gl::inv(ofs), beta);
      E acc = gl::e0();
      for (int k = ar; k-- > 0;) acc = gl::eadd(gl::emul(acc, bo), c[k]);
      nv[jj] = gl::escale(inv_ar, acc);
    }
    step_trees.push_back(std::move(t));
    layers.push_back(std::move(nv));
    shift = gl::pow(shift, (u64)ar);
    logn -= ab;
  }
  // final polynomial: values on shift*<eta_f> (bit-reversed) -> coefficients
  if (flags & 2) { Rng cr(pi_seed + 77); for (auto& x : layers.back()) x = gl::eadd(x, gl::eb(cr.field())); }
  std::vector<E> fin = layers.back();
  size_t nf = fin.size();
  std::vector<E> nat(nf);
  for (size_t i = 0; i < nf; i++) nat[gl::rev_bits(logn, (uint32_t)i)] = fin[i];
  efft(nat, logn, gl::inv(gl::subgroup_gen(logn)));
  u64 inv_nf = gl::inv((u64)nf), sinv = gl::inv(shift), sp = 1;
  int sum_a = 0; for (int a : C.arities) sum_a += a;
  size_t final_len = (size_t)1 << (C.degree_bits - sum_a);
  std::vector<E> final_poly(final_len);
  for (size_t k = 0; k < nf; k++) {
    E ck = gl::escale(gl::mul(inv_nf, sp), nat[k]);
    sp = gl::mul(sp, sinv);
    if (k < final_len) final_poly[k] = ck;
    else if (!(ck.a == 0 && ck.b == 0) && !(flags & 7)) throw std::runtime_error("generator: final polynomial has too high degree");
  }
  // flags 8: two trailing zero coefficients (the same polynomial at another length: the reference
  // absorbs and evaluates whatever length it is given, Challenge/FRI.hs:83, Plonk/FRI.hs:325-327)
  if (flags & 8) { final_poly.push_back(gl::e0()); final_poly.push_back(gl::e0()); }
  d.absorb_e(final_poly);
  // proof of work: find w s.t. the top pow_bits of the squeezed response are zero
  u64 mask = C.pow_bits ? (((1ULL << C.pow_bits) - 1) << (64 - C.pow_bits)) : 0;
  u64 witness = 0;
  for (u64 w = rg.next() & 0xFFFFFFFFULL;; w++) {
    Duplex t = d; t.absorb(w);
    u64 resp = t.squeeze();
    if ((resp & mask) == 0) { witness = w; break; }
  }
  d.absorb(witness);
  (void)d.squeeze();
  std::vector<size_t> qidx(C.num_queries);
  for (auto& q : qidx) q = (size_t)(d.squeeze() & (M - 1));

  // ---------------------------------------------------------------- JSON
  J j;
  j.raw("{\"proof\":{\"wires_cap\":"); j.cap(W.wires_tree.cap());
  j.raw(",\"plonk_zs_partial_products_cap\":"); j.cap(W.zs_tree.cap());
  j.raw(",\"quotient_polys_cap\":"); j.cap(W.q_tree.cap());
  j.raw(",\"openings\":{\"constants\":"); j.es(o_const); j.raw(",\"plonk_sigmas\":"); j.es(o_sig);
  j.raw(",\"wires\":"); j.es(o_wires); j.raw(",\"plonk_zs\":"); j.es(o_zs); j.raw(",\"plonk_zs_next\":"); j.es(o_zs_next);
  j.raw(",\"partial_products\":"); j.es(o_pp); j.raw(",\"quotient_polys\":"); j.es(o_quot);
  j.raw(",\"lookup_zs\":"); j.es(o_lzs); j.raw(",\"lookup_zs_next\":"); j.es(o_lzs_next); j.raw("}");
  j.raw(",\"opening_proof\":{\"commit_phase_merkle_caps\":[");
  for (size_t s = 0; s < step_trees.size(); s++) { if (s) j.raw(","); j.cap(step_trees[s].cap()); }
  j.raw("],\"query_round_proofs\":[");
  for (int q = 0; q < C.num_queries; q++) {
    if (q) j.raw(",");
    size_t idx = qidx[q];
    j.raw("{\"initial_trees_proof\":{\"evals_proofs\":[");
    std::vector<u64> lr;
    auto emit = [&](const u64* rowp, int width, const Tree& t, const std::vector<u64>& salt, bool comma) {
      if (comma) j.raw(",");
      leaf_row(rowp, width, salt, idx, lr);
      j.raw("["); j.fs(lr.data(), lr.size()); j.raw(",{\"siblings\":"); j.cap(t.path(idx)); j.raw("}]");
    };
    emit(&C.const_lde[idx * C.const_width], C.const_width, C.const_tree, {}, false);
    emit(&W.wires_lde[idx * C.num_wires], C.num_wires, W.wires_tree, W.salt[0], true);
    emit(&W.zs_lde[idx * W.zw], W.zw, W.zs_tree, W.salt[1], true);
    emit(&W.q_lde[idx * W.qw], W.qw, W.q_tree, W.salt[2], true);
    j.raw("]},\"steps\":[");
    size_t qi = idx;
    for (size_t s = 0; s < step_trees.size(); s++) {
      int ab = C.arities[s], ar = 1 << ab;
      size_t leaf = qi >> ab;
      std::vector<E> ev(layers[s].begin() + leaf * ar, layers[s].begin() + (leaf + 1) * ar);
      if (s) j.raw(",");
      j.raw("{\"evals\":"); j.es(ev); j.raw(",\"merkle_proof\":{\"siblings\":"); j.cap(step_trees[s].path(leaf)); j.raw("}}");
      qi = leaf;
    }
    j.raw("]}");
  }
  j.raw("],\"final_poly\":{\"coeffs\":"); j.es(final_poly); j.raw("},\"pow_witness\":"); j.u(witness); j.raw("}}");
  j.raw(",\"public_inputs\":"); j.fs(pis.data(), pis.size()); j.raw("}");
  return std::move(j.s);
}

thread_local std::string g_err;

char* dupstr(const std::string& s) { char* p = (char*)malloc(s.size() + 1); memcpy(p, s.data(), s.size() + 1); return p; }

}  // namespace

extern "C" {

// spec: degree_bits, num_public_inputs, lookups (0 none, 1/2/3 table sets, see below), circuit_seed
// mode 0: the degenerate circuit (gate filters 0 at every point), `ngroups` selector groups
//         (1: the column is NoopGate's index); mode 1: a real circuit over the recursion gate
//         set; mode 2: a real circuit over a small gate set (Noop, Constant, PublicInput,
//         Arithmetic) that fits one selector group.  Real modes choose their own groups.
// ext / arities (narities > 0): the opt-in plonky2 conventions of the Circuit fields above
void* p2v_gen_circuit_new3(int degree_bits, int num_pis, int lookups, uint64_t circuit_seed, int num_queries, int pow_bits,
                           int ngroups, int mode, unsigned ext, const int* arities, int narities) {
  try {
    auto* C = new Circuit();
    C->degree_bits = degree_bits; C->num_pis = num_pis; C->circuit_seed = circuit_seed;
    C->ext = ext;
    if ((ext & 1) && narities <= 0) throw std::runtime_error("gen: the MinSize form needs the arity list");
    for (int k = 0; k < narities; k++) C->arity_seq.push_back(arities[k]);
    if (ngroups > 0) C->ngroups = ngroups;
    C->real = mode != 0; C->gate_set = mode == 2 ? 1 : 0;
    if (num_queries > 0) C->num_queries = num_queries;
    if (pow_bits >= 0) C->pow_bits = pow_bits;
    if (lookups >= 4) {
      // small tables that fit a 64-row circuit: 4 one table of 40 u6 entries; 5 that table and
      // a 30-entry table with field-sized outputs; 6 the 2^16-entry range table alone
      C->nlp = 7;
      std::vector<std::pair<u64, u64>> a, b, c;
      for (u64 i = 0; i < 40; i++) a.push_back({i, (i * 37 + 11) & 63});
      for (u64 i = 0; i < 30; i++) b.push_back({1000 + 3 * i, (i * 0x9E3779B97F4A7C15ULL + 5) % 0xFFFFFFFF00000001ULL});
      for (u64 i = 0; i < 65536; i++) c.push_back({i, 0});
      if (lookups == 6) C->luts.push_back(c);
      else { C->luts.push_back(a); if (lookups == 5) C->luts.push_back(b); }
    } else if (lookups) {
      C->nlp = 7;
      std::vector<std::pair<u64, u64>> t8, t16;
      for (u64 i = 0; i < 256; i++) t8.push_back({i, (i * i + 7) & 255});
      // 1: 1000-entry table; 2: 2^16-entry range table (BASELINE C3); 3: 300 entries with
      // field-sized outputs (exercises the verifier's generic evalFinalRE path)
      int big = lookups == 2 ? 65536 : lookups == 3 ? 300 : 1000;
      for (u64 i = 0; i < (u64)big; i++) t16.push_back({i, lookups == 3 ? (i * 0x9E3779B97F4A7C15ULL) % 0xFFFFFFFF00000001ULL : 0});
      C->luts.push_back(t8); C->luts.push_back(t16);
    }
    build_circuit(*C);
    return C;
  } catch (std::exception& e) { g_err = e.what(); return nullptr; }
}
void* p2v_gen_circuit_new2(int degree_bits, int num_pis, int lookups, uint64_t circuit_seed, int num_queries, int pow_bits,
                           int ngroups, int mode) {
  return p2v_gen_circuit_new3(degree_bits, num_pis, lookups, circuit_seed, num_queries, pow_bits, ngroups, mode, 0, nullptr, 0);
}
void* p2v_gen_circuit_new(int degree_bits, int num_pis, int lookups, uint64_t circuit_seed, int num_queries, int pow_bits) {
  return p2v_gen_circuit_new2(degree_bits, num_pis, lookups, circuit_seed, num_queries, pow_bits, 0, 0);
}
void p2v_gen_circuit_free(void* c) { delete (Circuit*)c; }
// A witness row of gate `gate` of a real-mode circuit (plonky2 semantics, gates.hpp fill()) with
// random free inputs and row constants: wires (num_wires), consts (num_gate_consts), pih (4).
// Returns the number of constraints of the gate's program (all zero on this row), < 0 on error.
int p2v_gen_gate_row(void* c, int gate, uint64_t seed, uint64_t* wires, uint64_t* consts, uint64_t* pih) {
  try {
    const Circuit& C = *(Circuit*)c;
    if (!C.real || gate < 0 || gate >= (int)C.G.size()) { g_err = "p2v_gen_gate_row: not a real-mode gate"; return -1; }
    gg::Rng rg(seed);
    const int NW = C.num_wires, NK = C.num_gate_consts;
    for (int i = 0; i < 4; i++) pih[i] = rg.field();
    for (int i = 0; i < NK; i++) consts[i] = i < gg::num_row_constants(C.G[gate]) ? rg.field() : 0;
    std::vector<uint8_t> pre(NW, 0);
    gg::fill(C.G[gate], wires, pre.data(), NW, consts, pih, rg);
    std::vector<u64> out;
    gg::eval(C.G[gate], wires, NW, consts, NK, pih, out);
    for (u64 x : out) if (x) { g_err = "p2v_gen_gate_row: row does not satisfy the gate"; return -2; }
    return (int)out.size();
  } catch (std::exception& e) { g_err = e.what(); return -3; }
}
int p2v_gen_num_gates(void* c) { return (int)((Circuit*)c)->gates.size(); }
const char* p2v_gen_common_json(void* c) { return ((Circuit*)c)->common_json.c_str(); }
const char* p2v_gen_vkey_json(void* c) { return ((Circuit*)c)->vkey_json.c_str(); }
void* p2v_gen_witness_new(void* c, uint64_t seed) {
  try {
    const Circuit& C = *(Circuit*)c;
    return C.real ? make_witness_real(C, seed) : make_witness(C, seed);
  } catch (std::exception& e) { g_err = e.what(); return nullptr; }
}
void p2v_gen_witness_free(void* w) { delete (Witness*)w; }
char* p2v_gen_proof_json(void* c, void* w, uint64_t pi_seed) {
  try { return dupstr(make_proof(*(Circuit*)c, *(Witness*)w, pi_seed)); } catch (std::exception& e) { g_err = e.what(); return nullptr; }
}
char* p2v_gen_proof_json_flags(void* c, void* w, uint64_t pi_seed, unsigned flags) {
  try { return dupstr(make_proof(*(Circuit*)c, *(Witness*)w, pi_seed, flags)); } catch (std::exception& e) { g_err = e.what(); return nullptr; }
}
void p2v_gen_free_str(char* s) { free(s); }
const char* p2v_gen_last_error(void) { return g_err.c_str(); }

}  // extern "C"
