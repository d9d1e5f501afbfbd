// circuit.cpp — VerifierCircuitData decode/validation, packed layout, proof packing.
#include "circuit.hpp"
#include "gl.h"
#include "../../include/p2v.h"
#include <algorithm>
#include <cstring>

namespace p2v {

// ------------------------------------------------------------------ gate strings
// A restatement of the Parsec grammar of Gate/Parser.hs:112-240.  Every alternative is
// wrapped in `try` there, so each pattern is matched from the start of the string; the
// `withEOF` ones must consume everything, the others ignore trailing text.
namespace {
struct Cur {
  const char* p;
  void spaces() { while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r' || *p == '\f' || *p == '\v') p++; }
  bool lit(const char* s) { size_t n = strlen(s); if (strncmp(p, s, n)) return false; p += n; return true; }
  bool ch(char c) { if (*p != c) return false; p++; return true; }
  bool integer(int64_t* iv, uint64_t* fv) {
    if (*p < '0' || *p > '9') return false;
    uint64_t w = 0; unsigned __int128 m = 0;
    while (*p >= '0' && *p <= '9') { unsigned d = (unsigned)(*p - '0'); w = w * 10 + d; m = (m * 10 + d) % GL_P; p++; }
    if (iv) *iv = (int64_t)w;
    if (fv) *fv = (uint64_t)m;
    return true;
  }
  bool comma() { if (!ch(',')) return false; spaces(); return true; }
  bool kv_int(const char* key, int64_t* v) { return lit(key) && (spaces(), ch(':')) && (spaces(), integer(v, nullptr)) && (spaces(), true); }
  bool list(std::vector<uint64_t>* out) {
    if (!ch('[')) return false;
    spaces();
    int64_t iv; uint64_t fv;
    if (integer(&iv, &fv)) {
      if (out) out->push_back(fv);
      while (*p == ',') {
        comma();
        if (!integer(&iv, &fv)) return false;
        if (out) out->push_back(fv);
      }
    }
    if (!ch(']')) return false;
    spaces();
    return true;
  }
  bool kv_list(const char* key, std::vector<uint64_t>* out) { return lit(key) && (spaces(), ch(':')) && (spaces(), list(out)) && (spaces(), true); }
  bool open(const char* name) { return lit(name) && (spaces(), ch('{')) && (spaces(), true); }
  bool close() { spaces(); if (!ch('}')) return false; spaces(); return true; }
  bool eof() const { return *p == 0; }
};
const char* kPhantom = "_phantom: PhantomData<plonky2_field::goldilocks_field::GoldilocksField>";
}  // namespace

GateDesc parse_gate_string(const std::string& s) {
  GateDesc g; g.text = s;
  const char* str = s.c_str();
  int64_t a, b, c;
  { Cur u{str}; if (u.open("ArithmeticGate") && u.kv_int("num_ops", &a) && u.close() && u.eof()) { g.kind = G_ARITH; g.p0 = a; return g; } }
  { Cur u{str}; if (u.open("ArithmeticExtensionGate") && u.kv_int("num_ops", &a) && u.close() && u.eof()) { g.kind = G_ARITH_EXT; g.p0 = a; return g; } }
  { Cur u{str}; if (u.open("BaseSumGate") && u.kv_int("num_limbs", &a) && u.close() && u.ch('+')) { u.spaces(); if (u.kv_int("Base", &b) && u.eof()) { g.kind = G_BASESUM; g.p0 = a; g.p1 = b; return g; } } }
  { Cur u{str}; std::vector<uint64_t> w;
    if (u.open("CosetInterpolationGate") && u.kv_int("subgroup_bits", &a) && u.comma() && u.kv_int("degree", &b) && u.comma() &&
        u.kv_list("barycentric_weights", &w) && u.comma() && u.lit(kPhantom)) {
      u.spaces();
      if (u.close() && u.lit("<D=2>") && u.eof()) { g.kind = G_COSET; g.p0 = a; g.p1 = b; g.weights = w; return g; }
    } }
  { Cur u{str}; if (u.open("ConstantGate") && u.kv_int("num_consts", &a) && u.close()) { g.kind = G_CONST; g.p0 = a; return g; } }
  { Cur u{str}; if (u.open("ExponentiationGate") && u.kv_int("num_power_bits", &a) && u.close()) { g.kind = G_EXP; g.p0 = a; return g; } }
  { Cur u{str}; if (u.open("LookupGate") && u.kv_int("num_slots", &a) && u.comma() && u.kv_list("lut_hash", nullptr) && u.close()) { g.kind = G_LOOKUP; g.p0 = a; return g; } }
  { Cur u{str}; if (u.open("LookupTableGate") && u.kv_int("num_slots", &a) && u.comma() && u.kv_list("lut_hash", nullptr) && u.comma() &&
                    u.kv_int("last_lut_row", &c) && u.close()) { g.kind = G_LOOKUPTABLE; g.p0 = a; g.p2 = c; return g; } }
  { Cur u{str}; if (u.open("MulExtensionGate") && u.kv_int("num_ops", &a) && u.close()) { g.kind = G_MULEXT; g.p0 = a; return g; } }
  { Cur u{str}; if (u.lit("NoopGate")) { g.kind = G_NOOP; return g; } }
  { Cur u{str}; if (u.lit("PublicInputGate")) { g.kind = G_PI; return g; } }
  { Cur u{str}; if (u.lit("PoseidonGate(PhantomData<plonky2_field::goldilocks_field::GoldilocksField>)<WIDTH=") && u.integer(&a, nullptr) && u.ch('>') && u.eof()) { g.kind = G_POSEIDON; g.p0 = a; return g; } }
  { Cur u{str}; if (u.lit("PoseidonMdsGate(PhantomData<plonky2_field::goldilocks_field::GoldilocksField>)<WIDTH=") && u.integer(&a, nullptr) && u.ch('>') && u.eof()) { g.kind = G_POSEIDON_MDS; g.p0 = a; return g; } }
  { Cur u{str}; if (u.open("RandomAccessGate") && u.kv_int("bits", &a) && u.comma() && u.kv_int("num_copies", &b) && u.comma() &&
                    u.kv_int("num_extra_constants", &c) && u.comma() && u.lit(kPhantom)) {
      u.spaces();
      if (u.close() && u.lit("<D=2>")) { g.kind = G_RANDACC; g.p0 = a; g.p1 = b; g.p2 = c; return g; }
    } }
  { Cur u{str}; if (u.open("ReducingGate") && u.kv_int("num_coeffs", &a)) { u.lit("<D=2>"); if (u.close()) { g.kind = G_REDUCING; g.p0 = a; return g; } } }
  { Cur u{str}; if (u.open("ReducingExtensionGate") && u.kv_int("num_coeffs", &a)) { u.lit("<D=2>"); if (u.close()) { g.kind = G_REDUCING_EXT; g.p0 = a; return g; } } }
  g.kind = G_UNKNOWN;
  return g;
}

// highest wire / constant index a gate program reads (Gate/Constraints.hs, Gate/Custom/*):
// the reference raises an Array index `error` when it exceeds the opening vectors.
static void gate_footprint(const GateDesc& g, int64_t& max_wire, int64_t& max_const) {
  max_wire = -1; max_const = -1;
  switch (g.kind) {
    case G_ARITH: if (g.p0 > 0) { max_wire = 4 * g.p0 - 1; max_const = 1; } break;
    case G_ARITH_EXT: if (g.p0 > 0) { max_wire = 8 * g.p0 - 1; max_const = 1; } break;
    case G_BASESUM: max_wire = std::max<int64_t>(g.p0, 1); break;
    case G_COSET: {
      int64_t n = (int64_t)1 << g.p0, d = g.p1;
      int64_t nint = d - 1 != 0 ? (n - 2) / (d - 1) : 0;
      max_wire = 1 + 2 * (n + 2) + 4 * nint + 1;
      break; }
    case G_CONST: if (g.p0 > 0) { max_wire = g.p0 - 1; max_const = g.p0 - 1; } break;
    case G_EXP: max_wire = 2 * g.p0 + 1; break;
    case G_MULEXT: if (g.p0 > 0) { max_wire = 6 * g.p0 - 1; max_const = 0; } break;
    case G_PI: max_wire = 3; break;
    case G_POSEIDON: max_wire = 29 + 36 + 22 + 48 - 1; break;
    case G_POSEIDON_MDS: max_wire = 2 * 23 + 1; break;
    case G_RANDACC: {
      int64_t width = 2 + ((int64_t)1 << g.p0);
      int64_t bstart = width * g.p1 + g.p2;
      max_wire = std::max<int64_t>(bstart + g.p1 * g.p0 - 1, g.p1 * width + g.p2 - 1);
      if (g.p2 > 0) max_const = g.p2 - 1;
      break; }
    case G_REDUCING: { int64_t n = g.p0; max_wire = std::max<int64_t>({5, n + 5, n >= 2 ? 3 * n + 3 : 5}); break; }
    case G_REDUCING_EXT: { int64_t n = g.p0; max_wire = std::max<int64_t>({5, 2 * n + 5, n >= 2 ? 4 * n + 3 : 5}); break; }
    default: break;
  }
}

static void digest_of(const JVal& d, uint64_t* out) {   // Hash/Digest.hs:40-44
  const auto& e = d.at("elements").arr();
  if (e.size() != 4) throw ParseError("digest must have 4 elements");
  for (int i = 0; i < 4; i++) out[i] = j_field(e[i]);
}

// expandReductionStrategy starts from degree_bits (Plonk/FRI.hs:337-354, :378)
enum { STRAT_FIXED = 0, STRAT_CONSTANT_ARITY_BITS = 1, STRAT_MIN_SIZE = 2 };   // FriReductionStrategy, Types.hs:128-131
static void expand_strategy(Circuit& C, int tag, const std::vector<int64_t>& a) {
  // bounds first: the step list is expanded before finalize_circuit validates the
  // sizes, so an absurd degree_bits / final_poly_bits must not drive the expansion loop
  constexpr int kMaxSteps = 64;
  if (C.degree_bits < 0 || C.degree_bits > 64) throw CircuitError("unsupported FRI sizes");
  for (int64_t x : a) if (x < -64 || x > 64) throw CircuitError("reduction strategy argument out of range");
  if (tag == STRAT_CONSTANT_ARITY_BITS) {
    if (a.size() != 2) throw ParseError("ConstantArityBits: expecting [arity_bits, final_poly_bits]");
    const int ab = (int)a[0], f = (int)a[1];
    if (ab <= 0 && C.degree_bits > f) throw CircuitError("reduction strategy does not terminate (arity_bits <= 0)");
    for (int logn = C.degree_bits; logn > f; logn -= ab) {
      if ((int)C.arities.size() == kMaxSteps) throw CircuitError("reduction strategy: too many FRI steps");
      C.arities.push_back(ab);
    }
  } else if (tag == STRAT_FIXED) {
    if (a.size() > (size_t)kMaxSteps) throw CircuitError("reduction strategy: too many FRI steps");
    for (int64_t x : a) C.arities.push_back((int)x);
  } else if (tag == STRAT_MIN_SIZE) {
    if (a.size() > 1) throw ParseError("MinSize: expecting an optional max arity");
    throw CircuitError("reduction strategy not implemented (MinSize), Plonk/FRI.hs:342");
  } else {
    throw ParseError("FriReductionStrategy: unknown constructor tag");
  }
}

// The FRI steps: the reference expands the strategy (above); P2V_EXT_PARAMS_ARITIES takes
// fri_params.reduction_arity_bits as plonky2's verifier does (any strategy, MinSize included;
// the strategy is still decoded and its shape checked).
static void fri_steps(Circuit& C, int tag, const std::vector<int64_t>& a) {
  if (C.ext & P2V_EXT_PARAMS_ARITIES) {
    if (tag == STRAT_CONSTANT_ARITY_BITS && a.size() != 2) throw ParseError("ConstantArityBits: expecting [arity_bits, final_poly_bits]");
    if (tag == STRAT_MIN_SIZE && a.size() > 1) throw ParseError("MinSize: expecting an optional max arity");
    if (tag < STRAT_FIXED || tag > STRAT_MIN_SIZE) throw ParseError("FriReductionStrategy: unknown constructor tag");
    C.arities = C.params_arities;
  } else {
    expand_strategy(C, tag, a);
  }
}

static void finalize_circuit(Circuit& C);

Circuit parse_circuit(const JVal& common, const JVal& vkey, uint32_t ext) {
  Circuit C;
  C.ext = ext;
  const JVal& cfg = common.at("config");
  C.num_wires = j_i32(cfg.at("num_wires"));
  C.num_routed = j_i32(cfg.at("num_routed_wires"));
  C.num_gate_consts = j_i32(cfg.at("num_constants"));
  (void)j_bool(cfg.at("use_base_arithmetic_gate"));
  (void)j_int(cfg.at("security_bits"));
  C.r = j_i32(cfg.at("num_challenges"));
  (void)j_bool(cfg.at("zero_knowledge"));
  (void)j_bool(cfg.at("randomize_unused_wires"));
  C.max_qdf = j_i32(cfg.at("max_quotient_degree_factor"));
  const JVal& fc = cfg.at("fri_config");
  C.rate_bits = j_i32(fc.at("rate_bits"));
  C.cap_height = j_i32(fc.at("cap_height"));
  C.pow_bits = j_i32(fc.at("proof_of_work_bits"));
  C.num_queries = j_i32(fc.at("num_query_rounds"));
  const JVal& rs = fc.at("reduction_strategy");
  if (rs.kind != JVal::Obj || rs.keys.size() != 1) throw ParseError("reduction_strategy: expecting a singleton object");
  const JVal& fp = common.at("fri_params");
  C.hiding = j_bool(fp.at("hiding"));
  C.degree_bits = j_i32(fp.at("degree_bits"));
  for (const auto& x : fp.at("reduction_arity_bits").arr()) C.params_arities.push_back(j_i32(x));
  (void)fp.at("config");
  C.lde_bits = (int)std::max<int64_t>(INT32_MIN, std::min<int64_t>(INT32_MAX, (int64_t)C.degree_bits + C.rate_bits));   // range-checked in finalize_circuit
  if (rs.keys[0] == "ConstantArityBits") {
    const auto& ab = rs.items[0].arr();
    if (ab.size() != 2) throw ParseError("ConstantArityBits: expecting [arity_bits, final_poly_bits]");
    fri_steps(C, STRAT_CONSTANT_ARITY_BITS, {j_int(ab[0]), j_int(ab[1])});
  } else if (rs.keys[0] == "Fixed") {
    std::vector<int64_t> xs;
    for (const auto& x : rs.items[0].arr()) xs.push_back(j_int(x));
    fri_steps(C, STRAT_FIXED, xs);
  } else if (rs.keys[0] == "MinSize") {   // Maybe Log2: null or a number (Types.hs:131)
    const JVal& mx = rs.items[0];
    std::vector<int64_t> xs;
    if (mx.kind == JVal::Num) xs.push_back(j_int(mx));
    else if (mx.kind != JVal::Null) throw ParseError("MinSize: expecting null or an arity");
    fri_steps(C, STRAT_MIN_SIZE, xs);
  } else {
    throw ParseError("FromJSON/FriReductionStrategy: unrecognized FRI reduction strategy");
  }
  for (const auto& g : common.at("gates").arr()) {
    if (g.kind != JVal::Str) throw ParseError("gate must be a string");
    C.gates.push_back(parse_gate_string(g.text));
  }
  const JVal& si = common.at("selectors_info");
  for (const auto& x : si.at("selector_indices").arr()) C.sel_idx.push_back(j_i32(x));
  for (const auto& g : si.at("groups").arr()) { C.grp_start.push_back(j_i32(g.at("start"))); C.grp_end.push_back(j_i32(g.at("end"))); }
  C.qdf = j_i32(common.at("quotient_degree_factor"));
  C.num_gate_constraints = j_i32(common.at("num_gate_constraints"));
  C.num_constants = j_i32(common.at("num_constants"));
  C.num_pis = j_i32(common.at("num_public_inputs"));
  for (const auto& x : common.at("k_is").arr()) C.k_is.push_back(j_field(x));
  C.npp = j_i32(common.at("num_partial_products"));
  C.nlp = j_i32(common.at("num_lookup_polys"));
  C.nls = j_i32(common.at("num_lookup_selectors"));
  for (const auto& t : common.at("luts").arr()) {
    std::vector<uint64_t> in, out;
    for (const auto& e : t.arr()) {
      const auto& pr = e.arr();
      if (pr.size() != 2) throw ParseError("lut entry must be a pair");
      in.push_back(j_word64_mod_p(pr[0])); out.push_back(j_word64_mod_p(pr[1]));
    }
    C.lut_in.push_back(std::move(in)); C.lut_out.push_back(std::move(out));
  }
  for (const auto& d : vkey.at("constants_sigmas_cap").arr()) { uint64_t e[4]; digest_of(d, e); C.cs_cap.insert(C.cs_cap.end(), e, e + 4); }
  digest_of(vkey.at("circuit_digest"), C.digest);
  finalize_circuit(C);
  return C;
}

// Validation (circuit-level `error`s) and everything derived from the decoded fields; shared by
// the JSON and the word-encoded entry points.
static void finalize_circuit(Circuit& C) {
  // ---------------------------------------------------------------- validation
  // Circuit-level `error`s that the reference raises on every verification of this circuit.
  const int ngroups = (int)C.grp_start.size();
  const int nluts = (int)C.lut_in.size();
  if (C.r <= 0 || C.r > 4) throw CircuitError("num_challenges must be in 1..4 (this build)");
  if (C.cap_height < 0 || C.cap_height > 20 || C.degree_bits <= 0 || C.rate_bits < 0 || C.lde_bits > 30) throw CircuitError("unsupported FRI sizes");
  // this build's size limits (far above any Plonky2 config; they keep every derived size in range)
  constexpr int kMaxCount = 1 << 20;
  auto in_range = [](int64_t v, int64_t lo, int64_t hi) { return v >= lo && v <= hi; };
  if (!in_range(C.num_wires, 1, kMaxCount) || !in_range(C.num_routed, 0, C.num_wires) || !in_range(C.num_gate_consts, 0, kMaxCount) ||
      !in_range(C.num_constants, 0, kMaxCount) || !in_range(C.num_pis, 0, kMaxCount) || !in_range(C.npp, 0, kMaxCount) ||
      !in_range(C.nlp, 0, kMaxCount) || !in_range(C.nls, 0, kMaxCount) || !in_range(C.qdf, 0, 1 << 10) ||
      !in_range(C.num_queries, 0, 1 << 10) || !in_range(C.pow_bits, 0, 64) || (int64_t)C.lut_in.size() > kMaxCount)
    throw CircuitError("circuit sizes beyond this build's limits (DESIGN.md §8)");
  if (C.nls != (nluts == 0 ? 0 : 4 + nluts)) throw CircuitError("getSelectorConfig: fatal: num_lookup_selectors /= (4 + #nluts)");
  if (C.num_constants != ngroups + C.nls + C.num_gate_consts) throw CircuitError("getSelectorConfig: fatal: constant columns tally does not add up!");
  C.n_gate_eval = (int)std::min(C.sel_idx.size(), C.gates.size());
  if (C.n_gate_eval == 0) throw CircuitError("foldl1: empty gate list");
  for (int g = 0; g < C.n_gate_eval; g++) {
    const GateDesc& gd = C.gates[g];
    if (gd.kind == G_UNKNOWN) throw CircuitError("gateConstraints: unknown gate `" + gd.text + "`");
    if ((gd.kind == G_POSEIDON || gd.kind == G_POSEIDON_MDS) && gd.p0 != 12) throw CircuitError("PoseidonGate: unsupported width");
    if (gd.kind == G_COSET && (gd.p1 < 2 || gd.p0 < 1 || gd.p0 > 10)) throw CircuitError("CosetInterpolationGate: unsupported parameters");
    if (gd.kind == G_RANDACC && (gd.p0 < 0 || gd.p0 > 16)) throw CircuitError("RandomAccessGate: unsupported bits");
    if (gd.kind == G_BASESUM && (gd.p1 < 0 || gd.p1 > (1 << 16))) throw CircuitError("BaseSumGate: unsupported base");
    int grp = C.sel_idx[g];
    if (grp < 0 || grp >= ngroups) throw CircuitError("selector_groups !! group_idx: index out of range");
    int64_t mw, mc;
    gate_footprint(gd, mw, mc);
    if (mw >= C.num_wires) throw CircuitError("(Array.!): gate reads a wire beyond num_wires: " + gd.text);
    if (mc >= C.num_gate_consts) throw CircuitError("(Array.!): gate reads a constant beyond num_constants: " + gd.text);
  }
  if (C.qdf <= 0) throw CircuitError("quotient_degree_factor must be positive");
  if (C.npp <= 0) throw CircuitError("num_partial_products must be positive");
  {
    int npp_all = (C.num_routed + C.qdf - 1) / C.qdf;   // combineInitial sanity, Plonk/FRI.hs:168
    if (C.r * (npp_all + C.nlp) != C.r * (1 + C.npp + C.nlp)) throw CircuitError("combineInitial: sanity check failed");
  }
  if ((int64_t)C.k_is.size() < C.num_routed) throw CircuitError("k_is shorter than num_routed_wires");
  if (nluts > 0 && (C.nlp < 2 || C.num_routed < 3 || C.qdf < 2)) throw CircuitError("lookup argument: unsupported sizes");

  // ---------------------------------------------------------------- derived shapes
  C.cap_len = 1 << C.cap_height;
  if ((int)C.cs_cap.size() != 4 * C.cap_len) throw CircuitError("validateMerkleCapLength: constants_sigmas_cap has wrong size");
  int sum_a = 0; for (int a : C.arities) { if (a <= 0 || a > 8) throw CircuitError("unsupported FRI arity"); sum_a += a; }
  if (sum_a > C.degree_bits) throw CircuitError("reduction strategy folds below degree 1");
  if (C.arities.size() > 8) throw CircuitError("more than 8 FRI steps");
  C.final_len = C.final_len_override >= 0 ? C.final_len_override : 1 << (C.degree_bits - sum_a);
  C.oracle_width[0] = C.num_constants + C.num_routed;
  C.oracle_width[1] = C.num_wires;
  C.oracle_width[2] = C.r * (1 + C.npp + C.nlp);
  C.oracle_width[3] = C.r * C.qdf;
  {
    const int salt = (C.ext & P2V_EXT_HIDING) && C.hiding ? 4 : 0;   // SALT_SIZE; constants/sigmas are never salted
    for (int t = 0; t < 4; t++) C.leaf_width[t] = C.oracle_width[t] + (t == 0 ? 0 : salt);
  }
  C.noop_leaves = (C.ext & P2V_EXT_HASH_OR_NOOP) != 0;
  C.depth0 = C.lde_bits - C.cap_height;
  if (C.depth0 < 0) throw CircuitError("cap_height exceeds the LDE size");
  C.step_depth.clear();
  { int logn = C.lde_bits; for (int a : C.arities) { logn -= a; C.step_depth.push_back(std::max(0, logn - C.cap_height)); } }
  // term counts before the gate terms (Vanishing.hs:67-111, Lookups.hs:73-132)
  {
    int nnum = std::min<int>(C.num_routed, C.num_wires), nden = std::min<int>(C.num_routed, C.num_wires);
    int nnc = (nnum + C.qdf - 1) / C.qdf, ndc = (nden + C.qdf - 1) / C.qdf;
    int ncur = C.npp + 2;
    C.n_pp_terms_per_round = std::min({ncur - 1, nnc, ndc});
    C.n_lookup_terms_per_round = 0;
    if (nluts > 0) {
      int nlu = std::min(C.num_routed / 2, C.num_wires / 2), nlut = std::min(C.num_routed / 3, C.num_wires / 3);
      int nsldc = C.nlp - 1, lu_degree = C.qdf - 1, lut_degree = (C.num_routed / 3 + nsldc - 1) / nsldc;
      int nclu = (nlu + lu_degree - 1) / lu_degree, nclut = (nlut + lut_degree - 1) / lut_degree, ncm = (C.num_routed / 3 + lut_degree - 1) / lut_degree;
      int nz = std::min({nclu, nclut, ncm, nsldc});
      C.n_lookup_terms_per_round = 3 + nluts + 1 + 2 * nz;
      if (3 * (C.num_routed / 3 - 1) + 2 >= C.num_wires) throw CircuitError("lookup mults beyond num_wires");
    }
    C.alpha_base_gates = C.r + C.r * C.n_pp_terms_per_round + (nluts > 0 ? C.r * C.n_lookup_terms_per_round : 0);
  }
  // ---------------------------------------------------------------- layout
  C.L = Layout{};
  Layout& L = C.L;
  int64_t w = 0;
  L.pis = w; w += C.num_pis;
  L.wcap = w; w += 4 * C.cap_len;
  L.zcap = w; w += 4 * C.cap_len;
  L.qcap = w; w += 4 * C.cap_len;
  L.open = w;
  L.o_const = w; w += 2 * C.num_constants;
  L.o_sig = w; w += 2 * C.num_routed;
  L.o_wires = w; w += 2 * C.num_wires;
  L.o_zs = w; w += 2 * C.r;
  L.o_pp = w; w += 2 * C.r * C.npp;
  L.o_quot = w; w += 2 * C.r * C.qdf;
  L.o_lzs = w; w += 2 * C.r * C.nlp;
  L.n_this = (w - L.open) / 2;
  L.o_zs_next = w; w += 2 * C.r;
  L.o_lzs_next = w; w += 2 * C.r * C.nlp;
  L.n_next = (w - L.o_zs_next) / 2;
  L.ccaps = w; w += (int64_t)C.arities.size() * 4 * C.cap_len;
  L.final_poly = w; w += 2 * C.final_len;
  L.pow = w; w += 1;
  L.q0 = w;
  int64_t q = 0;
  for (int t = 0; t < 4; t++) { L.leaf[t] = q; q += C.leaf_width[t]; }
  for (int t = 0; t < 4; t++) { L.path[t] = q; q += 4 * C.depth0; }
  for (size_t s = 0; s < C.arities.size(); s++) {
    L.step_evals.push_back(q); q += 2 * (1 << C.arities[s]);
    L.step_path.push_back(q); q += 4 * C.step_depth[s];
  }
  L.qstride = q;
  w += q * C.num_queries;
  L.words = w;
  const int S = (int)C.arities.size(), Q = C.num_queries, r = C.r;
  C.trace_words = 4 + 3 * r + 4 * r + 4 + 2 * S + 1 + Q + 4 * r + 6 * Q + 1 + r * (int64_t)C.lut_in.size();
}

// ------------------------------------------------------------------ packing
namespace {
struct Packer {
  const Circuit& C;
  uint64_t* dst;
  int32_t* rec = nullptr;   // optional: packed word -> number ordinal (template recording)
  void put(int64_t idx, const JVal& v) { dst[idx] = j_field(v); if (rec) rec[idx] = v.ord; }
  void digest(const JVal& d, int64_t off) {   // Hash/Digest.hs:40-44
    const auto& e = d.at("elements").arr();
    if (e.size() != 4) throw ParseError("digest must have 4 elements");
    for (int i = 0; i < 4; i++) put(off + i, e[i]);
  }
  void fields(const JVal& v, int64_t off, int64_t n, const char* what) {
    const auto& a = v.arr();
    if ((int64_t)a.size() != n) throw ShapeError(std::string(what) + ": expected " + std::to_string(n) + " elements, got " + std::to_string(a.size()));
    for (int64_t i = 0; i < n; i++) put(off + i, a[i]);
  }
  void exts(const JVal& v, int64_t off, int64_t n, const char* what) {
    const auto& a = v.arr();
    if ((int64_t)a.size() != n) throw ShapeError(std::string(what) + ": expected " + std::to_string(n) + " F^2 values, got " + std::to_string(a.size()));
    for (int64_t i = 0; i < n; i++) {
      const auto& pr = a[i].arr();
      if (pr.size() != 2) throw ParseError("F^2 value must be a pair");
      put(off + 2 * i, pr[0]); put(off + 2 * i + 1, pr[1]);
    }
  }
  void digests(const JVal& v, int64_t off, int64_t n, const char* what) {
    const auto& a = v.arr();
    if ((int64_t)a.size() != n) throw ShapeError(std::string(what) + ": expected " + std::to_string(n) + " digests, got " + std::to_string(a.size()));
    for (int64_t i = 0; i < n; i++) digest(a[i], off + 4 * i);
  }
};
}  // namespace

void pack_proof(const Circuit& C, const JVal& root, uint64_t* dst, int32_t* rec) {
  const Layout& L = C.L;
  Packer P{C, dst, rec};
  const JVal& pr = root.at("proof");
  P.fields(root.at("public_inputs"), L.pis, C.num_pis, "public_inputs");
  P.digests(pr.at("wires_cap"), L.wcap, C.cap_len, "wires_cap");
  P.digests(pr.at("plonk_zs_partial_products_cap"), L.zcap, C.cap_len, "plonk_zs_partial_products_cap");
  P.digests(pr.at("quotient_polys_cap"), L.qcap, C.cap_len, "quotient_polys_cap");
  const JVal& o = pr.at("openings");
  P.exts(o.at("constants"), L.o_const, C.num_constants, "openings.constants");
  P.exts(o.at("plonk_sigmas"), L.o_sig, C.num_routed, "openings.plonk_sigmas");
  P.exts(o.at("wires"), L.o_wires, C.num_wires, "openings.wires");
  P.exts(o.at("plonk_zs"), L.o_zs, C.r, "openings.plonk_zs");
  P.exts(o.at("partial_products"), L.o_pp, (int64_t)C.r * C.npp, "openings.partial_products");
  P.exts(o.at("quotient_polys"), L.o_quot, (int64_t)C.r * C.qdf, "openings.quotient_polys");
  P.exts(o.at("lookup_zs"), L.o_lzs, (int64_t)C.r * C.nlp, "openings.lookup_zs");
  P.exts(o.at("plonk_zs_next"), L.o_zs_next, C.r, "openings.plonk_zs_next");
  P.exts(o.at("lookup_zs_next"), L.o_lzs_next, (int64_t)C.r * C.nlp, "openings.lookup_zs_next");
  const JVal& fp = pr.at("opening_proof");
  const auto& cc = fp.at("commit_phase_merkle_caps").arr();
  const int S = (int)C.arities.size();
  if ((int)cc.size() != S) throw ShapeError("commit_phase_merkle_caps: expected " + std::to_string(S));
  for (int s = 0; s < S; s++) P.digests(cc[s], L.ccaps + (int64_t)s * 4 * C.cap_len, C.cap_len, "commit_phase_merkle_caps[s]");
  P.exts(fp.at("final_poly").at("coeffs"), L.final_poly, C.final_len, "final_poly.coeffs");
  P.put(L.pow, fp.at("pow_witness"));
  const auto& qr = fp.at("query_round_proofs").arr();
  if ((int)qr.size() != C.num_queries) throw ShapeError("query_round_proofs: expected " + std::to_string(C.num_queries));
  for (int q = 0; q < C.num_queries; q++) {
    int64_t base = L.q0 + (int64_t)q * L.qstride;
    const auto& ep = qr[q].at("initial_trees_proof").at("evals_proofs").arr();
    if (ep.size() != 4) throw ShapeError("checkInitialTreeProofs: expecting 4 Merkle proofs for the 4 oracles");
    for (int t = 0; t < 4; t++) {
      const auto& pair = ep[t].arr();
      if (pair.size() != 2) throw ParseError("evals_proofs entry must be a pair");
      P.fields(pair[0], base + L.leaf[t], C.leaf_width[t], "initial tree leaf");
      P.digests(pair[1].at("siblings"), base + L.path[t], C.depth0, "initial tree siblings");
    }
    const auto& st = qr[q].at("steps").arr();
    if ((int)st.size() != S) throw ShapeError("steps: expected " + std::to_string(S));
    for (int s = 0; s < S; s++) {
      P.exts(st[s].at("evals"), base + L.step_evals[s], 1 << C.arities[s], "step evals");
      P.digests(st[s].at("merkle_proof").at("siblings"), base + L.step_path[s], C.step_depth[s], "step siblings");
    }
  }
}

// ------------------------------------------------------------------ shape variants
Circuit circuit_shape_variant(const Circuit& base, int num_pis, int final_len) {
  constexpr int kMaxPis = 1 << 20, kMaxFinal = 1 << 20;   // this build's limits
  if (num_pis < 0 || num_pis > kMaxPis || final_len < 0 || final_len > kMaxFinal)
    throw CircuitError("shape variant beyond this build's limits (public inputs / final polynomial length)");
  Circuit C = base;
  C.num_pis = num_pis;
  C.final_len_override = final_len;
  finalize_circuit(C);   // the same validation; the layout and trace size for these lengths
  return C;
}

void proof_shape_json(const JVal& root, int& num_pis, int& final_len) {
  const size_t np = root.at("public_inputs").arr().size();
  const size_t nf = root.at("proof").at("opening_proof").at("final_poly").at("coeffs").arr().size();
  if (np > (size_t)INT32_MAX || nf > (size_t)INT32_MAX) throw ParseError("proof lists too long");
  num_pis = (int)np; final_len = (int)nf;
}

// ------------------------------------------------------------------ word-encoded values
// The Types.hs values themselves, marshalled field by field into u64 words by a typed host
// (the Haskell shim bindings/haskell/Plonk/VerifierGPU.hs; p2v.py's circuit_words /
// proof_words mirror it): records in declaration order, lists as [length, items...], Int as
// two's complement, Bool as 0/1, F as its value (reduced mod p here, as aeson's Integer is),
// constructors as [tag, fields...] in declaration order.  Layout: include/p2v.h.
namespace {
struct WordReader {
  const uint64_t* w; size_t n; size_t i = 0;
  uint64_t u(const char* what) { if (i >= n) throw ParseError(std::string("words: truncated at ") + what); return w[i++]; }
  int64_t s(const char* what) { return (int64_t)u(what); }
  int i32(const char* what) {   // an Int stored as int here: out-of-range values are rejected, not truncated
    const int64_t x = s(what);
    if (x < INT32_MIN || x > INT32_MAX) throw ParseError(std::string("words: Int out of range in ") + what);
    return (int)x;
  }
  int64_t len(const char* what) {
    const int64_t k = s(what);
    if (k < 0 || (uint64_t)k > n - i) throw ParseError(std::string("words: bad list length of ") + what);
    return k;
  }
  uint64_t f(const char* what) { return u(what) % gl::P; }
  bool b(const char* what) { const uint64_t x = u(what); if (x > 1) throw ParseError(std::string("words: bad Bool in ") + what); return x == 1; }
  void magic(uint64_t m) { if (u("magic") != m) throw ParseError("words: bad magic / version"); }
};

void read_fri_config(WordReader& R, int& rate, int& cap, int& pow, int& tag, std::vector<int64_t>& args, int& nq) {
  rate = R.i32("fri_rate_bits"); cap = R.i32("fri_cap_height"); pow = R.i32("fri_proof_of_work_bits");
  tag = R.i32("fri_reduction_strategy");
  const int64_t k = R.len("reduction strategy fields");
  args.clear();
  for (int64_t i = 0; i < k; i++) args.push_back(R.s("reduction strategy field"));
  nq = R.i32("fri_num_query_rounds");
}

const char* gate_name(int k) {
  static const char* names[] = {"ArithmeticGate", "ArithmeticExtensionGate", "BaseSumGate", "CosetInterpolationGate", "ConstantGate",
                                "ExponentiationGate", "LookupGate", "LookupTableGate", "MulExtensionGate", "NoopGate", "PublicInputGate",
                                "PoseidonGate", "PoseidonMdsGate", "RandomAccessGate", "ReducingGate", "ReducingExtensionGate", "UnknownGate"};
  return k >= 0 && k <= 16 ? names[k] : "UnknownGate";
}
}  // namespace

Circuit parse_circuit_words(const uint64_t* w, size_t n, uint32_t ext) {
  WordReader R{w, n};
  R.magic(P2V_WORDS_CIRCUIT_MAGIC);
  Circuit C;
  C.ext = ext;
  // CircuitConfig (Types.hs:73-84)
  C.num_wires = R.i32("config_num_wires");
  C.num_routed = R.i32("config_num_routed_wires");
  C.num_gate_consts = R.i32("config_num_constants");
  (void)R.b("config_use_base_arithmetic_gate");
  (void)R.s("config_security_bits");
  C.r = R.i32("config_num_challenges");
  (void)R.b("config_zero_knowledge");
  (void)R.b("config_randomize_unused_wires");
  C.max_qdf = R.i32("config_max_quotient_degree_factor");
  int tag = 0, tag2 = 0, d0, d1, d2, d3;
  std::vector<int64_t> sargs, sargs2;
  read_fri_config(R, C.rate_bits, C.cap_height, C.pow_bits, tag, sargs, C.num_queries);
  // FriParams (Types.hs:151-157): its own FriConfig copy, hiding, degree_bits, arity bits
  read_fri_config(R, d0, d1, d2, tag2, sargs2, d3);
  C.hiding = R.b("fri_hiding");
  C.degree_bits = R.i32("fri_degree_bits");
  for (int64_t k = R.len("fri_reduction_arity_bits"); k > 0; k--) C.params_arities.push_back(R.i32("fri_reduction_arity_bits"));
  C.lde_bits = (int)std::max<int64_t>(INT32_MIN, std::min<int64_t>(INT32_MAX, (int64_t)C.degree_bits + C.rate_bits));   // range-checked in finalize_circuit
  fri_steps(C, tag, sargs);
  // gates (Gate/Base.hs:27-45)
  for (int64_t k = R.len("circuit_gates"); k > 0; k--) {
    GateDesc g;
    const int64_t t = R.s("gate constructor");
    auto field = [&]() { return R.s("gate field"); };
    std::string params;
    switch (t) {
      case G_ARITH: case G_ARITH_EXT: case G_CONST: case G_EXP: case G_MULEXT: case G_POSEIDON: case G_POSEIDON_MDS:
      case G_REDUCING: case G_REDUCING_EXT:
        g.p0 = field(); params = std::to_string(g.p0); break;
      case G_BASESUM: g.p0 = field(); g.p1 = field(); params = std::to_string(g.p0) + ", " + std::to_string(g.p1); break;
      case G_COSET: {
        g.p0 = field(); g.p1 = field();
        for (int64_t m = R.len("barycentric_weights"); m > 0; m--) g.weights.push_back(R.f("barycentric weight"));
        params = std::to_string(g.p0) + ", " + std::to_string(g.p1) + ", " + std::to_string(g.weights.size()) + " weights";
        break; }
      case G_LOOKUP: case G_LOOKUPTABLE:
        g.p0 = field();
        for (int64_t m = R.len("lut_hash"); m > 0; m--) (void)R.u("lut_hash byte");
        if (t == G_LOOKUPTABLE) g.p2 = field();
        params = std::to_string(g.p0);
        break;
      case G_NOOP: case G_PI: break;
      case G_RANDACC: g.p0 = field(); g.p1 = field(); g.p2 = field();
        params = std::to_string(g.p0) + ", " + std::to_string(g.p1) + ", " + std::to_string(g.p2); break;
      case G_UNKNOWN: {
        std::string name;
        for (int64_t m = R.len("UnknownGate name"); m > 0; m--) name.push_back((char)R.u("name byte"));
        params = name;
        break; }
      default: throw ParseError("words: unknown Gate constructor tag " + std::to_string(t));
    }
    g.kind = (int32_t)t;
    g.text = std::string(gate_name((int)t)) + "(" + params + ")";
    C.gates.push_back(std::move(g));
  }
  // SelectorsInfo (Types.hs:90-95)
  for (int64_t k = R.len("selector_indices"); k > 0; k--) C.sel_idx.push_back(R.i32("selector index"));
  for (int64_t k = R.len("selector_groups"); k > 0; k--) { C.grp_start.push_back(R.i32("range_start")); C.grp_end.push_back(R.i32("range_end")); }
  if (R.b("selector_vector present")) for (int64_t k = R.len("selector_vector"); k > 0; k--) (void)R.s("selector_vector");
  C.qdf = R.i32("circuit_quotient_degree_factor");
  C.num_gate_constraints = R.i32("circuit_num_gate_constraints");
  C.num_constants = R.i32("circuit_num_constants");
  C.num_pis = R.i32("circuit_num_public_inputs");
  for (int64_t k = R.len("circuit_k_is"); k > 0; k--) C.k_is.push_back(R.f("k_i"));
  C.npp = R.i32("circuit_num_partial_products");
  C.nlp = R.i32("circuit_num_lookup_polys");
  C.nls = R.i32("circuit_num_lookup_selectors");
  for (int64_t k = R.len("circuit_luts"); k > 0; k--) {   // LookupTable = [(Word64, Word64)], Types.hs:28-33
    std::vector<uint64_t> in, out;
    for (int64_t m = R.len("lookup table"); m > 0; m--) { in.push_back(R.u("lut input") % gl::P); out.push_back(R.u("lut output") % gl::P); }
    C.lut_in.push_back(std::move(in)); C.lut_out.push_back(std::move(out));
  }
  // VerifierOnlyCircuitData (Types.hs:236-240)
  for (int64_t k = R.len("constants_sigmas_cap"); k > 0; k--) for (int j = 0; j < 4; j++) C.cs_cap.push_back(R.f("cap digest"));
  for (int j = 0; j < 4; j++) C.digest[j] = R.f("circuit_digest");
  if (R.i != n) throw ParseError("words: trailing words after VerifierCircuitData");
  finalize_circuit(C);
  return C;
}

void pack_proof_words(const Circuit& C, const uint64_t* w, size_t n, uint64_t* dst) {
  WordReader R{w, n};
  R.magic(P2V_WORDS_PROOF_MAGIC);
  const Layout& L = C.L;
  auto fields = [&](int64_t off, int64_t want, const char* what) {
    const int64_t k = R.len(what);
    if (k != want) throw ShapeError(std::string(what) + ": expected " + std::to_string(want) + " elements, got " + std::to_string(k));
    for (int64_t i = 0; i < k; i++) dst[off + i] = R.f(what);
  };
  auto exts = [&](int64_t off, int64_t want, const char* what) {
    const int64_t k = R.len(what);
    if (k != want) throw ShapeError(std::string(what) + ": expected " + std::to_string(want) + " F^2 values, got " + std::to_string(k));
    for (int64_t i = 0; i < 2 * k; i++) dst[off + i] = R.f(what);
  };
  auto digests = [&](int64_t off, int64_t want, const char* what) {
    const int64_t k = R.len(what);
    if (k != want) throw ShapeError(std::string(what) + ": expected " + std::to_string(want) + " digests, got " + std::to_string(k));
    for (int64_t i = 0; i < 4 * k; i++) dst[off + i] = R.f(what);
  };
  // Proof (Types.hs:256-263)
  digests(L.wcap, C.cap_len, "wires_cap");
  digests(L.zcap, C.cap_len, "plonk_zs_partial_products_cap");
  digests(L.qcap, C.cap_len, "quotient_polys_cap");
  // OpeningSet, field order (Types.hs:265-276)
  exts(L.o_const, C.num_constants, "openings.constants");
  exts(L.o_sig, C.num_routed, "openings.plonk_sigmas");
  exts(L.o_wires, C.num_wires, "openings.wires");
  exts(L.o_zs, C.r, "openings.plonk_zs");
  exts(L.o_zs_next, C.r, "openings.plonk_zs_next");
  exts(L.o_pp, (int64_t)C.r * C.npp, "openings.partial_products");
  exts(L.o_quot, (int64_t)C.r * C.qdf, "openings.quotient_polys");
  exts(L.o_lzs, (int64_t)C.r * C.nlp, "openings.lookup_zs");
  exts(L.o_lzs_next, (int64_t)C.r * C.nlp, "openings.lookup_zs_next");
  // FriProof (Types.hs:176-181)
  const int S = (int)C.arities.size();
  if (R.len("commit_phase_merkle_caps") != S) throw ShapeError("commit_phase_merkle_caps: expected " + std::to_string(S));
  for (int s = 0; s < S; s++) digests(L.ccaps + (int64_t)s * 4 * C.cap_len, C.cap_len, "commit_phase_merkle_caps[s]");
  if (R.len("query_round_proofs") != C.num_queries) throw ShapeError("query_round_proofs: expected " + std::to_string(C.num_queries));
  for (int q = 0; q < C.num_queries; q++) {
    const int64_t base = L.q0 + (int64_t)q * L.qstride;
    if (R.len("evals_proofs") != 4) throw ShapeError("checkInitialTreeProofs: expecting 4 Merkle proofs for the 4 oracles");
    for (int t = 0; t < 4; t++) {
      fields(base + L.leaf[t], C.leaf_width[t], "initial tree leaf");
      digests(base + L.path[t], C.depth0, "initial tree siblings");
    }
    if (R.len("steps") != S) throw ShapeError("steps: expected " + std::to_string(S));
    for (int s = 0; s < S; s++) {
      exts(base + L.step_evals[s], 1 << C.arities[s], "step evals");
      digests(base + L.step_path[s], C.step_depth[s], "step siblings");
    }
  }
  exts(L.final_poly, C.final_len, "final_poly.coeffs");
  dst[L.pow] = R.f("pow_witness");
  fields(L.pis, C.num_pis, "public_inputs");   // ProofWithPublicInputs: the_proof, public_inputs
  if (R.i != n) throw ParseError("words: trailing words after ProofWithPublicInputs");
}

// the final polynomial's and the public inputs' lengths of a word-encoded proof, walking the
// self-describing list structure of pack_proof_words without assuming the circuit's shapes
void proof_shape_words(const uint64_t* w, size_t n, int& num_pis, int& final_len) {
  WordReader R{w, n};
  R.magic(P2V_WORDS_PROOF_MAGIC);
  auto skip = [&](int64_t per, const char* what) { const int64_t k = R.len(what); if ((uint64_t)k > (n - R.i) / (uint64_t)per) throw ParseError(std::string("words: bad list length of ") + what); R.i += (size_t)(k * per); return k; };
  for (int t = 0; t < 3; t++) skip(4, "cap");
  for (int t = 0; t < 9; t++) skip(2, "openings");
  for (int64_t s = R.len("commit_phase_merkle_caps"); s > 0; s--) skip(4, "commit cap");
  for (int64_t q = R.len("query_round_proofs"); q > 0; q--) {
    for (int64_t t = R.len("evals_proofs"); t > 0; t--) { skip(1, "initial tree leaf"); skip(4, "initial tree siblings"); }
    for (int64_t s = R.len("steps"); s > 0; s--) { skip(2, "step evals"); skip(4, "step siblings"); }
  }
  const int64_t nf = skip(2, "final_poly.coeffs");
  (void)R.u("pow_witness");
  const int64_t np = skip(1, "public_inputs");
  if (R.i != n) throw ParseError("words: trailing words after ProofWithPublicInputs");
  if (nf > INT32_MAX || np > INT32_MAX) throw ParseError("proof lists too long");
  final_len = (int)nf; num_pis = (int)np;
}

// ------------------------------------------------------------------ plonky2 binary proofs
// ProofWithPublicInputs in plonky2's own byte serialization (util/serialization: Write::
// write_proof_with_public_inputs), the step before JSON in deployments (SURVEY.md §8f row 3;
// unchecked in the reference, README.md:27).  Restated from plonky2 (not in /root/reference):
// u64 little-endian words; F = its canonical u64 (reduced mod p here, as the JSON path reduces);
// FExt = 2 F; HashOut = 4 F; MerkleCap = 2^cap_height hashes (no length); MerkleProof = u8
// sibling count, then the hashes; vectors whose length the circuit fixes carry no length.
//   Proof: wires_cap, plonk_zs_partial_products_cap, quotient_polys_cap,
//     OpeningSet: constants, plonk_sigmas, wires, plonk_zs, plonk_zs_next, lookup_zs,
//       lookup_zs_next, partial_products, quotient_polys,
//     FriProof: commit-phase caps, query rounds (4 x (leaf [F], MerkleProof), steps x
//       (evals [FExt], MerkleProof)), final_poly [FExt], pow_witness F
//   public_inputs: the remaining words, or a u64 count then the words (both forms occur; the
//     remaining byte count tells them apart).
// Parity unpinned: no binary fixture exists offline; tests check it against the JSON path.
namespace {
struct ByteReader {
  const uint8_t* b; size_t n; size_t i = 0;
  uint64_t u64(const char* what) {
    if (n - i < 8) throw ParseError(std::string("bytes: truncated at ") + what);
    uint64_t x = 0;
    for (int k = 7; k >= 0; k--) x = (x << 8) | b[i + k];
    i += 8;
    return x;
  }
  uint8_t u8(const char* what) { if (i >= n) throw ParseError(std::string("bytes: truncated at ") + what); return b[i++]; }
};
}  // namespace

// The fixed part of the format in order: fields(dst_word, nwords, what) for every run of u64
// words, count(expected, what) for every u8 sibling count.  Shared by the host reader below and
// the device packer's map (bytes_map), so both follow one order.
template <class Fields, class Count>
static void bytes_walk(const Circuit& C, Fields&& fields, Count&& count) {
  const Layout& L = C.L;
  auto exts = [&](int64_t off, int64_t k, const char* what) { fields(off, 2 * k, what); };
  auto cap = [&](int64_t off, const char* what) { fields(off, 4 * (int64_t)C.cap_len, what); };
  auto path = [&](int64_t off, int depth, const char* what) { count(depth, what); fields(off, 4 * (int64_t)depth, what); };
  cap(L.wcap, "wires_cap");
  cap(L.zcap, "plonk_zs_partial_products_cap");
  cap(L.qcap, "quotient_polys_cap");
  exts(L.o_const, C.num_constants, "openings.constants");
  exts(L.o_sig, C.num_routed, "openings.plonk_sigmas");
  exts(L.o_wires, C.num_wires, "openings.wires");
  exts(L.o_zs, C.r, "openings.plonk_zs");
  exts(L.o_zs_next, C.r, "openings.plonk_zs_next");
  exts(L.o_lzs, (int64_t)C.r * C.nlp, "openings.lookup_zs");
  exts(L.o_lzs_next, (int64_t)C.r * C.nlp, "openings.lookup_zs_next");
  exts(L.o_pp, (int64_t)C.r * C.npp, "openings.partial_products");
  exts(L.o_quot, (int64_t)C.r * C.qdf, "openings.quotient_polys");
  const int S = (int)C.arities.size();
  for (int s = 0; s < S; s++) cap(L.ccaps + (int64_t)s * 4 * C.cap_len, "commit_phase_merkle_caps");
  for (int q = 0; q < C.num_queries; q++) {
    const int64_t base = L.q0 + (int64_t)q * L.qstride;
    for (int t = 0; t < 4; t++) {
      fields(base + L.leaf[t], C.leaf_width[t], "initial tree leaf");
      path(base + L.path[t], C.depth0, "initial tree siblings");
    }
    for (int s = 0; s < S; s++) {
      exts(base + L.step_evals[s], 1 << C.arities[s], "step evals");
      path(base + L.step_path[s], C.step_depth[s], "step siblings");
    }
  }
  exts(L.final_poly, C.final_len, "final_poly.coeffs");
  fields(L.pow, 1, "pow_witness");
}

void pack_proof_bytes(const Circuit& C, const uint8_t* bytes, size_t n, uint64_t* dst) {
  const Layout& L = C.L;
  ByteReader R{bytes, n};
  auto fields = [&](int64_t off, int64_t k, const char* what) { for (int64_t i = 0; i < k; i++) dst[off + i] = R.u64(what) % gl::P; };
  auto count = [&](int depth, const char* what) {
    const int len = R.u8(what);
    if (len != depth) throw ShapeError(std::string(what) + ": expected " + std::to_string(depth) + " siblings, got " + std::to_string(len));
  };
  bytes_walk(C, fields, count);
  const size_t rest = n - R.i, np = (size_t)C.num_pis;
  if (rest == 8 * np) fields(L.pis, C.num_pis, "public_inputs");
  else if (rest == 8 * (np + 1)) {
    if (R.u64("public_inputs length") != np) throw ShapeError("public_inputs: length prefix differs from num_public_inputs");
    fields(L.pis, C.num_pis, "public_inputs");
  } else {
    throw ShapeError("public_inputs: " + std::to_string(rest) + " trailing bytes for " + std::to_string(np) + " public inputs");
  }
}

BytesMap bytes_map(const Circuit& C) {
  BytesMap m;
  int64_t pos = 0;
  auto fields = [&](int64_t off, int64_t k, const char*) {
    if (k <= 0) return;
    const size_t r = m.run_len.size();
    if (r && m.run_src[r - 1] + 8 * m.run_len[r - 1] == pos && m.run_dst[r - 1] + m.run_len[r - 1] == off) m.run_len[r - 1] += k;
    else { m.run_src.push_back(pos); m.run_dst.push_back(off); m.run_len.push_back(k); }
    pos += 8 * k;
  };
  auto count = [&](int depth, const char*) { m.chk_off.push_back(pos); m.chk_val.push_back((uint8_t)depth); pos += 1; };
  bytes_walk(C, fields, count);
  m.fixed = pos;
  return m;
}

// ------------------------------------------------------------------ template-guided pack
// Proofs of one circuit from one producer share their JSON text except for the numbers.
// The template proof is parsed by the DOM reader recording every number token's span and
// the packed word it lands in; a later proof whose bytes between number tokens equal the
// template's has the same JSON tree, so its numbers go straight to those words.  Anything
// else (other whitespace or key order, a non-integral token where a field element is
// read) returns false and the caller uses the DOM reader, which also produces the
// reference's error for malformed input.
bool ProofTemplate::build(const Circuit& C, const char* s, size_t n, uint64_t* dst) {
  spans.clear();
  JVal root = JParser(s, n, &spans).parse();
  std::vector<int32_t> rec((size_t)C.L.words, -1);
  pack_proof(C, root, dst, rec.data());
  dst_of.assign(spans.size(), -1);
  for (int64_t w = 0; w < C.L.words; w++) if (rec[w] >= 0) dst_of[rec[w]] = w;
  text.assign(s, n);
  return true;
}

namespace {
// 8 ASCII bytes (little-endian load) all in '0'..'9'?  Then their value (SWAR: three
// multiplies instead of eight multiply-adds; the usual branch-free digit-block parse).
inline bool eight_digits(uint64_t v) {
  return (((v & 0xF0F0F0F0F0F0F0F0ULL) | (((v + 0x0606060606060606ULL) & 0xF0F0F0F0F0F0F0F0ULL) >> 4)) == 0x3333333333333333ULL);
}
inline uint32_t eight_value(uint64_t v) {
  v -= 0x3030303030303030ULL;
  v = v * 10 + (v >> 8);
  v = (((v & 0x000000FF000000FFULL) * 0x000F424000000064ULL) + (((v >> 16) & 0x000000FF000000FFULL) * 0x0000271000000001ULL)) >> 32;
  return (uint32_t)v;
}
inline uint64_t load8(const char* p) { uint64_t w; memcpy(&w, p, 8); return w; }
// per byte of 8 ASCII bytes: 0x80 where the byte is not '0'..'9' (bytes >= 0x80: caller checks)
inline uint64_t nondigit_mask(uint64_t v) {
  const uint64_t a = (v & 0xF0F0F0F0F0F0F0F0ULL) ^ 0x3030303030303030ULL;
  const uint64_t b = ((v + 0x0606060606060606ULL) & 0xF0F0F0F0F0F0F0F0ULL) ^ 0x3030303030303030ULL;
  const uint64_t m = a | b;
  return (((m & 0x7F7F7F7F7F7F7F7FULL) + 0x7F7F7F7F7F7F7F7FULL) | m) & 0x8080808080808080ULL;
}
// integer token starting at s (optional '-', then digits) -> its end and its field value;
// false if the token continues with a fraction / exponent character (caller falls back)
inline bool number_fast(const char* s, const char* end, const char*& tok_end, uint64_t& out) {
  const char* p = s;
  const bool neg = *p == '-';
  p += neg;
  const char* q = p;
  for (;;) {   // digit run
    if (q + 8 <= end) {
      const uint64_t v = load8(q);
      if (v & 0x8080808080808080ULL) { while (q < end && *q >= '0' && *q <= '9') q++; break; }
      const uint64_t m = nondigit_mask(v);
      if (m) { q += __builtin_ctzll(m) >> 3; break; }
      q += 8;
    } else { while (q < end && *q >= '0' && *q <= '9') q++; break; }
  }
  tok_end = q;
  if (q < end && is_num_char(*q)) return false;   // '.', 'e', 'E', '+', '-' inside the token
  const size_t nd = (size_t)(q - p);
  if (nd == 0) return false;
  uint64_t acc;
  if (nd > 20) {
    if (!field_of_text(s, (size_t)(q - s), out)) return false;
    return true;
  }
  acc = 0;
  size_t i = 0;
  const size_t head = nd > 19 ? 19 : nd;
  for (; i + 8 <= head; i += 8) acc = acc * 100000000ULL + eight_value(load8(p + i));
  for (; i < head; i++) acc = acc * 10 + (uint64_t)(p[i] - '0');
  if (nd == 20) {   // acc < 10^19: acc*10 + d < 2^64 * 10 -> fold 2^64 == 2^32 - 1 (mod p)
    const unsigned __int128 x = (unsigned __int128)acc * 10 + (uint64_t)(p[19] - '0');
    const uint64_t hi = (uint64_t)(x >> 64), lo = (uint64_t)x;
    uint64_t r = lo + hi * 0xFFFFFFFFULL;
    if (r < lo) r += 0xFFFFFFFFULL;
    acc = r;
  }
  while (acc >= GL_P) acc -= GL_P;
  out = (neg && acc) ? GL_P - acc : acc;
  return true;
}
inline bool same(const char* a, const char* b, size_t n) {
  if (n <= 16) { for (size_t i = 0; i < n; i++) if (a[i] != b[i]) return false; return true; }
  return memcmp(a, b, n) == 0;
}
}  // namespace

bool ProofTemplate::device_form(std::vector<uint8_t>& skel, std::vector<int32_t>& tok_dst) const {
  auto numc = [](char c) { return (c >= '0' && c <= '9') || c == '-'; };
  skel.clear(); tok_dst.clear();
  size_t k = 0, i = 0;
  const size_t n = text.size();
  while (i < n) {
    if (!numc(text[i])) { skel.push_back((uint8_t)text[i]); i++; continue; }
    size_t j = i;
    while (j < n && numc(text[j])) j++;
    if (k >= spans.size() || spans[k].first != i || spans[k].second != j) return false;
    tok_dst.push_back((int32_t)dst_of[k]);
    k++;
    i = j;
  }
  return k == spans.size();
}

bool ProofTemplate::pack(const char* s, size_t n, uint64_t* dst) const {
  const char* t = text.data();
  size_t ps = 0, pt = 0;
  for (size_t k = 0; k < spans.size(); k++) {
    const size_t seg = spans[k].first - pt;   // skeleton bytes before number k
    if (ps + seg > n || !same(s + ps, t + pt, seg)) return false;
    ps += seg;
    pt = spans[k].second;
    if (ps >= n || !(s[ps] == '-' || (s[ps] >= '0' && s[ps] <= '9'))) return false;
    const char* te;
    uint64_t val;
    if (!number_fast(s + ps, s + n, te, val)) return false;
    ps = (size_t)(te - s);
    const int64_t w = dst_of[k];
    if (w >= 0) dst[w] = val;
  }
  const size_t tail = text.size() - pt;
  return ps + tail == n && memcmp(s + ps, t + pt, tail) == 0;
}

}  // namespace p2v
