// circuit.hpp — host side of the drop-in boundary: decode VerifierCircuitData
// (reference src/Types.hs:47-240, Gate strings src/Gate/Parser.hs:27-242), validate it
// once (circuit-level `error`s of the reference surface here), derive the fixed packed
// proof layout, and pack ProofWithPublicInputs JSON (Types.hs:245-279) into it.
#pragma once
#include <cstdint>
#include <string>
#include <vector>
#include "json.hpp"

namespace p2v {

enum GateKind : int32_t {   // Gate/Base.hs:27-45
  G_ARITH = 0, G_ARITH_EXT, G_BASESUM, G_COSET, G_CONST, G_EXP, G_LOOKUP, G_LOOKUPTABLE,
  G_MULEXT, G_NOOP, G_PI, G_POSEIDON, G_POSEIDON_MDS, G_RANDACC, G_REDUCING, G_REDUCING_EXT, G_UNKNOWN
};

struct GateDesc {
  int32_t kind = G_UNKNOWN;
  int64_t p0 = 0, p1 = 0, p2 = 0;
  std::vector<uint64_t> weights;   // CosetInterpolationGate barycentric weights
  std::string text;
};

// Fixed per-circuit packed proof layout (u64 words).  Order:
//   pis | wires_cap | zs_pp_cap | quotient_cap | openings(batch_this ++ batch_next)
//   | commit caps | final poly | pow witness | Q x [4 leaves | 4 paths | steps x (evals | path)]
struct Layout {
  int64_t pis = 0, wcap = 0, zcap = 0, qcap = 0;
  int64_t open = 0;                         // start of the F^2 openings (2 words each)
  int64_t o_const = 0, o_sig = 0, o_wires = 0, o_zs = 0, o_pp = 0, o_quot = 0, o_lzs = 0;   // batch_this
  int64_t o_zs_next = 0, o_lzs_next = 0;    // batch_next
  int64_t n_this = 0, n_next = 0;           // F^2 counts
  int64_t ccaps = 0, final_poly = 0, pow = 0;
  int64_t q0 = 0, qstride = 0;
  int64_t leaf[4] = {0, 0, 0, 0}, path[4] = {0, 0, 0, 0};   // offsets inside one query
  std::vector<int64_t> step_evals, step_path;                 // offsets inside one query
  int64_t words = 0;
};

struct Circuit {
  // CircuitConfig (Types.hs:73-84)
  int num_wires = 0, num_routed = 0, num_gate_consts = 0, r = 0, max_qdf = 0;
  // FriConfig / FriParams (Types.hs:116-174)
  int rate_bits = 0, cap_height = 0, pow_bits = 0, num_queries = 0, degree_bits = 0, lde_bits = 0;
  std::vector<int> arities;                 // expandReductionStrategy, Plonk/FRI.hs:337-354
  bool hiding = false;                      // fri_params.hiding (Types.hs:153)
  std::vector<int> params_arities;          // fri_params.reduction_arity_bits (Types.hs:155)
  uint32_t ext = 0;                         // P2V_EXT_* (include/p2v.h): opt-in plonky2 conventions
  // CommonCircuitData (Types.hs:47-61)
  std::vector<GateDesc> gates;
  std::vector<int> sel_idx;
  std::vector<int> grp_start, grp_end;
  int qdf = 0, num_gate_constraints = 0, num_constants = 0, num_pis = 0;
  std::vector<uint64_t> k_is;
  int npp = 0, nlp = 0, nls = 0;
  std::vector<std::vector<uint64_t>> lut_in, lut_out;
  // VerifierOnlyCircuitData (Types.hs:236-240)
  std::vector<uint64_t> cs_cap;             // 4 words per digest
  uint64_t digest[4] = {0, 0, 0, 0};
  int final_len_override = -1;               // shape variant (circuit_shape_variant): final_poly length
  // derived
  int cap_len = 0, final_len = 0;
  int oracle_width[4] = {0, 0, 0, 0};       // data columns per initial oracle (Plonk/FRI.hs:56-65)
  int leaf_width[4] = {0, 0, 0, 0};         // packed leaf words: + SALT_SIZE salts under P2V_EXT_HIDING
  bool noop_leaves = false;                 // P2V_EXT_HASH_OR_NOOP: leaves of <= 4 words are their digest
  int depth0 = 0;                           // initial Merkle path length
  std::vector<int> step_depth;
  int n_gate_eval = 0;                      // gates actually evaluated: min(#selector_indices, #gates)
  int64_t alpha_base_gates = 0;             // #terms before the gate terms (Vanishing.hs:67-72)
  int64_t n_pp_terms_per_round = 0, n_lookup_terms_per_round = 0;
  Layout L;
  int64_t trace_words = 0;
};

Circuit parse_circuit(const JVal& common, const JVal& vkey, uint32_t ext = 0);   // throws ParseError / CircuitError
// the same from the word-encoded Types.hs values (include/p2v.h, "Word-encoded values")
Circuit parse_circuit_words(const uint64_t* words, size_t n, uint32_t ext = 0);   // throws ParseError / CircuitError
void pack_proof_words(const Circuit& c, const uint64_t* words, size_t n, uint64_t* dst);   // ParseError / ShapeError
// plonky2's binary ProofWithPublicInputs serialization (circuit.cpp); ParseError / ShapeError
void pack_proof_bytes(const Circuit& c, const uint8_t* bytes, size_t n, uint64_t* dst);
// The same format as a fixed map for the device packer (json_pack.hip k_bytes_pack): runs of u64
// words (source byte offset, packed word, count) in file order, the sibling-count bytes and their
// expected values, and the byte length before the public inputs.
struct BytesMap {
  std::vector<int64_t> run_src, run_dst, run_len;
  std::vector<int64_t> chk_off;
  std::vector<uint8_t> chk_val;
  int64_t fixed = 0;
};
BytesMap bytes_map(const Circuit& c);
// throws ParseError / ShapeError; rec (optional, [words]) receives each packed word's number ordinal
void pack_proof(const Circuit& c, const JVal& proof, uint64_t* dst, int32_t* rec = nullptr);

// template-guided fast path of pack_proof (circuit.cpp); pack() == false: use pack_proof
struct ProofTemplate {
  std::string text;
  std::vector<std::pair<size_t, size_t>> spans;   // number tokens of the template text
  std::vector<int64_t> dst_of;                    // number ordinal -> packed word (-1: unused)
  bool build(const Circuit& c, const char* s, size_t n, uint64_t* dst);   // throws like pack_proof
  bool pack(const char* s, size_t n, uint64_t* dst) const;
  // the device form of the template (json_pack.hip): the skeleton (every byte outside the
  // number tokens, concatenated) and the packed word of each token.  False when a byte-level
  // scan for runs of [0-9-] would not find exactly the template's number tokens (e.g. digits
  // inside a key): the device path is then unusable for this template.
  bool device_form(std::vector<uint8_t>& skel, std::vector<int32_t>& tok_dst) const;
};
GateDesc parse_gate_string(const std::string& s);              // Gate/Parser.hs:107-130

// Shape variants.  The reference reads public_inputs and final_poly.coeffs at whatever length a
// proof carries (Hash/Sponge.hs:26-31, Plonk/FRI.hs:325-327, Challenge/FRI.hs:83); the packed
// layout is fixed per circuit, so a proof with other lengths is verified against a variant of the
// circuit whose layout has them.  Throws CircuitError past this build's limits.
Circuit circuit_shape_variant(const Circuit& base, int num_pis, int final_len);
// the two lengths as a proof carries them (JSON / word-encoded); ParseError if they cannot be read
void proof_shape_json(const JVal& proof, int& num_pis, int& final_len);
void proof_shape_words(const uint64_t* words, size_t n, int& num_pis, int& final_len);

}  // namespace p2v
