/*
 * p2v.h — C-ABI of libp2v, the MI355X-native batch Plonky2 verifier.
 *
 * This is the drop-in boundary for the reference's single entry point
 *
 *     verifyProof :: VerifierCircuitData -> ProofWithPublicInputs -> Bool
 *                                              (reference src/Plonk/Verifier.hs:56-65)
 *
 * whose inputs are the Types.hs values decoded from JSON by the aeson instances
 * (reference src/Types.hs:47-279, Gate strings via src/Gate/Parser.hs:27-242).
 * The reference has no FFI; INTEGRATION.md shows the Haskell `foreign import ccall`
 * binding (and the ctypes stub used by our Python mirror) for every entry point here.
 *
 * Conventions
 *   - plain pointers + sizes only; no torch / HIP types in any signature
 *   - functions return int: 0 = OK, < 0 = P2V_E_* (message via p2v_last_error_message())
 *   - per-proof results are int8 status codes P2V_ACCEPT / P2V_REJECT / P2V_ERR_*
 *     reproducing the reference's evaluation order:
 *     Plonk identity -> PoW -> query rounds in order (initial Merkle, steps
 *     (Merkle, eval, arity), final polynomial).
 *   - the caller owns every buffer; the library owns opaque handles.
 */
#ifndef P2V_H
#define P2V_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- per-proof status codes (int8) -------------------------------------------- */
#define P2V_ACCEPT             1   /* verifyProof == True                                   */
#define P2V_REJECT             0   /* verifyProof == False (Plonk identity, PoW, final poly) */
#define P2V_ERR_INITIAL_MERKLE (-1) /* error "checkInitialTreeProofs: ... Merkle proof failed" Plonk/FRI.hs:108 */
#define P2V_ERR_STEP_MERKLE    (-2) /* error "folding step Merkle proof does not check out"   Plonk/FRI.hs:310 */
#define P2V_ERR_STEP_EVAL      (-3) /* error "folding step evaluation does not match ..."      Plonk/FRI.hs:311 */
#define P2V_ERR_STEP_ARITY     (-4) /* error "folding stpe: reduction strategy ..."            Plonk/FRI.hs:312 */
#define P2V_ERR_SHAPE          (-5) /* a list-length / shape `error` (safeZip*, buildListOracle, caps)      */
#define P2V_ERR_CIRCUIT        (-6) /* circuit-level `error` (unknown gate, selector tally, MinSize, ...)   */
#define P2V_ERR_PARSE          (-7) /* JSON did not decode (aeson `decode` == Nothing)                      */

/* ---- function return codes ---------------------------------------------------- */
#define P2V_OK          0
#define P2V_E_PARSE    (-1)
#define P2V_E_CIRCUIT  (-2)
#define P2V_E_SHAPE    (-3)
#define P2V_E_ARG      (-4)
#define P2V_E_DEVICE   (-5)
#define P2V_E_NODEVICE (-6)

typedef struct p2v_circuit  p2v_circuit;   /* parsed VerifierCircuitData (Types.hs:220-224)   */
typedef struct p2v_verifier p2v_verifier;  /* per-device workspace bound to one circuit         */

/* Shape summary of a circuit (all derived from CommonCircuitData). */
typedef struct p2v_circuit_info {
  int32_t degree_bits;        /* fri_params.degree_bits                          Types.hs:165 */
  int32_t lde_bits;           /* degree_bits + rate_bits                         Types.hs:165-167 */
  int32_t cap_height;
  int32_t num_challenges;     /* r                                               */
  int32_t num_query_rounds;   /* Q                                               */
  int32_t num_fri_steps;      /* from the reduction strategy, Plonk/FRI.hs:337-354 */
  int32_t final_poly_len;     /* coefficients (F^2) of the final polynomial      */
  int32_t num_public_inputs;
  int32_t num_openings_this;  /* F^2 values in the first FRI opening batch       */
  int32_t num_openings_next;  /* F^2 values in the second batch                   */
  int32_t has_lookups;
  int32_t num_gates;
  int64_t proof_words;        /* u64 words of one packed proof                    */
  int64_t trace_words;        /* u64 words of one debug trace (see p2v_trace_layout) */
  int32_t oracle_widths[4];   /* data widths of the 4 initial oracles  Plonk/FRI.hs:56-65 */
  int32_t step_arity_bits[8];
  int32_t leaf_widths[4];     /* packed leaf widths: oracle_widths + salts (P2V_EXT_HIDING), else equal */
  uint32_t ext;               /* the P2V_EXT_* flags the circuit was created with */
} p2v_circuit_info;

/* ---- circuits (host-only, no GPU needed) --------------------------------------- */
int  p2v_circuit_from_json(const char* common_json, size_t common_len,
                           const char* vkey_json,   size_t vkey_len,
                           p2v_circuit** out);
void p2v_circuit_free(p2v_circuit* c);

/* ---- opt-in plonky2 semantics the reference does not implement ------
 * With ext = 0 (p2v_circuit_from_json / _from_words) every entry point follows the reference
 * exactly.  The flags below switch single conventions to what plonky2's own verifier does, for
 * circuits the reference rejects; nothing in the reference pins them (parity unpinned).
 *   P2V_EXT_PARAMS_ARITIES  the FRI steps are fri_params.reduction_arity_bits, as plonky2's
 *                           verifier reads them, instead of expanding the strategy from
 *                           degree_bits (Plonk/FRI.hs:337-354, :378); MinSize (an `error` in the
 *                           reference, Plonk/FRI.hs:342) is then accepted
 *   P2V_EXT_HIDING          when fri_params.hiding: the wires, zs/partial-products and quotient
 *                           leaves carry SALT_SIZE = 4 trailing salt elements, hashed into the leaf
 *                           and left out of combineInitial (plonky2 FriInitialTreeProof::
 *                           unsalted_evals; the reference errors in buildListOracle, Plonk/FRI.hs:74)
 *   P2V_EXT_HASH_OR_NOOP    Merkle leaves (initial and FRI step) of <= 4 elements are the digest
 *                           itself, zero-padded (plonky2 hash_or_noop; the reference always
 *                           sponges, Hash/Merkle.hs:27-28, commentary/FRI.md:14) */
#define P2V_EXT_PARAMS_ARITIES 1u
#define P2V_EXT_HIDING         2u
#define P2V_EXT_HASH_OR_NOOP   4u
#define P2V_EXT_PLONKY2        7u   /* all of the above */
int  p2v_circuit_from_json_ex(const char* common_json, size_t common_len,
                              const char* vkey_json,   size_t vkey_len,
                              uint32_t ext, p2v_circuit** out);
int  p2v_circuit_get_info(const p2v_circuit* c, p2v_circuit_info* info);

/* Pack one ProofWithPublicInputs JSON (Types.hs:245-254) into the circuit's fixed
 * layout: dst must hold info.proof_words u64.  Field elements are canonicalised mod p
 * (Goldilocks.hs:101-102).  Returns P2V_E_PARSE on bad JSON, P2V_E_SHAPE when a list
 * length differs from what the circuit implies (the reference would raise a shape
 * `error` or mis-verify on such input). */
int  p2v_pack_proof_json(const p2v_circuit* c, const char* proof_json, size_t len, uint64_t* dst);

/* Batch form of p2v_pack_proof_json, on `threads` host threads (<= 0: all cores): proof i
 * goes to dst[i * proof_words], its code (P2V_OK / P2V_E_PARSE / P2V_E_SHAPE) to codes[i].
 * Proofs whose JSON text equals the first proof's except for the numbers take a
 * template-guided linear scan; any other proof goes through the full reader (same results,
 * same errors).  Returns the number of proofs that failed (message of the first one in
 * p2v_last_error_message), or a negative code on bad arguments.
 * Replaces: `decode` of a list of ProofWithPublicInputs (Types.hs:245-254). */
int  p2v_pack_proofs_json(const p2v_circuit* c, const char* const* jsons, const size_t* lens, size_t n,
                          uint64_t* dst, int32_t* codes, int threads);

/* ---- word-encoded Types.hs values (typed hosts: the Haskell shim) -----------------
 * A host that holds decoded Types.hs values (VerifierCircuitData, ProofWithPublicInputs —
 * neither CommonCircuitData nor ProofWithPublicInputs has a ToJSON instance, Types.hs:71,251)
 * marshals them into u64 words instead of re-encoding JSON.  Encoding (version 1):
 *   record          its fields in declaration order
 *   [a]             length n, then the n items
 *   Int / Log2      two's complement            Bool   0 / 1
 *   F               its value (any u64; reduced mod p like aeson's Integer, Goldilocks.hs:98-102)
 *   FExt            re, im                      Digest  4 x F            MerkleCap  [Digest]
 *   Maybe a         0 | 1, a                    constructor: tag (declaration order), then fields
 * VerifierCircuitData words = P2V_WORDS_CIRCUIT_MAGIC, then
 *   CircuitConfig (Types.hs:73-84): num_wires, num_routed_wires, num_constants,
 *       use_base_arithmetic_gate, security_bits, num_challenges, zero_knowledge,
 *       randomize_unused_wires, max_quotient_degree_factor, FriConfig
 *   FriConfig (:116-122): rate_bits, cap_height, proof_of_work_bits,
 *       reduction_strategy = tag (0 Fixed, 1 ConstantArityBits, 2 MinSize) + [its Log2 fields]
 *       (Fixed: the arity list; ConstantArityBits: [arity_bits, final_poly_bits]; MinSize: [] or
 *       [max]), num_query_rounds
 *   FriParams (:151-157): FriConfig, hiding, degree_bits, [reduction_arity_bits]
 *   [Gate] (Gate/Base.hs:27-45): tag 0..16 in constructor order (Arithmetic, ArithmeticExtension,
 *       BaseSum, CosetInterpolation, Constant, Exponentiation, Lookup, LookupTable, MulExtension,
 *       Noop, PublicInput, Poseidon, PoseidonMds, RandomAccess, Reducing, ReducingExtension,
 *       Unknown) then its fields; KeccakHash = [Word8] as [u64]; UnknownGate's String as [byte]
 *   SelectorsInfo (:90-95): [selector_indices], [groups as (start, end)], Maybe [selector_vector]
 *   quotient_degree_factor, num_gate_constraints, num_constants, num_public_inputs, [k_is],
 *   num_partial_products, num_lookup_polys, num_lookup_selectors,
 *   [LookupTable] (each [(Word64, Word64)] as [inp, out] pairs)
 *   VerifierOnlyCircuitData (:236-240): constants_sigmas_cap, circuit_digest
 * ProofWithPublicInputs words = P2V_WORDS_PROOF_MAGIC, then
 *   Proof (:256-263): wires_cap, plonk_zs_partial_products_cap, quotient_polys_cap,
 *     OpeningSet (:265-276, field order): 9 x [FExt],
 *     FriProof (:176-181): [MerkleCap] commit caps, [FriQueryRound] (each: [([F], [Digest])]
 *       initial trees, [([FExt], [Digest])] steps), final_poly [FExt], pow_witness F
 *   public_inputs [F]
 * bindings/haskell/Plonk/VerifierGPU.hs writes exactly this; p2v.py circuit_words / proof_words
 * derive it from the JSON files (tests: words path == JSON path, bit for bit). */
#define P2V_WORDS_CIRCUIT_MAGIC 0x5032564300000001ULL   /* "P2VC", version 1 */
#define P2V_WORDS_PROOF_MAGIC   0x5032565000000001ULL   /* "P2VP", version 1 */

/* VerifierCircuitData from its word encoding (same validation and errors as
 * p2v_circuit_from_json).  Replaces: MkVerifierCircuitData of decoded values (Types.hs:220-224). */
int  p2v_circuit_from_words(const uint64_t* words, size_t n, p2v_circuit** out);
int  p2v_circuit_from_words_ex(const uint64_t* words, size_t n, uint32_t ext, p2v_circuit** out);
/* ProofWithPublicInputs from its word encoding into the circuit's packed layout (dst holds
 * info.proof_words u64); P2V_E_PARSE on a malformed encoding, P2V_E_SHAPE on list lengths the
 * circuit does not imply (as p2v_pack_proof_json). */
int  p2v_pack_proof_words(const p2v_circuit* c, const uint64_t* words, size_t n, uint64_t* dst);

/* ---- plonky2's binary proof serialization (not in the reference,
 * README.md:27) -----------------------------------------------------------------------
 * One ProofWithPublicInputs as plonky2's `to_bytes` writes it (Write::write_proof_with_public_inputs):
 * u64 little-endian words (F reduced mod p), caps as 2^cap_height hashes, Merkle proofs as a u8
 * sibling count then the hashes, the circuit-sized vectors without lengths, in the order
 * wires_cap, zs_pp_cap, quotient_cap, openings (constants, plonk_sigmas, wires, plonk_zs,
 * plonk_zs_next, lookup_zs, lookup_zs_next, partial_products, quotient_polys), commit caps, query
 * rounds (4 x (leaf, proof), steps x (evals, proof)), final_poly, pow_witness, then the public
 * inputs (the remaining words, or a u64 count and the words).  Packed into the circuit's layout as
 * p2v_pack_proof_json does; P2V_E_PARSE when truncated, P2V_E_SHAPE on a sibling count or public
 * input count the circuit does not imply.  Parity unpinned (no binary fixture offline). */
int  p2v_pack_proof_bytes(const p2v_circuit* c, const uint8_t* bytes, size_t n, uint64_t* dst);

/* ---- shape variants --------------------------------------------------------------------
 * The reference reads public_inputs and final_poly.coeffs at whatever length a proof carries:
 * the public inputs enter only through their sponge (Hash/Sponge.hs:26-31, Challenge/
 * Verifier.hs:68, Plonk/Vanishing.hs:86), the final polynomial through its absorb and its
 * evaluation (Challenge/FRI.hs:83, Plonk/FRI.hs:325-327).  A proof whose lengths differ from
 * the circuit's (num_public_inputs; 2^(degree_bits - sum arity_bits)) fails to pack with
 * P2V_E_SHAPE; p2v_proof_shape_* read its two lengths and p2v_circuit_shape_variant derives the
 * circuit whose packed layout has them (same circuit otherwise; free with p2v_circuit_free), so
 * the proof is verified on the GPU with the reference's outcome (False in practice: the
 * transcript diverges).  Limits: up to 2^20 public inputs / coefficients (else P2V_E_SHAPE).
 * Every other length mismatch is an `error` in the reference too and stays P2V_E_SHAPE. */
int  p2v_proof_shape_json(const char* proof_json, size_t len, int* num_public_inputs, int* final_poly_len);
int  p2v_proof_shape_words(const uint64_t* words, size_t n, int* num_public_inputs, int* final_poly_len);
int  p2v_circuit_shape_variant(const p2v_circuit* c, int num_public_inputs, int final_poly_len, p2v_circuit** out);

/* ---- verification (GPU) ------------------------------------------------------------ */
#define P2V_FLAG_INPUT_DEVICE  1u  /* `proofs` is a device pointer on the verifier's device  */
#define P2V_FLAG_RESULT_DEVICE 2u  /* `results` (and trace) are device pointers              */
#define P2V_FLAG_NO_SYNC       4u  /* do not synchronise the stream before returning          */
#define P2V_FLAG_INPUT_TILED  16u  /* `proofs` is in the 64-proof tiled layout below (p2v_tile_proofs) instead of
                                      proof-major: every wave's loads are then whole 512-B rows          */
#define P2V_FLAG_LOOKAHEAD    32u  /* with P2V_FLAG_INPUT_DEVICE: the batch is complete in device memory when the
                                       call is made (nothing queued on `stream` still writes it), so its transcript
                                       may run ahead of this workspace's earlier batches, on a stream of its own
                                       with a second challenge buffer, overlapping their Merkle / FRI work
                                       (DESIGN.md §5.2); results are unchanged.  A measurement build that
                                       transposes the batch (P2V_PROOF_MAJOR=0) rejects it with P2V_E_ARG   */
#define P2V_FLAG_UNIT_FILTERS  8u  /* parity mode: every gate filter and lookup selector := 1, so the
                                      trace's combined values C_i expose every constraint program
                                      (the oracle's or_verify full_trace bit 1); statuses are then
                                      meaningless.  Tests only. */

/* Tiled batch layout (P2V_FLAG_INPUT_TILED): word w of proof i at
 *   tiled[((i / 64) * proof_words + w) * 64 + i % 64],
 * i.e. ceil(n / 64) tiles of [proof_words][64]; a tile's rows past n are never read (lanes past n
 * re-read proof n - 1, as in the proof-major form).  The packed values are the same; only their
 * order differs, so a packer can write either.  p2v_tiled_words gives the buffer size in u64. */
size_t p2v_tiled_words(size_t n, size_t proof_words);
void   p2v_tile_proofs(const uint64_t* proof_major, size_t n, size_t proof_words, uint64_t* tiled);   /* host; pads with 0 */

int  p2v_device_count(void);

/* Create a verifier on `device` able to take batches up to max_batch proofs.  All device
 * memory is allocated here, none in p2v_verifier_run (graph-capturable). */
int  p2v_verifier_create(const p2v_circuit* c, int device, size_t max_batch, p2v_verifier** out);
void p2v_verifier_free(p2v_verifier* v);

/* Verify n packed proofs (n * proof_words u64, proof-major, each word a canonical field
 * element < p as p2v_pack_proof_json writes it).  results[i] gets the status of proof i.
 * trace (optional, may be NULL) receives n * trace_words u64 of intermediates for parity
 * checks.  stream: a hipStream_t cast to void* (NULL = the default stream).  A verifier is
 * one workspace: one run at a time per verifier (use one verifier per concurrent stream);
 * circuits are read-only and may be shared. */
int  p2v_verifier_run(p2v_verifier* v, const uint64_t* proofs, size_t n,
                      int8_t* results, uint64_t* trace, void* stream, uint32_t flags);

/* Stagger two or more workspaces that run back-to-back batches on their own streams: after
 * p2v_verifier_chain(v, prev), every later run of v starts its phase 1 (transcript + leaf
 * hashing) only once the phase 1 most recently enqueued on prev has finished (a device-side
 * event wait; the host never blocks).  Chaining two verifiers to each other alternates their
 * phase 1 with the other batch's Merkle / FRI / vanishing work instead of running both batches'
 * phases in lockstep.  prev = NULL removes the link.  Results are unaffected; v and prev must be
 * on the same device.  Freeing either verifier removes its links (the other side then runs
 * unchained); links and runs may be used from different host threads.  Not part of the
 * reference (a batching schedule). */
int  p2v_verifier_chain(p2v_verifier* v, p2v_verifier* prev);

/* Verify n proofs given as ProofWithPublicInputs JSON texts (Types.hs:245-279) in host memory:
 * proof i is blob[offsets[i] .. offsets[i+1]) (n + 1 offsets; pinned memory makes the copy
 * fastest).  The texts are copied to the device and packed there against a template taken
 * from the batch's first decodable proof (json_pack.hip); a proof that does not fit the
 * template is packed by the host reader instead, so the packed words and the decode codes
 * (codes[i]: P2V_OK / P2V_E_PARSE / P2V_E_SHAPE) are those of p2v_pack_proof_json.  Proofs
 * that do not decode get results[i] = P2V_ERR_PARSE / P2V_ERR_SHAPE.  Host results only.
 * n_device (optional, may be NULL) receives how many proofs the device packer took.
 * Replaces: decode + verifyProof per proof (Types.hs:245-254, Plonk/Verifier.hs:56-65). */
int  p2v_verifier_run_json(p2v_verifier* v, const char* blob, const uint64_t* offsets, size_t n,
                           int8_t* results, int32_t* codes, size_t* n_device, void* stream);

/* The packing half of p2v_verifier_run_json: the texts are packed on the device as there, and
 * the n * proof_words packed words copied to `words` (host memory; rows of proofs that do not
 * decode are zero).  Bit-identical to p2v_pack_proofs_json.
 * Replaces: decode :: ProofWithPublicInputs over a batch (Types.hs:245-254). */
int  p2v_verifier_pack_json(p2v_verifier* v, const char* blob, const uint64_t* offsets, size_t n,
                            int32_t* codes, size_t* n_device, uint64_t* words, void* stream);

/* plonky2 binary proofs on the GPU: proof i is blob[offsets[i] .. offsets[i+1]) in the format of
 * p2v_pack_proof_bytes.  For a given circuit that format is a fixed map of byte offsets, so the
 * texts are copied to the device and packed there by one workgroup per proof (json_pack.hip
 * k_bytes_pack); a proof that fails a length / sibling-count / public-input check is packed by the
 * host reader instead, so words and codes (P2V_OK / P2V_E_PARSE / P2V_E_SHAPE) always equal
 * p2v_pack_proof_bytes.  n_device (optional) receives how many proofs the device packed.  run:
 * then verified (results as p2v_verifier_run_json); pack: the packed words copied to `words`. */
int  p2v_verifier_run_bytes(p2v_verifier* v, const uint8_t* blob, const uint64_t* offsets, size_t n,
                            int8_t* results, int32_t* codes, size_t* n_device, void* stream);
int  p2v_verifier_pack_bytes(p2v_verifier* v, const uint8_t* blob, const uint64_t* offsets, size_t n,
                             int32_t* codes, size_t* n_device, uint64_t* words, void* stream);

/* One-shot form of verifyProof over a batch in host memory (proof-major packed rows), on `device`.
 * The circuit handle keeps the verifier it runs on (a pool per circuit and device, created on
 * first use, freed with the circuit), so a repeated call -- a drop-in verifyProof per proof --
 * costs the kernels and the copies, not a workspace.  Up to 64 proofs run as one latency-mode
 * launch; larger batches are verified in chunks (about n/8, 256..16384 proofs) whose H2D copies
 * run on a copy stream of their own, overlapped with the verification of the chunks before them
 * (three chunk buffers in flight).  Thread-safe: concurrent calls on one circuit use distinct
 * pooled verifiers.  Replaces: map (verifyProof vkey) (Plonk/Verifier.hs:56-65). */
int  p2v_verify_batch(const p2v_circuit* c, const uint64_t* proofs, size_t n,
                      int8_t* results, int device);

/* The same for plonky2 binary proofs (the p2v_pack_proof_bytes format): blob + offsets[n + 1] in
 * host memory (pinned for the full link rate).  Per chunk the bytes are copied on the copy stream,
 * packed on the device and verified, chunks overlapped as above; proofs the device packer does not
 * take are packed by the host reader and verified afterwards, so results / codes / n_device are
 * those of p2v_verifier_run_bytes.  chunk: proofs per chunk (0: automatic). */
int  p2v_verify_batch_bytes(const p2v_circuit* c, const uint8_t* blob, const uint64_t* offsets, size_t n,
                            int8_t* results, int32_t* codes, size_t* n_device, int device, size_t chunk);

/* Single-process multi-GPU form of p2v_verify_batch: the batch (host memory,
 * proof-major) is split into ndevices contiguous near-equal shards, shard i verified on
 * devices[i] (a device may repeat) by the circuit's pooled pipeline for that device, in chunks of
 * `chunk` proofs (0: automatic, as p2v_verify_batch) whose H2D copies overlap the verification of
 * the chunks before them.  One host thread per shard (none for a single shard).  Proofs are
 * independent, so there is no cross-device traffic.  On failure returns the first failing
 * shard's code and message.
 * Replaces: map (verifyProof vkey) over a batch (Plonk/Verifier.hs:56-65) on N GPUs. */
int  p2v_verify_batch_devices(const p2v_circuit* c, const uint64_t* proofs, size_t n, int8_t* results,
                              const int* devices, int ndevices, size_t chunk);

/* Self-test of the device primitives every verifier kernel is built from, on `device`
 * (host buffers; n items):
 *   op 0: out[i] = a[i] * b[i] mod p, canonical            (Algebra/Goldilocks.hs:126-133)
 *   op 3: the same through the Poseidon S-box's multiply form
 *   op 1: out[12i..] = Poseidon permutation of a[12i..]     (Hash/Poseidon.hs:42-46)
 *   op 2: out[12i..12i+4) = compress form: words 8..11 of a[12i..] taken as 0, words 0..3 of
 *         the permutation returned, the rest 0               (Hash/Merkle.hs:21-24)
 *   op 4: out[12i..] = M a[12i..] + (b[0..12) + 2^32 b[12..24)) mod p, not canonicalised: one MDS
 *         layer with the next round's constants as the permutation computes it (the row
 *         reduction's rare carry fix-up included; b, 24 words, shared by all items) (Poseidon.hs:100-101)
 *   ops 5-8: out[i] = a[i]^7 mod p, canonical, through each S-box form with its rare -2^64
 *         fix-up (Poseidon.hs:92-96): 5 the throughput permutation's (one S-box), 6 its grouped
 *         pair (a[i], b[i]) -> out[2i], out[2i+1], 7 the row form's, 8 the quad / pair forms'
 *   ops 9-11: out[12i..] = the Poseidon permutation of a[12i..] in the latency forms of the
 *         transcript and the small-batch Merkle paths: 9 row (16 lanes per state), 10 quad
 *         (4 lanes), 11 pair (2 lanes)                     (Hash/Poseidon.hs:42-46)
 * Inputs may be any u64 (values >= p are congruent, as the reference reads them).
 * Test hook for the parity suite (edge values the synthetic proofs never produce). */
int  p2v_selftest(int device, int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n);

/* Measurement helpers (bench.py; device pointers, enqueued on `stream`, no host sync):
 * p2v_count_mismatches: counters[0] += #{i < n : results[i] != expect[i]}, counters[1] += 1 --
 *   a device-side status check after each timed launch, so every timed batch is verified
 *   without a host round trip (counters: 2 u64 in device memory, zeroed by the caller).
 * p2v_clock_probe: nblocks one-wave workgroups; workgroup b writes (XCC id, s_memtime,
 *   s_memrealtime) to stamps[3b .. 3b+2].  Two probes around a timed pass give the shader clock
 *   the chip held over it per XCD: d(memtime) / d(memrealtime) x 100 MHz. */
int  p2v_count_mismatches(const int8_t* results, const int8_t* expect, size_t n, uint64_t* counters, void* stream);
int  p2v_clock_probe(uint64_t* stamps, int nblocks, void* stream);

/* Per-launch timing of the last run (milliseconds, from HIP events on the run's stream):
 * out[k] for kernel k in the order named by p2v_kernel_names(). Returns count. */
int  p2v_verifier_last_timings(const p2v_verifier* v, float* out, int max);
const char* p2v_kernel_names(void);   /* comma-separated */

const char* p2v_last_error_message(void);
const char* p2v_version(void);

#ifdef __cplusplus
}
#endif

/* ---- debug trace layout (u64 words per proof), shared by the oracle --------------
 *   off_pi_hash      4
 *   off_betas        r          off_gammas   r          off_alphas  r
 *   off_deltas       4r   (zero when the circuit has no lookups)
 *   off_zeta         2          off_fri_alpha 2
 *   off_fri_betas    2S         off_pow_response 1       off_query_idx Q
 *   off_combined     2r   C_i(zeta) after alpha-combination  Plonk/Vanishing.hs:48-56
 *   off_quotient     2r   sum_k zeta^(nk) q_{i,k}            Plonk/Verifier.hs:43-47
 *   off_q_initial    2Q   combineInitial per query          Plonk/FRI.hs:151-207
 *   off_q_folded     2Q   value after the last folding step Plonk/FRI.hs:306-323
 *   off_q_final      2Q   final polynomial at x_final       Plonk/FRI.hs:325-327
 *   off_flags        1    bit0 eqs_ok, bit1 pow_ok
 *   off_lut_re       rL   evalFinalRE of table k in challenge round i at [i*L + k]
 *                         (L = #luts)                       Plonk/Lookups.hs:103-109
 * total = 4 + 3r + 4r + 4 + 2S + 1 + Q + 4r + 6Q + 1 + rL
 */
#define P2V_TRACE_WORDS(r, S, Q, L) (4 + 3*(r) + 4*(r) + 4 + 2*(S) + 1 + (Q) + 4*(r) + 6*(Q) + 1 + (r)*(L))

#endif /* P2V_H */
