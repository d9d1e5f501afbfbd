// dev.h — POD circuit descriptor passed by value to every kernel, plus the device-side
// scratch layout.  All proofs of a batch share one circuit, so every shape below is
// wave-uniform; the lane index is the proof index (SoA layout [word][B]).
#pragma once
#include <stdint.h>

#define P2V_MAX_STEPS 8
#define P2V_MAX_R 4
#define P2V_LUT_CHUNK 16   // baby steps of the LUT evaluation
#define P2V_LUT_PIECE 256  // chunks per k_lut work unit (4096 table entries)

struct DevCircuit {
  int32_t B;            // lane stride (batch padded to a multiple of 64)
  int32_t n;            // proofs in this run
  int32_t r, Q, S, T;   // challenges, queries, FRI steps, trees per query (4 + S)
  int32_t num_pis, cap_len, degree_bits, lde_bits, pow_bits;
  int32_t num_wires, num_routed, num_constants, ngc, ngroups, nls, nlp, npp, qdf, nluts;
  int32_t depth0, final_len;
  int32_t arity[P2V_MAX_STEPS], step_depth[P2V_MAX_STEPS], step_logn[P2V_MAX_STEPS];
  int32_t width[4];                // data columns per initial oracle (combineInitial)
  int32_t lwidth[4];               // packed leaf words (width + salts under P2V_EXT_HIDING): the sponged row
  int32_t noop_leaves;             // P2V_EXT_HASH_OR_NOOP: a leaf of <= 4 words is its own digest
  int32_t tiled;                   // P2V_FLAG_INPUT_TILED: the batch is [n/64][words][64] (devcommon.h ld())
  int64_t wstride;                 // distance between a proof's consecutive words: 64 tiled, else 1
  // tree t of each unit position, most expensive first, so long waves dispatch first and short
  // ones fill the tail: leaf hashing by sponge length, Merkle paths by depth
  int8_t leaf_order[4 + P2V_MAX_STEPS], merkle_order[4 + P2V_MAX_STEPS];
  int32_t n_gates;                 // gates evaluated = min(#selector_indices, #gates)
  int32_t unit_filters;            // P2V_FLAG_UNIT_FILTERS (parity mode)
  int32_t n_pp_terms, n_lookup_terms;
  int64_t alpha_base_gates;
  // packed layout (u64 word offsets)
  int64_t pis, wcap, zcap, qcap, o_const, o_sig, o_wires, o_zs, o_pp, o_quot, o_lzs, o_zs_next, o_lzs_next;
  int64_t n_this, n_next, ccaps, final_poly, pow, q0, qstride;
  int64_t leaf[4], path[4], step_evals[P2V_MAX_STEPS], step_path[P2V_MAX_STEPS];
  int64_t words;
  // small constant tables
  uint64_t digest[4];
  uint64_t root_pow2[33];          // TWO_ADIC_GEN^(2^m): subgroup_gen(k)^(2^j) = root_pow2[32-k+j]
  uint64_t step_shift[P2V_MAX_STEPS + 1];     // MULT_GEN^(prod of earlier arities)
  uint64_t step_shift_inv[P2V_MAX_STEPS + 1];
  uint64_t inv_arity[P2V_MAX_STEPS];          // 1 / 2^arity
  // device tables
  const uint64_t* cs_cap;          // [cap_len][4]
  const uint64_t* k_is;            // [num_routed]
  const int32_t* gate_kind;        // [n_gates]
  const int64_t* gate_par;         // [n_gates][3]
  const int32_t* gate_grp;         // [n_gates] selector group
  const int32_t* gate_woff;        // [n_gates] offset into weights
  const uint64_t* weights;         // CosetInterpolation barycentric weights
  const int32_t* grp_start;        // [ngroups]
  const int32_t* grp_end;
  const uint64_t* lut_in;          // concatenated LUTs
  const uint64_t* lut_out;
  const int64_t* lut_off;          // [nluts]
  const int64_t* lut_len;
  // evalFinalRE fast path (Lookups.hs:103-109): per LUT the padded entry sequence reversed
  // (coefficient of delta^t) and zero-filled to P2V_LUT_CHUNK, as u32; lut_rchunks[k] = 0 when
  // an entry is >= 2^24 (then the per-entry Horner over lut_in/lut_out is used)
  const uint32_t* lut_rin;
  const uint32_t* lut_rout;
  const int64_t* lut_roff;         // [nluts]
  const int32_t* lut_rchunks;      // [nluts]
  const int32_t* lut_pbase;        // [nluts + 1] first k_lut piece of each table
  int32_t n_lut_pieces;
  const uint64_t* twiddles;        // per step: omega_{a}^{-j}, j < 2^a  (offset 256*s)
  const int32_t* tops;             // transcript op program [ntops][3] (see TOP_*)
  int32_t ntops;
  const int32_t* vitems;           // vanishing work items [n_vitems][4] = {VI_*, a, b, first term}
  int32_t n_vitems;
  int32_t vcls[5];                 // item ranges of the vanishing kernel classes (Poseidon, coset, misc, lookup)
  const uint64_t* pos_w;           // PoseidonGate part 3: W = A'M [12][12] then k = A' rc [12] (vanish_poseidon.hip)
  // batch buffers
  const uint64_t* soa;             // [words][B]
  uint64_t* chal;                  // [CH_WORDS][B]
  uint64_t* leafdig;               // [Q][T][4][B]
  uint8_t* mk_ok;                  // [Q][T][B]
  uint32_t* fri_bits;              // [Q][B]: bit s = step-s evaluation check, bit 31 = final check
  uint64_t* qvals;                 // [Q][6][B]: initial, folded, final (F^2 each)
  uint64_t* van;                   // [1 + 4r][B]: eqs_ok, C_i, quotient_i
  uint64_t* vparts;                // [n_vitems][2r][B]: per-item partial alpha-sums
  uint64_t* lutre;                 // [r][nluts][B]: evalFinalRE values (debug trace)
  uint64_t* lutpart;               // [r][n_lut_pieces][B]: k_lut partial sums
  // Merkle paths with every shared node hashed once (kernels.hip k_merkle_plan / k_merkle_cse /
  // k_merkle_fix / k_merkle_resolve; mcse = 0: k_merkle, one full path per lane)
  int32_t mcse;
  int64_t mcap;                    // chains per bucket (T * Q * Bmax)
  uint32_t* mplan;                 // [1 + S][Q][B]: e | owner << 4 | same_leaf << 9 | root << 10
  uint64_t* mfol;                  // [1 + S][Q][B]: per owned level l, bits 5l..5l+4: the follower (31: none)
  uint32_t* mchain;                // [depth0 + 1][mcap]: chain ids t << 27 | q << 22 | p, bucket = chain length
  int32_t* mcount;                 // [depth0 + 1] x 16: chains per bucket, 64 B apart (k_merkle_resolve zeroes them)
  int32_t* mfixn;                  // flagged followers listed in mfix (k_merkle_resolve zeroes it)
  uint32_t* mfix;                  // [mcap]: chain ids of the followers k_merkle_fix re-runs
  uint8_t* mbadq;                  // [T][Q][B]: the follower failed a shared-node check
  uint64_t* mnode;                 // [T][Q][4][B]: a follower's node at its meeting level
};
#define P2V_CSE_MAX_DEPTH 12       // 5-bit follower fields of one u64 per owned level
#define P2V_CSE_MAX_Q 31           // 5-bit query ids, 31 = none
#define P2V_CSE_MAX_B (1 << 22)    // 22-bit proof index in a chain id

// transcript op program (built on the host from the circuit; uniform across the batch)
#define TOP_ABSORB_SOA 0    // absorb n words of the proof (SoA) from word a
#define TOP_ABSORB_PIH 1    // absorb the 4-word public-inputs hash
#define TOP_ABSORB_DIGEST 2 // absorb the circuit digest (n = 4)
#define TOP_SQUEEZE 3       // squeeze n words into challenge words a..
#define TOP_SQUEEZE_IDX 4   // squeeze n query indices (mod 2^lde_bits) into a..
#define TOP_COPY 5          // challenge words a..a+n = words a-3r..  (lookup deltas := betas ++ gammas)
#define TOP_ZERO 6          // challenge words a..a+n = 0

// vanishing work items (host-built list; each is a contiguous run of the alpha-combined
// term sequence, evaluated by one wave per 64 proofs)
#define VI_ZS1 0      // the r Z(1) boundary terms
#define VI_PP 1       // partial-product terms of challenge round a
#define VI_LOOKUP 2   // lookup terms of challenge round a
#define VI_GATE 3     // gate a, part b (PoseidonGate: 8 parts, others: 1)
#define P2V_POSEIDON_PARTS 8
// first term (in the gate's own numbering) of PoseidonGate part k (see vanish.hip)
static inline constexpr int p2v_poseidon_part_first_term(int part) {
  return part == 0 ? 0 : part <= 2 ? 17 + 12 * (part - 1) : part == 3 ? 41 : 75 + 12 * (part - 4);
}

// CosetInterpolationGate (Gate/Custom/CosetInterp.hs:51-121): its chunks start from the witness's
// intermediate evaluation / product wires, so each chunk is an independent vanishing item (part);
// the number of chunks the reference evaluates (zipWith worker initials chunks) and the first term
// of part k in the gate's own numbering (eval_loc: terms 0-1; chunk k < last: 4 terms from 2 + 4k;
// the last chunk's eval_result term after them)
#if defined(__HIPCC__)
#define P2V_HD __host__ __device__
#else
#define P2V_HD
#endif
static inline P2V_HD int64_t p2v_coset_parts(int bits, int64_t degree, int64_t nweights) {
  const int64_t npts = (int64_t)1 << bits;
  const int64_t nint = (npts - 2) / (degree - 1);
  const int64_t first = degree < npts ? degree : npts;
  const int64_t nchunks_v = 1 + (npts - first + (degree - 2)) / (degree - 1);
  const int64_t wfirst = degree < nweights ? degree : nweights;
  const int64_t nchunks_w = 1 + (nweights - wfirst + (degree - 2)) / (degree - 1);
  const int64_t nch = nchunks_v < nchunks_w ? nchunks_v : nchunks_w;
  return nint + 1 < nch ? nint + 1 : nch;
}
static inline P2V_HD int64_t p2v_coset_part_first_term(int64_t part) { return part == 0 ? 0 : 2 + 4 * part; }

// challenge buffer offsets (match the P2V_TRACE layout prefix in include/p2v.h)
#define CH_PI(c) 0
#define CH_BETA(c) 4
#define CH_GAMMA(c) (4 + (c).r)
#define CH_ALPHA(c) (4 + 2 * (c).r)
#define CH_DELTA(c) (4 + 3 * (c).r)
#define CH_ZETA(c) (4 + 7 * (c).r)
#define CH_FRI_ALPHA(c) (CH_ZETA(c) + 2)
#define CH_FRI_BETA(c) (CH_FRI_ALPHA(c) + 2)
#define CH_POW(c) (CH_FRI_BETA(c) + 2 * (c).S)
#define CH_QIDX(c) (CH_POW(c) + 1)
#define CH_Y0(c) (CH_QIDX(c) + (c).Q)
#define CH_Y1(c) (CH_Y0(c) + 2)
#define CH_WORDS(c) (CH_Y1(c) + 2)
