// api.cpp — the C-ABI of libp2v (include/p2v.h): the drop-in boundary for
// verifyProof :: VerifierCircuitData -> ProofWithPublicInputs -> Bool
// (reference src/Plonk/Verifier.hs:56-65), batched, on MI355X.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include "../../include/p2v.h"
#include "circuit.hpp"
#include "dev.h"
#ifndef P2V_PROOF_MAJOR
#define P2V_PROOF_MAJOR 1   // see devcommon.h ld()
#endif
#include "gl.h"
#include "poseidon_constants.h"

extern "C" __global__ void k_transpose(const uint64_t*, int64_t, int, uint64_t*, int);
extern "C" __global__ void k_phase1(DevCircuit, int, int);
extern "C" __global__ void k_phase1_lane(DevCircuit, int, int);
extern "C" __global__ void k_phase1_pair(DevCircuit, int, int);
extern "C" __global__ void k_transcript(DevCircuit, int);
extern "C" __global__ void k_transcript_lane(DevCircuit, int);
extern "C" __global__ void k_transcript_pair(DevCircuit, int);
extern "C" __global__ void k_transcript_x(DevCircuit, int);
extern "C" __global__ void k_leaf(DevCircuit);
extern "C" __global__ void k_merkle(DevCircuit);
extern "C" __global__ void k_merkle_row(DevCircuit);
extern "C" __global__ void k_merkle_plan(DevCircuit);
extern "C" __global__ void k_merkle_cse(DevCircuit);
extern "C" __global__ void k_merkle_fix(DevCircuit);
#ifndef P2V_PLAN_WAVES
#define P2V_PLAN_WAVES 16   // as kernels.hip
#endif
#ifndef P2V_FIX_BLOCKS
#define P2V_FIX_BLOCKS 256   // k_merkle_fix grid: its blocks wait for free slots beside the other batch's kernels
#endif
extern "C" __global__ void k_merkle_resolve(DevCircuit);
extern "C" __global__ void k_fri(DevCircuit);
extern "C" __global__ void k_vanish_r2(DevCircuit);
extern "C" __global__ void k_vanish_rn(DevCircuit);
extern "C" __global__ void k_vanish_poseidon_r2(DevCircuit);
extern "C" __global__ void k_vanish_poseidon_rn(DevCircuit);
extern "C" __global__ void k_vanish_coset_r2(DevCircuit);
extern "C" __global__ void k_vanish_coset_rn(DevCircuit);
extern "C" __global__ void k_vanish_lookup_r2(DevCircuit);
extern "C" __global__ void k_vanish_lookup_rn(DevCircuit);
extern "C" __global__ void k_lut(DevCircuit);
extern "C" __global__ void k_vanish_final(DevCircuit);
extern "C" __global__ void k_status(DevCircuit, int8_t*, uint64_t*, int64_t);
extern "C" __global__ void k_selftest(int, const uint64_t*, const uint64_t*, uint64_t*, int64_t);
extern "C" __global__ void k_selftest_forms(int, const uint64_t*, uint64_t*, int64_t);
extern "C" __global__ void k_count_mismatches(const int8_t*, const int8_t*, int64_t, unsigned long long*);
extern "C" __global__ void k_clock_probe(unsigned long long*);
extern "C" __global__ void k_json_pack(const uint8_t*, const uint64_t*, int, const uint8_t*, int64_t, const int32_t*, int64_t, uint64_t*, int64_t, int8_t*);
extern "C" __global__ void k_bytes_pack(const uint8_t*, const uint64_t*, int, const int64_t*, const int64_t*, const int64_t*, int,
                                        const int64_t*, const uint8_t*, int, int64_t, int64_t, int64_t, uint64_t*, int64_t, int8_t*);

using namespace p2v;

namespace {
thread_local std::string g_err;
int fail(int code, const std::string& msg) { g_err = msg; return code; }

// per-kernel timing slots; k_fri and k_vanish run on the side stream, concurrently with k_merkle
// (k_leaf + k_transcript: the split form of k_phase1, env P2V_PHASE1=split, measurement only)
const char* kKernelNames = "k_transpose,k_phase1,k_merkle,k_fri,k_vanish,k_status,k_vanish_final,k_lut,k_leaf,k_transcript";
constexpr int kNumKernels = 10;

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  hipError_t alloc(size_t n) { bytes = n; return hipMalloc(&p, n ? n : 16); }
  void free_() { if (p) (void)hipFree(p); p = nullptr; }
};
}  // namespace

struct HostPipe;
// The circuit handle also owns the verifiers the one-shot entry points (p2v_verify_batch,
// p2v_verify_batch_devices) run on, kept across calls (a drop-in verifyProof
// call must not re-create workspaces, streams and events).  Read-only for the circuit itself.
struct p2v_circuit {
  Circuit c;
  mutable std::mutex pool_mu;
  mutable std::vector<HostPipe*> pool;   // idle and busy pipes of every device
  ~p2v_circuit();
};

namespace {
template <class T>
hipError_t upload(DevBuf& b, const std::vector<T>& h) {
  hipError_t e = b.alloc(h.size() * sizeof(T));
  if (e != hipSuccess) return e;
  if (!h.empty()) e = hipMemcpy(b.p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice);
  return e;
}

std::mutex g_chain_mu;   // p2v_verifier_chain links (chain_prev / chain_next of every verifier)

// PoseidonGate part 3 (vanish_poseidon.hip): the state entering the fast partial rounds is
// A'(M sb + rc) (Gate/Custom/Poseidon.hs:92-104: mdsLayer, + fastPartialFirstConstant,
// mdsInitPartial with A' = diag(1, A), A[i][j] = INITIAL_MATRIX[j][i]); as one affine map of the
// S-box outputs sb: W = A'M (12 x 12) and k = A' rc, mod p.  Returns [W row-major | k].
std::vector<uint64_t> poseidon_part3_table() {
  static const uint64_t init[121] = P2V_FAST_PARTIAL_ROUND_INITIAL_MATRIX_INIT;
  static const uint64_t rc[12] = P2V_FAST_PARTIAL_FIRST_ROUND_CONSTANT_INIT;
  static const uint32_t circ[12] = {17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20};
  auto M = [&](int i, int j) -> uint64_t { return circ[((j - i) % 12 + 12) % 12] + (i == 0 && j == 0 ? 8 : 0); };
  auto Ap = [&](int i, int l) -> uint64_t {   // A'[i][l]
    if (i == 0 || l == 0) return (i == l) ? 1 : 0;
    return init[11 * (l - 1) + (i - 1)];
  };
  std::vector<uint64_t> t(156, 0);
  for (int i = 0; i < 12; i++) {
    for (int j = 0; j < 12; j++) {
      uint64_t acc = 0;
      for (int l = 0; l < 12; l++) acc = gl::add(acc, gl::mul(Ap(i, l), M(l, j)));
      t[12 * i + j] = acc;
    }
    uint64_t acc = 0;
    for (int l = 0; l < 12; l++) acc = gl::add(acc, gl::mul(Ap(i, l), rc[l] % gl::P));
    t[144 + i] = acc;
  }
  return t;
}

}  // namespace


struct p2v_verifier {
  const p2v_circuit* circ = nullptr;
  int device = 0;
  size_t max_batch = 0, Bmax = 0;
  DevCircuit dc{};
  std::vector<DevBuf> bufs;
  size_t in_bytes = 0;              // the host-input staging buffer `in`, allocated by the first run that needs it
                                    // (device-resident batches never do: a 131 072-proof workspace saves 16.6 GB)
  DevBuf in, soa, chal, leafdig, mk, fbits, qvals, van, vparts, lutre, lutpart, res, trace;
  DevBuf m_plan, m_fol, m_chain, m_count, m_fix, m_badq, m_node;   // shared-node Merkle paths (dev.h mcse)
  DevBuf t_cs, t_kis, t_gkind, t_gpar, t_ggrp, t_gwoff, t_w, t_gs, t_ge, t_lin, t_lout, t_loff, t_llen, t_tw, t_ops, t_vit, t_rin, t_rout, t_roff, t_rch, t_pbase, t_pw;
  hipEvent_t ev[2 * kNumKernels];   // start/end per kernel
  hipEvent_t dep_p1 = nullptr, dep_side = nullptr, dep_tr = nullptr;
  hipEvent_t p1_done = nullptr;      // recorded on the caller's stream after phase 1 (p2v_verifier_chain)
  std::atomic<bool> p1_recorded{false};   // read by the workspaces chained to this one, from their host threads
  p2v_verifier* chain_prev = nullptr;     // chain links: guarded by g_chain_mu
  std::vector<p2v_verifier*> chain_next;  // workspaces whose chain_prev is this one (cleared when this one is freed)
  hipStream_t side = nullptr;
  hipStream_t side2 = nullptr;      // small batches: k_fri beside the vanishing kernels (latency mode)
  hipEvent_t dep_fri = nullptr;
  // transcript lookahead (P2V_FLAG_LOOKAHEAD): its own stream, two challenge buffers used by
  // alternate runs; tr_done[s]: the transcript into buffer s is complete, chal_free[s]: the run
  // that read buffer s has completed (k_status)
  hipStream_t ts = nullptr;
  hipStream_t side3 = nullptr;      // latency mode: the coset / misc vanishing kernels beside the Poseidon parts
  hipEvent_t dep_v3 = nullptr;
  hipEvent_t tr_done[2] = {nullptr, nullptr}, chal_free[2] = {nullptr, nullptr};
  DevBuf chal2;
  unsigned la_seq = 0;
  float last_ms[kNumKernels] = {0};
  bool timed = false;
  bool fri_first = false;           // side stream order: k_fri before the vanishing kernels (env P2V_FRI_FIRST=1)
  int transcript_mode = 0;          // 0 auto, 1 row, 2 quad, 3 lane, 4 pair (env P2V_TRANSCRIPT)
  int quad_min_batch = 4096;        // auto: quad form from this batch size on (env P2V_QUAD_MIN); round 5: with the
                                    // latency row form (lposeidon.h) the row transcript wins up to 2048 proofs
                                    // (2048: 2.40 against 2.98 ms serial, 1.084 against 1.077 M proofs/s at two in
                                    // flight; 4096: the same serial, 1.13 against 1.225 M; profiles/r05h_*)
  int lane_min_batch = 16384;       // auto: lane form from this batch size on (env P2V_LANE_MIN)
  bool merkle_cse = true;           // shared Merkle nodes hashed once (env P2V_MERKLE_CSE=0: one full path per lane)
  bool cse_dirty = false;           // a run enqueued k_merkle_plan but not k_merkle_resolve
  int lat_max_batch = 64;           // latency mode (row-form Merkle paths, k_fri on its own stream) up to this
                                    // batch size (env P2V_LAT_MAX, measurement)
  bool single_stream = false;       // env P2V_SINGLE_STREAM=1: no side stream (measurement)
  int side_prio = 0;                // env P2V_SIDE_PRIO=1: side stream at the device's highest priority (measured: no effect)
  int side_wg = 256;                // env P2V_SIDE_WG=64: one-wave groups for k_fri / k_vanish_final on the side stream
                                    // (measured 1.119-1.121 M against 1.128-1.130 M, profiles/r03l_side_wg.txt)
  int split_phase1 = 0;             // env P2V_PHASE1=split (1): k_transcript (side stream) + k_leaf instead of k_phase1.
                                    // Measured (profiles/r02_phase1_split.txt): serial 0.94x, pipelined 1.00x; the
                                    // transcript waves, latency-bound, stretch to 2.9 ms beside k_leaf.
                                    // P2V_PHASE1=excl (2): k_transcript_x (main stream, a SIMD per wave) + k_leaf (side)
  bool debug_sync = false;          // env P2V_DEBUG_SYNC=1: name each launch on stderr and synchronise after it (fault isolation)
  // JSON ingest on the device (p2v_verifier_run_json): the current template and its device
  // form, and buffers grown on demand
  ProofTemplate tmpl;
  bool have_tmpl = false;
  int64_t skel_len = 0, ntok = 0;
  DevBuf j_blob, j_offs, j_skel, j_tok, j_ok;
  // binary-proof ingest (p2v_verifier_run_bytes): the circuit's byte map on the device, made once
  DevBuf b_rsrc, b_rdst, b_rlen, b_coff, b_cval;
  bool have_bmap = false;
  int nruns = 0, nchk = 0;
  int64_t bfixed = 0;
  // pinned host staging for the small device->host results (statuses, JSON ok flags): a copy
  // to pageable memory would stage through the runtime and stall the other streams' work
  int8_t* h_res = nullptr;
};

// One device's pipeline for batches in host memory (p2v_verify_batch / _devices): a verifier, a
// compute stream and a copy stream, and a ring of kRing device chunk buffers, so chunk i+1's H2D
// copy (copy stream) overlaps chunk i's verification (compute stream) and up to kRing chunks are in
// flight.  Owned by the circuit's pool, reused across calls.
struct HostPipe {
  static constexpr int kRing = 3;
  int device = -1;
  size_t cap = 0;                 // the verifier's max_batch = the largest chunk
  p2v_verifier* v = nullptr;
  hipStream_t st = nullptr, cs = nullptr;
  DevBuf ring[kRing];
  hipEvent_t copied[kRing] = {}, freed[kRing] = {};
  bool have_ring = false;
  DevBuf dres;                    // device statuses of the whole call (grown on demand)
  int8_t* h_res = nullptr;        // pinned staging for them
  size_t h_res_cap = 0;
  // binary-proof ingest (p2v_verify_batch_bytes): per ring slot the chunk's bytes and offsets on
  // the device, the offsets' host copy (rewritten once the slot's previous copy is done), and the
  // device packer's ok flags of the whole call
  DevBuf bbytes[kRing], boffs[kRing], dok;
  std::vector<uint64_t> hoffs[kRing];
  int8_t* h_ok = nullptr;
  size_t h_ok_cap = 0;
  bool busy = false;
};

namespace {
void pipe_free(HostPipe* p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  if (p->st) (void)hipStreamSynchronize(p->st);
  if (p->cs) (void)hipStreamSynchronize(p->cs);
  for (int k = 0; k < HostPipe::kRing; k++) {
    p->ring[k].free_();
    if (p->copied[k]) (void)hipEventDestroy(p->copied[k]);
    if (p->freed[k]) (void)hipEventDestroy(p->freed[k]);
  }
  p->dres.free_();
  p->dok.free_();
  for (int k = 0; k < HostPipe::kRing; k++) { p->bbytes[k].free_(); p->boffs[k].free_(); }
  if (p->h_res) (void)hipHostFree(p->h_res);
  if (p->h_ok) (void)hipHostFree(p->h_ok);
  if (p->st) (void)hipStreamDestroy(p->st);
  if (p->cs) (void)hipStreamDestroy(p->cs);
  p2v_verifier_free(p->v);
  delete p;
}
constexpr int kPoolIdleMax = 4;   // idle pipes kept per (circuit, device)
}  // namespace

p2v_circuit::~p2v_circuit() {
  for (HostPipe* p : pool) pipe_free(p);
}

extern "C" {

const char* p2v_last_error_message(void) { return g_err.c_str(); }
const char* p2v_kernel_names(void) { return kKernelNames; }

int p2v_circuit_from_json(const char* common_json, size_t common_len, const char* vkey_json, size_t vkey_len, p2v_circuit** out) {
  return p2v_circuit_from_json_ex(common_json, common_len, vkey_json, vkey_len, 0, out);
}

int p2v_circuit_from_json_ex(const char* common_json, size_t common_len, const char* vkey_json, size_t vkey_len, uint32_t ext,
                             p2v_circuit** out) {
  if (!common_json || !vkey_json || !out) return fail(P2V_E_ARG, "null argument");
  if (ext & ~P2V_EXT_PLONKY2) return fail(P2V_E_ARG, "unknown P2V_EXT_* flag");
  try {
    JVal cj = parse_json(common_json, common_len);
    JVal vj = parse_json(vkey_json, vkey_len);
    auto* pc = new p2v_circuit();
    try { pc->c = parse_circuit(cj, vj, ext); } catch (...) { delete pc; throw; }
    *out = pc;
    return P2V_OK;
  } catch (const ParseError& e) { return fail(P2V_E_PARSE, e.what()); }
  catch (const CircuitError& e) { return fail(P2V_E_CIRCUIT, e.what()); }
  catch (const std::exception& e) { return fail(P2V_E_PARSE, e.what()); }
}

int p2v_circuit_from_words(const uint64_t* words, size_t n, p2v_circuit** out) {
  return p2v_circuit_from_words_ex(words, n, 0, out);
}

int p2v_circuit_from_words_ex(const uint64_t* words, size_t n, uint32_t ext, p2v_circuit** out) {
  if (!words || !out) return fail(P2V_E_ARG, "null argument");
  if (ext & ~P2V_EXT_PLONKY2) return fail(P2V_E_ARG, "unknown P2V_EXT_* flag");
  try {
    auto* pc = new p2v_circuit();
    try { pc->c = parse_circuit_words(words, n, ext); } catch (...) { delete pc; throw; }
    *out = pc;
    return P2V_OK;
  } catch (const ParseError& e) { return fail(P2V_E_PARSE, e.what()); }
  catch (const CircuitError& e) { return fail(P2V_E_CIRCUIT, e.what()); }
  catch (const std::exception& e) { return fail(P2V_E_PARSE, e.what()); }
}

int p2v_pack_proof_words(const p2v_circuit* pc, const uint64_t* words, size_t n, uint64_t* dst) {
  if (!pc || !words || !dst) return fail(P2V_E_ARG, "null argument");
  try {
    pack_proof_words(pc->c, words, n, dst);
    return P2V_OK;
  } catch (const ShapeError& e) { return fail(P2V_E_SHAPE, e.what()); }
  catch (const ParseError& e) { return fail(P2V_E_PARSE, e.what()); }
  catch (const std::exception& e) { return fail(P2V_E_PARSE, e.what()); }
}

int p2v_pack_proof_bytes(const p2v_circuit* pc, const uint8_t* bytes, size_t n, uint64_t* dst) {
  if (!pc || !bytes || !dst) return fail(P2V_E_ARG, "null argument");
  try {
    pack_proof_bytes(pc->c, bytes, n, dst);
    return P2V_OK;
  } catch (const ShapeError& e) { return fail(P2V_E_SHAPE, e.what()); }
  catch (const ParseError& e) { return fail(P2V_E_PARSE, e.what()); }
  catch (const std::exception& e) { return fail(P2V_E_PARSE, e.what()); }
}

void p2v_circuit_free(p2v_circuit* c) { delete c; }

int p2v_circuit_get_info(const p2v_circuit* pc, p2v_circuit_info* info) {
  if (!pc || !info) return fail(P2V_E_ARG, "null argument");
  const Circuit& c = pc->c;
  memset(info, 0, sizeof *info);
  info->degree_bits = c.degree_bits; info->lde_bits = c.lde_bits; info->cap_height = c.cap_height;
  info->num_challenges = c.r; info->num_query_rounds = c.num_queries; info->num_fri_steps = (int)c.arities.size();
  info->final_poly_len = c.final_len; info->num_public_inputs = c.num_pis;
  info->num_openings_this = (int)c.L.n_this; info->num_openings_next = (int)c.L.n_next;
  info->has_lookups = c.lut_in.empty() ? 0 : 1; info->num_gates = (int)c.gates.size();
  info->proof_words = c.L.words; info->trace_words = c.trace_words;
  for (int t = 0; t < 4; t++) { info->oracle_widths[t] = c.oracle_width[t]; info->leaf_widths[t] = c.leaf_width[t]; }
  info->ext = c.ext;
  for (size_t s = 0; s < c.arities.size() && s < 8; s++) info->step_arity_bits[s] = c.arities[s];
  return P2V_OK;
}

int p2v_pack_proof_json(const p2v_circuit* pc, const char* proof_json, size_t len, uint64_t* dst) {
  if (!pc || !proof_json || !dst) return fail(P2V_E_ARG, "null argument");
  try {
    JVal pj = parse_json(proof_json, len);
    pack_proof(pc->c, pj, dst);
    return P2V_OK;
  } catch (const ShapeError& e) { return fail(P2V_E_SHAPE, e.what()); }
  catch (const ParseError& e) { return fail(P2V_E_PARSE, e.what()); }
  catch (const std::exception& e) { return fail(P2V_E_PARSE, e.what()); }
}

int p2v_proof_shape_json(const char* proof_json, size_t len, int* num_public_inputs, int* final_poly_len) {
  if (!proof_json || !num_public_inputs || !final_poly_len) return fail(P2V_E_ARG, "null argument");
  try {
    proof_shape_json(parse_json(proof_json, len), *num_public_inputs, *final_poly_len);
    return P2V_OK;
  } catch (const std::exception& e) { return fail(P2V_E_PARSE, e.what()); }
}

int p2v_proof_shape_words(const uint64_t* words, size_t n, int* num_public_inputs, int* final_poly_len) {
  if (!words || !num_public_inputs || !final_poly_len) return fail(P2V_E_ARG, "null argument");
  try {
    proof_shape_words(words, n, *num_public_inputs, *final_poly_len);
    return P2V_OK;
  } catch (const std::exception& e) { return fail(P2V_E_PARSE, e.what()); }
}

int p2v_circuit_shape_variant(const p2v_circuit* pc, int num_public_inputs, int final_poly_len, p2v_circuit** out) {
  if (!pc || !out) return fail(P2V_E_ARG, "null argument");
  *out = nullptr;
  try {
    auto* v = new p2v_circuit();
    v->c = circuit_shape_variant(pc->c, num_public_inputs, final_poly_len);
    *out = v;
    return P2V_OK;
  } catch (const CircuitError& e) { return fail(P2V_E_SHAPE, e.what()); }
  catch (const std::exception& e) { return fail(P2V_E_SHAPE, e.what()); }
}

int p2v_pack_proofs_json(const p2v_circuit* pc, const char* const* jsons, const size_t* lens, size_t n, uint64_t* dst,
                         int32_t* codes, int threads) {
  if (!pc || (n && (!jsons || !lens || !dst || !codes))) return fail(P2V_E_ARG, "null argument");
  if (n == 0) return 0;
  const Circuit& C = pc->c;
  const int64_t W = C.L.words;
  auto dom_pack = [&](size_t i, std::string* msg) -> int32_t {
    try {
      JVal pj = parse_json(jsons[i], lens[i]);
      pack_proof(C, pj, dst + (size_t)W * i);
      return P2V_OK;
    } catch (const ShapeError& e) { if (msg) *msg = e.what(); return P2V_E_SHAPE; }
    catch (const ParseError& e) { if (msg) *msg = e.what(); return P2V_E_PARSE; }
    catch (const std::exception& e) { if (msg) *msg = e.what(); return P2V_E_PARSE; }
  };
  // template from the first proof that packs
  ProofTemplate T;
  bool have_t = false;
  size_t first = 0;
  std::vector<std::string> msgs(n);
  for (; first < n && !have_t; first++) {
    try { have_t = T.build(C, jsons[first], lens[first], dst + (size_t)W * first); codes[first] = P2V_OK; }
    catch (...) { codes[first] = dom_pack(first, &msgs[first]); }
  }
  auto work = [&](size_t a, size_t b) {
    for (size_t i = a; i < b; i++) {
      if (have_t && T.pack(jsons[i], lens[i], dst + (size_t)W * i)) { codes[i] = P2V_OK; continue; }
      codes[i] = dom_pack(i, &msgs[i]);
    }
  };
  const size_t rest = n - first;
  int nt = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
  if (nt < 1) nt = 1;
  if ((size_t)nt > rest) nt = (int)(rest ? rest : 1);
  if (nt <= 1) work(first, n);
  else {
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; t++) pool.emplace_back(work, first + rest * t / nt, first + rest * (t + 1) / nt);
    for (auto& th : pool) th.join();
  }
  int nfail = 0;
  for (size_t i = 0; i < n; i++)
    if (codes[i] != P2V_OK) { if (!nfail) g_err = "proof " + std::to_string(i) + ": " + msgs[i]; nfail++; }
  return nfail;
}

int p2v_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

#define HCK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { return fail(P2V_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); } } while (0)

// the staging buffer for batches given in host memory (run from host, JSON / binary ingest)
static hipError_t input_buf(p2v_verifier* v) {
  return v->in.p ? hipSuccess : v->in.alloc(v->in_bytes);
}

void p2v_verifier_free(p2v_verifier* v) {
  if (!v) return;
  {   // unlink: no workspace keeps a pointer to this one, and its own link goes away
    std::lock_guard<std::mutex> lk(g_chain_mu);
    for (p2v_verifier* n : v->chain_next) n->chain_prev = nullptr;
    if (v->chain_prev) {
      auto& nx = v->chain_prev->chain_next;
      nx.erase(std::remove(nx.begin(), nx.end(), v), nx.end());
    }
  }
  (void)hipSetDevice(v->device);
  for (DevBuf* b : {&v->in, &v->soa, &v->chal, &v->leafdig, &v->mk, &v->fbits, &v->qvals, &v->van, &v->vparts, &v->lutre, &v->res, &v->trace, &v->t_cs, &v->t_kis,
                    &v->t_gkind, &v->t_gpar, &v->t_ggrp, &v->t_gwoff, &v->t_w, &v->t_gs, &v->t_ge, &v->t_lin, &v->t_lout, &v->t_loff, &v->t_llen, &v->t_tw, &v->t_ops, &v->t_vit, &v->t_rin, &v->t_rout, &v->t_roff, &v->t_rch, &v->t_pbase, &v->t_pw, &v->lutpart, &v->chal2, &v->j_blob, &v->j_offs, &v->j_skel, &v->j_tok, &v->j_ok,
                    &v->b_rsrc, &v->b_rdst, &v->b_rlen, &v->b_coff, &v->b_cval,
                    &v->m_plan, &v->m_fol, &v->m_chain, &v->m_count, &v->m_fix, &v->m_badq, &v->m_node})
    b->free_();
  if (v->timed) for (auto& e : v->ev) (void)hipEventDestroy(e);
  if (v->dep_p1) (void)hipEventDestroy(v->dep_p1);
  if (v->dep_side) (void)hipEventDestroy(v->dep_side);
  if (v->dep_tr) (void)hipEventDestroy(v->dep_tr);
  if (v->p1_done) (void)hipEventDestroy(v->p1_done);
  if (v->side) (void)hipStreamDestroy(v->side);
  if (v->side2) (void)hipStreamDestroy(v->side2);
  if (v->ts) (void)hipStreamDestroy(v->ts);
  if (v->side3) (void)hipStreamDestroy(v->side3);
  if (v->dep_v3) (void)hipEventDestroy(v->dep_v3);
  for (int k = 0; k < 2; k++) {
    if (v->tr_done[k]) (void)hipEventDestroy(v->tr_done[k]);
    if (v->chal_free[k]) (void)hipEventDestroy(v->chal_free[k]);
  }
  if (v->dep_fri) (void)hipEventDestroy(v->dep_fri);
  if (v->h_res) (void)hipHostFree(v->h_res);
  delete v;
}

int p2v_verifier_chain(p2v_verifier* v, p2v_verifier* prev) {
  if (!v) return fail(P2V_E_ARG, "null verifier");
  if (prev && prev->device != v->device) return fail(P2V_E_ARG, "p2v_verifier_chain: verifiers on different devices");
  std::lock_guard<std::mutex> lk(g_chain_mu);
  if (v->chain_prev) {
    auto& nx = v->chain_prev->chain_next;
    nx.erase(std::remove(nx.begin(), nx.end(), v), nx.end());
  }
  v->chain_prev = prev;
  if (prev) prev->chain_next.push_back(v);
  return P2V_OK;
}

int p2v_verifier_create(const p2v_circuit* pc, int device, size_t max_batch, p2v_verifier** out) {
  if (!pc || !out || max_batch == 0) return fail(P2V_E_ARG, "null argument / zero batch");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(P2V_E_NODEVICE, "no HIP device available: libp2v verifies on MI355X only (no CPU fallback)");
  if (device < 0 || device >= ndev) return fail(P2V_E_ARG, "bad device index");
  HCK(hipSetDevice(device));
  const Circuit& C = pc->c;
  auto* v = new p2v_verifier();
  v->circ = pc; v->device = device; v->max_batch = max_batch;
  v->Bmax = (max_batch + 63) / 64 * 64;
  if (const char* ss = getenv("P2V_SINGLE_STREAM")) v->single_stream = ss[0] == '1';
  if (const char* sp = getenv("P2V_SIDE_PRIO")) v->side_prio = sp[0] == '1';
  if (const char* ds = getenv("P2V_DEBUG_SYNC")) v->debug_sync = ds[0] == '1';
  if (const char* f1 = getenv("P2V_PHASE1")) v->split_phase1 = !strcmp(f1, "split") ? 1 : !strcmp(f1, "excl") ? 2 : 0;
  if (const char* ff = getenv("P2V_FRI_FIRST")) v->fri_first = ff[0] == '1';
  if (const char* sw = getenv("P2V_SIDE_WG")) v->side_wg = atoi(sw) == 64 ? 64 : 256;
  if (const char* lm = getenv("P2V_LANE_MIN")) v->lane_min_batch = atoi(lm) > 0 ? atoi(lm) : v->lane_min_batch;
  if (const char* qm = getenv("P2V_QUAD_MIN")) v->quad_min_batch = atoi(qm) > 0 ? atoi(qm) : v->quad_min_batch;
  if (const char* mc = getenv("P2V_MERKLE_CSE")) v->merkle_cse = mc[0] != '0';
  if (const char* lx = getenv("P2V_LAT_MAX")) v->lat_max_batch = atoi(lx) >= 0 ? atoi(lx) : v->lat_max_batch;
  if (const char* tm = getenv("P2V_TRANSCRIPT")) v->transcript_mode = !strcmp(tm, "row") ? 1 : !strcmp(tm, "quad") ? 2 : !strcmp(tm, "lane") ? 3 : !strcmp(tm, "pair") ? 4 : 0;
  DevCircuit& d = v->dc;
  memset(&d, 0, sizeof d);
  d.r = C.r; d.Q = C.num_queries; d.S = (int)C.arities.size(); d.T = 4 + d.S;
  d.num_pis = C.num_pis; d.cap_len = C.cap_len; d.degree_bits = C.degree_bits; d.lde_bits = C.lde_bits; d.pow_bits = C.pow_bits;
  d.num_wires = C.num_wires; d.num_routed = C.num_routed; d.num_constants = C.num_constants; d.ngc = C.num_gate_consts;
  d.ngroups = (int)C.grp_start.size(); d.nls = C.nls; d.nlp = C.nlp; d.npp = C.npp; d.qdf = C.qdf; d.nluts = (int)C.lut_in.size();
  d.depth0 = C.depth0; d.final_len = C.final_len;
  for (int t = 0; t < 4; t++) { d.width[t] = C.oracle_width[t]; d.lwidth[t] = C.leaf_width[t]; }
  d.noop_leaves = C.noop_leaves ? 1 : 0;
  d.n_gates = C.n_gate_eval; d.n_pp_terms = (int)C.n_pp_terms_per_round; d.n_lookup_terms = (int)C.n_lookup_terms_per_round;
  d.alpha_base_gates = C.alpha_base_gates;
  const Layout& L = C.L;
  d.pis = L.pis; d.wcap = L.wcap; d.zcap = L.zcap; d.qcap = L.qcap; d.o_const = L.o_const; d.o_sig = L.o_sig; d.o_wires = L.o_wires;
  d.o_zs = L.o_zs; d.o_pp = L.o_pp; d.o_quot = L.o_quot; d.o_lzs = L.o_lzs; d.o_zs_next = L.o_zs_next; d.o_lzs_next = L.o_lzs_next;
  d.n_this = L.n_this; d.n_next = L.n_next; d.ccaps = L.ccaps; d.final_poly = L.final_poly; d.pow = L.pow; d.q0 = L.q0; d.qstride = L.qstride;
  for (int t = 0; t < 4; t++) { d.leaf[t] = L.leaf[t]; d.path[t] = L.path[t]; }
  {   // unit orders: most expensive tree first (stable), see DevCircuit::leaf_order
    std::vector<std::pair<int64_t, int>> lc, mc;
    for (int t = 0; t < d.T; t++) {
      const int64_t len = t < 4 ? C.leaf_width[t] : (2ll << C.arities[t - 4]);
      lc.push_back({-(len + 7) / 8, t});
      mc.push_back({-(int64_t)(t < 4 ? C.depth0 : C.step_depth[t - 4]), t});
    }
    std::stable_sort(lc.begin(), lc.end()); std::stable_sort(mc.begin(), mc.end());
    for (int k = 0; k < d.T; k++) { d.leaf_order[k] = (int8_t)lc[k].second; d.merkle_order[k] = (int8_t)mc[k].second; }
  }
  for (int s = 0; s < d.S; s++) { d.step_evals[s] = L.step_evals[s]; d.step_path[s] = L.step_path[s]; d.arity[s] = C.arities[s]; d.step_depth[s] = C.step_depth[s]; }
  d.words = L.words;
  for (int i = 0; i < 4; i++) d.digest[i] = C.digest[i];
  { uint64_t x = gl::TWO_ADIC_GEN; for (int m = 0; m <= 32; m++) { d.root_pow2[m] = x; x = gl::mul(x, x); } }
  {
    uint64_t shift = gl::MULT_GEN; int logn = C.lde_bits;
    for (int s = 0; s <= d.S; s++) {
      d.step_shift[s] = shift; d.step_shift_inv[s] = gl::inv(shift);
      if (s < d.S) { d.step_logn[s] = logn; d.inv_arity[s] = gl::inv(1ULL << C.arities[s]); shift = gl::pow(shift, 1ULL << C.arities[s]); logn -= C.arities[s]; }
    }
  }
  // circuit tables
  std::vector<int32_t> gkind, ggrp, gwoff; std::vector<int64_t> gpar; std::vector<uint64_t> wts;
  for (int g = 0; g < C.n_gate_eval; g++) {
    const GateDesc& gd = C.gates[g];
    gkind.push_back(gd.kind); ggrp.push_back(C.sel_idx[g]);
    gpar.push_back(gd.p0); gpar.push_back(gd.p1); gpar.push_back(gd.p2);
    gwoff.push_back((int32_t)wts.size()); wts.insert(wts.end(), gd.weights.begin(), gd.weights.end());
  }
  gwoff.push_back((int32_t)wts.size());
  std::vector<uint64_t> lin, lout; std::vector<int64_t> loff, llen;
  for (size_t t = 0; t < C.lut_in.size(); t++) { loff.push_back((int64_t)lin.size()); llen.push_back((int64_t)C.lut_in[t].size()); lin.insert(lin.end(), C.lut_in[t].begin(), C.lut_in[t].end()); lout.insert(lout.end(), C.lut_out[t].begin(), C.lut_out[t].end()); }
  // evalFinalRE (Lookups.hs:103-109): cur = sum_i delta^(N-1-i) (inp_i + B out_i) over the table
  // padded to N = ceil(len / slots) * slots entries with its FIRST entry.  Stored reversed
  // (index t = N-1-i is the power of delta) and zero-filled to a multiple of P2V_LUT_CHUNK, so
  // the device evaluates it as sum_c delta^(16c) sum_j delta^j e'_(16c+j) (baby/giant steps).
  std::vector<uint32_t> rin, rout; std::vector<int64_t> roff; std::vector<int32_t> rch, pbase{0};
  {
    const int64_t slots = C.num_routed / 3;
    for (size_t t = 0; t < C.lut_in.size(); t++) {
      const auto& li = C.lut_in[t]; const auto& lo = C.lut_out[t];
      const int64_t len = (int64_t)li.size();
      const int64_t N = slots > 0 ? (len + slots - 1) / slots * slots : 0;
      bool small = len > 0;
      for (int64_t i = 0; i < len && small; i++) small = li[i] < (1u << 24) && lo[i] < (1u << 24);
      const int64_t nch = small ? (N + P2V_LUT_CHUNK - 1) / P2V_LUT_CHUNK : 0;
      roff.push_back((int64_t)rin.size()); rch.push_back((int32_t)nch);
      pbase.push_back(pbase.back() + (int32_t)((nch + P2V_LUT_PIECE - 1) / P2V_LUT_PIECE));
      for (int64_t k = 0; k < nch * P2V_LUT_CHUNK; k++) {
        const int64_t i = N - 1 - k, ii = i < len ? i : 0;
        rin.push_back(k < N ? (uint32_t)li[ii] : 0u);
        rout.push_back(k < N ? (uint32_t)lo[ii] : 0u);
      }
    }
  }
  std::vector<uint64_t> tw(256 * (size_t)(d.S ? d.S : 1), 0);
  for (int s = 0; s < d.S; s++) {
    int ab = C.arities[s];
    uint64_t om_inv = gl::inv(gl::subgroup_gen(ab)), x = 1;
    for (int j = 0; j < (1 << ab) && j < 256; j++) { tw[256 * s + j] = x; x = gl::mul(x, om_inv); }
  }
  std::vector<int32_t> gs(C.grp_start.begin(), C.grp_start.end()), ge(C.grp_end.begin(), C.grp_end.end());
  // transcript op program: proofChallenges (Challenge/Verifier.hs:58-103) + friChallenges (Challenge/FRI.hs:65-104)
  std::vector<int32_t> ops;
  auto op = [&](int t, int64_t a_, int64_t n_) { ops.push_back(t); ops.push_back((int32_t)a_); ops.push_back((int32_t)n_); };
  {
    const int r = d.r, C4 = 4 * C.cap_len;
    op(TOP_ABSORB_DIGEST, 0, 4);
    op(TOP_ABSORB_PIH, 0, 4);
    op(TOP_ABSORB_SOA, L.wcap, C4);
    op(TOP_SQUEEZE, CH_BETA(d), r);
    op(TOP_SQUEEZE, CH_GAMMA(d), r);
    if (C.nlp > 0) { op(TOP_COPY, CH_DELTA(d), 2 * r); op(TOP_SQUEEZE, CH_DELTA(d) + 2 * r, 2 * r); }
    else op(TOP_ZERO, CH_DELTA(d), 4 * r);
    op(TOP_ABSORB_SOA, L.zcap, C4);
    op(TOP_SQUEEZE, CH_ALPHA(d), r);
    op(TOP_ABSORB_SOA, L.qcap, C4);
    op(TOP_SQUEEZE, CH_ZETA(d), 2);
    op(TOP_ABSORB_SOA, L.o_const, 2 * (L.n_this + L.n_next));
    op(TOP_SQUEEZE, CH_FRI_ALPHA(d), 2);
    for (int s = 0; s < d.S; s++) { op(TOP_ABSORB_SOA, L.ccaps + (int64_t)s * C4, C4); op(TOP_SQUEEZE, CH_FRI_BETA(d) + 2 * s, 2); }
    op(TOP_ABSORB_SOA, L.final_poly, 2 * C.final_len);
    op(TOP_ABSORB_SOA, L.pow, 1);
    op(TOP_SQUEEZE, CH_POW(d), 1);
    op(TOP_SQUEEZE_IDX, CH_QIDX(d), d.Q);
  }
  d.ntops = (int)(ops.size() / 3);
  // vanishing work items, heaviest first so their waves are dispatched first
  std::vector<int32_t> vit;
  {
    auto item = [&](int t, int a_, int b_, int64_t first) { vit.push_back(t); vit.push_back(a_); vit.push_back(b_); vit.push_back((int32_t)first); };
    d.vcls[0] = 0;
    for (int g = 0; g < C.n_gate_eval; g++)
      if (gkind[g] == G_POSEIDON) for (int k = 0; k < P2V_POSEIDON_PARTS; k++) item(VI_GATE, g, k, p2v_poseidon_part_first_term(k));
    d.vcls[1] = (int)(vit.size() / 4);
    for (int g = 0; g < C.n_gate_eval; g++)   // one item per interpolation chunk (dev.h p2v_coset_parts)
      if (gkind[g] == G_COSET) {
        const int64_t parts = p2v_coset_parts((int)gpar[3 * g], gpar[3 * g + 1], gwoff[g + 1] - gwoff[g]);
        for (int64_t k = 0; k < parts; k++) item(VI_GATE, g, (int)k, p2v_coset_part_first_term(k));
      }
    d.vcls[2] = (int)(vit.size() / 4);
    for (int g = 0; g < C.n_gate_eval; g++) if (gkind[g] != G_POSEIDON && gkind[g] != G_COSET) item(VI_GATE, g, 0, 0);
    for (int j = 0; j < d.r; j++) item(VI_PP, j, 0, d.r + (int64_t)j * d.n_pp_terms);
    item(VI_ZS1, 0, 0, 0);
    d.vcls[3] = (int)(vit.size() / 4);
    if (d.nluts > 0)
      for (int j = 0; j < d.r; j++) item(VI_LOOKUP, j, 0, d.r + (int64_t)d.r * d.n_pp_terms + (int64_t)j * d.n_lookup_terms);
  }
  d.n_vitems = (int)(vit.size() / 4);
  d.vcls[4] = d.n_vitems;
  hipError_t e = hipSuccess;
#define UP(buf, vec) if (e == hipSuccess) e = upload(buf, vec)
  UP(v->t_cs, C.cs_cap); UP(v->t_kis, C.k_is); UP(v->t_gkind, gkind); UP(v->t_gpar, gpar); UP(v->t_ggrp, ggrp); UP(v->t_gwoff, gwoff);
  UP(v->t_w, wts); UP(v->t_gs, gs); UP(v->t_ge, ge); UP(v->t_lin, lin); UP(v->t_lout, lout); UP(v->t_loff, loff); UP(v->t_llen, llen); UP(v->t_tw, tw); UP(v->t_ops, ops); UP(v->t_vit, vit);
  UP(v->t_rin, rin); UP(v->t_rout, rout); UP(v->t_roff, roff); UP(v->t_rch, rch); UP(v->t_pbase, pbase);
  UP(v->t_pw, poseidon_part3_table());
  d.n_lut_pieces = pbase.back();
#undef UP
  const size_t B = v->Bmax;
  const size_t chw = (size_t)(4 + 7 * d.r + 4 + 2 * d.S + 1 + d.Q + 4);
  v->in_bytes = (size_t)L.words * v->Bmax * 8;   // whole 64-proof tiles (P2V_FLAG_INPUT_TILED); allocated on first use
  if (e == hipSuccess && !P2V_PROOF_MAJOR) e = v->soa.alloc((size_t)L.words * B * 8);   // the transposed batch
  if (e == hipSuccess) e = v->chal.alloc(chw * B * 8);
  if (e == hipSuccess) e = v->chal2.alloc(chw * B * 8);
  if (e == hipSuccess) e = v->leafdig.alloc((size_t)d.Q * d.T * 4 * B * 8);
  if (e == hipSuccess) e = v->mk.alloc((size_t)d.Q * d.T * B);
  if (e == hipSuccess) e = v->fbits.alloc((size_t)d.Q * B * 4);
  if (e == hipSuccess) e = v->qvals.alloc((size_t)d.Q * 6 * B * 8);
  if (e == hipSuccess) e = v->van.alloc((size_t)(1 + 4 * d.r) * B * 8);
  if (e == hipSuccess) e = v->vparts.alloc((size_t)d.n_vitems * 2 * d.r * B * 8);
  if (e == hipSuccess) e = v->lutre.alloc((size_t)d.r * (d.nluts ? d.nluts : 1) * B * 8);
  if (e == hipSuccess) e = v->lutpart.alloc((size_t)d.r * (d.n_lut_pieces ? d.n_lut_pieces : 1) * B * 8);
  if (e == hipSuccess) e = v->res.alloc(B);
  if (e == hipSuccess) e = hipHostMalloc((void**)&v->h_res, B);
  if (e == hipSuccess) e = v->trace.alloc((size_t)C.trace_words * B * 8);
  // shared-node Merkle paths: on unless P2V_MERKLE_CSE=0 or the shape exceeds the plan's fields
  d.mcse = v->merkle_cse && d.Q <= P2V_CSE_MAX_Q && d.depth0 <= P2V_CSE_MAX_DEPTH && B <= (size_t)P2V_CSE_MAX_B && d.T < 32;
  if (d.mcse) {
    const size_t ncls = 1 + (size_t)d.S, nb = 1 + (size_t)d.depth0;
    d.mcap = (int64_t)d.T * d.Q * (int64_t)B;
    if (e == hipSuccess) e = v->m_plan.alloc(ncls * d.Q * B * 4);
    if (e == hipSuccess) e = v->m_fol.alloc(ncls * d.Q * B * 8);
    if (e == hipSuccess) e = v->m_chain.alloc(nb * (size_t)d.mcap * 4);
    const size_t cnt_bytes = (nb + 1) * 64;   // bucket counters and the fix-list length, 64 B apart
    if (e == hipSuccess) e = v->m_count.alloc(cnt_bytes);
    if (e == hipSuccess) e = hipMemset(v->m_count.p, 0, cnt_bytes);   // then zeroed by each run's k_merkle_resolve
    if (e == hipSuccess) e = v->m_fix.alloc((size_t)d.mcap * 4);
    if (e == hipSuccess) e = v->m_badq.alloc((size_t)d.T * d.Q * B);
    if (e == hipSuccess) e = v->m_node.alloc((size_t)d.T * d.Q * 4 * B * 8);
    d.mplan = (uint32_t*)v->m_plan.p; d.mfol = (uint64_t*)v->m_fol.p; d.mchain = (uint32_t*)v->m_chain.p;
    d.mcount = (int32_t*)v->m_count.p; d.mfixn = d.mcount + nb * 16; d.mfix = (uint32_t*)v->m_fix.p;
    d.mbadq = (uint8_t*)v->m_badq.p; d.mnode = (uint64_t*)v->m_node.p;
  }
  if (e == hipSuccess) { for (auto& x : v->ev) { e = hipEventCreate(&x); if (e != hipSuccess) break; } v->timed = e == hipSuccess; }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&v->dep_p1, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&v->dep_side, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&v->dep_tr, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&v->p1_done, hipEventDisableTiming);
  // the side stream carries few, long-latency waves (vanishing items, FRI queries); a
  // high-priority queue for it was measured (P2V_SIDE_PRIO=1) and changed nothing
  if (e == hipSuccess) {
    int least = 0, greatest = 0;
    if (v->side_prio && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
      e = hipStreamCreateWithPriority(&v->side, hipStreamNonBlocking, greatest);
    else
      e = hipStreamCreateWithFlags(&v->side, hipStreamNonBlocking);
  }
  // (the latency-mode and lookahead streams are created on first use: every stream a process
  // creates may take one of its few hardware queues, GPU_MAX_HW_QUEUES = 4, and two workspaces'
  // main and side streams must not share one)
  if (e == hipSuccess) e = hipEventCreateWithFlags(&v->dep_v3, hipEventDisableTiming);
  for (int k = 0; k < 2 && e == hipSuccess; k++) {
    e = hipEventCreateWithFlags(&v->tr_done[k], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&v->chal_free[k], hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&v->dep_fri, hipEventDisableTiming);
  if (e != hipSuccess) { p2v_verifier_free(v); return fail(P2V_E_DEVICE, std::string("device allocation: ") + hipGetErrorString(e)); }
  d.cs_cap = (const uint64_t*)v->t_cs.p; d.k_is = (const uint64_t*)v->t_kis.p; d.gate_kind = (const int32_t*)v->t_gkind.p;
  d.gate_par = (const int64_t*)v->t_gpar.p; d.gate_grp = (const int32_t*)v->t_ggrp.p; d.gate_woff = (const int32_t*)v->t_gwoff.p;
  d.weights = (const uint64_t*)v->t_w.p; d.grp_start = (const int32_t*)v->t_gs.p; d.grp_end = (const int32_t*)v->t_ge.p;
  d.lut_in = (const uint64_t*)v->t_lin.p; d.lut_out = (const uint64_t*)v->t_lout.p; d.lut_off = (const int64_t*)v->t_loff.p; d.lut_len = (const int64_t*)v->t_llen.p;
  d.lut_rin = (const uint32_t*)v->t_rin.p; d.lut_rout = (const uint32_t*)v->t_rout.p; d.lut_roff = (const int64_t*)v->t_roff.p; d.lut_rchunks = (const int32_t*)v->t_rch.p; d.lut_pbase = (const int32_t*)v->t_pbase.p;
  d.twiddles = (const uint64_t*)v->t_tw.p; d.tops = (const int32_t*)v->t_ops.p; d.vitems = (const int32_t*)v->t_vit.p;
  d.pos_w = (const uint64_t*)v->t_pw.p;
  d.soa = (const uint64_t*)v->soa.p; d.chal = (uint64_t*)v->chal.p; d.leafdig = (uint64_t*)v->leafdig.p; d.mk_ok = (uint8_t*)v->mk.p;
  d.fri_bits = (uint32_t*)v->fbits.p; d.qvals = (uint64_t*)v->qvals.p; d.van = (uint64_t*)v->van.p; d.vparts = (uint64_t*)v->vparts.p; d.lutre = (uint64_t*)v->lutre.p; d.lutpart = (uint64_t*)v->lutpart.p;
  *out = v;
  return P2V_OK;
}

size_t p2v_tiled_words(size_t n, size_t proof_words) { return (n + 63) / 64 * 64 * proof_words; }

void p2v_tile_proofs(const uint64_t* pm, size_t n, size_t W, uint64_t* tiled) {
  if (!pm || !tiled) return;
  const size_t tiles = (n + 63) / 64;
  for (size_t t = 0; t < tiles; t++) {
    uint64_t* dst = tiled + t * W * 64;
    for (size_t w = 0; w < W; w++)
      for (size_t l = 0; l < 64; l++) {
        const size_t i = t * 64 + l;
        dst[w * 64 + l] = i < n ? pm[i * W + w] : 0;
      }
  }
}

int p2v_verifier_run(p2v_verifier* v, const uint64_t* proofs, size_t n, int8_t* results, uint64_t* trace, void* stream_, uint32_t flags) {
  if (!v || (!proofs && n) || !results) return fail(P2V_E_ARG, "null argument");
  if (n > v->max_batch) return fail(P2V_E_ARG, "batch larger than max_batch");
  if (n == 0) return P2V_OK;
  HCK(hipSetDevice(v->device));
  hipStream_t st = (hipStream_t)stream_;
  const Circuit& C = v->circ->c;
  DevCircuit d = v->dc;
  d.n = (int)n;
  d.unit_filters = (flags & P2V_FLAG_UNIT_FILTERS) ? 1 : 0;
  d.tiled = (flags & P2V_FLAG_INPUT_TILED) ? 1 : 0;
  d.wstride = d.tiled ? 64 : 1;
  if (d.tiled && !P2V_PROOF_MAJOR) return fail(P2V_E_ARG, "P2V_FLAG_INPUT_TILED needs the in-place build (P2V_PROOF_MAJOR=1)");
  // the lookahead transcript runs on its own stream and reads the batch in place; the transposing
  // build's k_transpose writes v->soa on the caller's stream, which that stream does not wait for
  if ((flags & P2V_FLAG_LOOKAHEAD) && !P2V_PROOF_MAJOR) return fail(P2V_E_ARG, "P2V_FLAG_LOOKAHEAD needs the in-place build (P2V_PROOF_MAJOR=1)");
  d.B = (int)((n + 63) / 64 * 64);
  const int64_t words = C.L.words;
  const uint64_t* src = proofs;
  if (!(flags & P2V_FLAG_INPUT_DEVICE)) {
    const size_t in_words = d.tiled ? p2v_tiled_words(n, (size_t)words) : (size_t)words * n;
    HCK(input_buf(v));
    HCK(hipMemcpyAsync(v->in.p, proofs, in_words * 8, hipMemcpyHostToDevice, st));
    src = (const uint64_t*)v->in.p;
  }
  int8_t* dres = (flags & P2V_FLAG_RESULT_DEVICE) ? results : (int8_t*)v->res.p;
  uint64_t* dtrace = nullptr;
  if (trace) dtrace = (flags & P2V_FLAG_RESULT_DEVICE) ? trace : (uint64_t*)v->trace.p;
  const int NPB = d.B / 64;
  const bool tm = v->timed;
  hipStream_t sd = v->single_stream ? st : v->side;
  uint32_t timed_mask = 0;   // slots recorded in this run (only those are read back)
#define T0(k, s_) do { if (tm) { HCK(hipEventRecord(v->ev[2 * (k)], s_)); timed_mask |= 1u << (k); } } while (0)
#define T1(k, s_) do { if (tm) HCK(hipEventRecord(v->ev[2 * (k) + 1], s_)); } while (0)
  // fault isolation (P2V_DEBUG_SYNC=1): each launch is named before it runs and waited for
#define DBG(name, s_) do { if (v->debug_sync) { fprintf(stderr, "p2v: launched %s\n", name); fflush(stderr); \
    HCK(hipStreamSynchronize(s_)); HCK(hipGetLastError()); fprintf(stderr, "p2v: finished %s\n", name); fflush(stderr); } } while (0)
#if P2V_PROOF_MAJOR
  d.soa = src;   // kernels read the proof-major batch in place (devcommon.h ld()); no k_transpose
#else
  T0(0, st);
  k_transpose<<<dim3((unsigned)((words + 63) / 64), NPB), 256, 0, st>>>(src, words, (int)n, (uint64_t*)v->soa.p, d.B);
  DBG("k_transpose", st);
  T1(0, st);
#endif
  // phase 1: transcript waves + leaf-hash waves in one launch (the leaf sponges do not
  // depend on the challenges, so they fill the GPU while the serial transcripts run)
  // transcript form: the row form (16 lanes/proof) has the lowest latency, the quad form
  // (4 lanes/proof) a lower total cost; batches from 4096 proofs hide the quad latency behind
  // their leaf hashing.  P2V_TRANSCRIPT=row|quad|lane|pair overrides (measurement).
  // From lane_min_batch on, the lane form (one lane per proof, about half of the quad's issue
  // cycles per proof: 85.9 M against 169.4 M VALU instructions per 4096 proofs, DESIGN.md §7.0,
  // with a ~5.7 ms chain): the batch's leaf hashing in the same launch outlasts the chain, so it
  // costs no latency (C5's 131 072-proof launches +2.9 %, C3's 16 384 +1 %)
  int tl = d.B >= v->lane_min_batch ? 1 : d.B >= v->quad_min_batch ? 4 : 16;
  if (v->transcript_mode == 1) tl = 16;
  else if (v->transcript_mode == 2) tl = 4;
  else if (v->transcript_mode == 3) tl = 1;
  else if (v->transcript_mode == 4) tl = 2;
  // P2V_PHASE1=excl (measurement) takes the row or quad transcript only: the lane / pair forms
  // fall back to the quad form here, before anything is enqueued
  if (v->split_phase1 == 2 && tl <= 2) tl = 4;
  const int nt_blocks = (tl * d.B + 255) / 256;
  const int leaf_units = d.Q * d.T * NPB;
  // staggered workspaces (p2v_verifier_chain): phase 1 after the linked workspace's latest one
  bool chained = false;   // read under the lock: chain links may change from other host threads
  {
    std::lock_guard<std::mutex> lk(g_chain_mu);   // the linked workspace cannot be freed meanwhile
    chained = v->chain_prev != nullptr;
    if (v->chain_prev && v->chain_prev->p1_recorded.load(std::memory_order_acquire))
      HCK(hipStreamWaitEvent(st, v->chain_prev->p1_done, 0));
  }
  // transcript lookahead: the transcript on v->ts into the challenge buffer of this run's parity,
  // after the run that last read that buffer; the leaf hashing on st; k_merkle after both
  const bool la = (flags & P2V_FLAG_LOOKAHEAD) && (flags & P2V_FLAG_INPUT_DEVICE) && sd != st && !chained;
  int la_slot = 0;
  if (la) {
    if (!v->ts) HCK(hipStreamCreateWithFlags(&v->ts, hipStreamNonBlocking));
    la_slot = (int)(v->la_seq++ & 1u);
    d.chal = (uint64_t*)(la_slot ? v->chal2.p : v->chal.p);
    HCK(hipStreamWaitEvent(v->ts, v->chal_free[la_slot], 0));
    T0(9, v->ts);
    if (tl == 1) k_transcript_lane<<<nt_blocks, 256, 0, v->ts>>>(d, tl);
    else if (tl == 2) k_transcript_pair<<<nt_blocks, 256, 0, v->ts>>>(d, tl);
    else k_transcript<<<nt_blocks, 256, 0, v->ts>>>(d, tl);
    DBG("k_transcript", v->ts);
    T1(9, v->ts);
    HCK(hipEventRecord(v->tr_done[la_slot], v->ts));
    T0(8, st);
    k_leaf<<<(leaf_units + 3) / 4, 256, 0, st>>>(d);
    DBG("k_leaf", st);
    T1(8, st);
    HCK(hipStreamWaitEvent(st, v->tr_done[la_slot], 0));   // k_merkle reads the query indices
    HCK(hipEventRecord(v->dep_p1, st));                     // the side kernels read the challenges
    HCK(hipStreamWaitEvent(sd, v->dep_p1, 0));
  } else if (!v->split_phase1 || sd == st) {
    T0(1, st);
    if (tl == 1) k_phase1_lane<<<nt_blocks + (leaf_units + 3) / 4, 256, 0, st>>>(d, nt_blocks, tl);
    else if (tl == 2) k_phase1_pair<<<nt_blocks + (leaf_units + 3) / 4, 256, 0, st>>>(d, nt_blocks, tl);
    else k_phase1<<<nt_blocks + (leaf_units + 3) / 4, 256, 0, st>>>(d, nt_blocks, tl);
    DBG("k_phase1", st);
    T1(1, st);
    if (sd != st) {
      HCK(hipEventRecord(v->dep_p1, st));
      HCK(hipStreamWaitEvent(sd, v->dep_p1, 0));
    }
  } else if (v->split_phase1 == 2) {
    // the transcripts first, on st, so their waves claim empty SIMDs before the leaf waves land
    HCK(hipEventRecord(v->dep_p1, st));   // the batch is ready on st
    T0(9, st);
    k_transcript_x<<<nt_blocks, 256, 0, st>>>(d, tl);
    DBG("k_transcript_x", st);
    T1(9, st);
    HCK(hipStreamWaitEvent(sd, v->dep_p1, 0));
    T0(8, sd);
    k_leaf<<<(leaf_units + 3) / 4, 256, 0, sd>>>(d);
    DBG("k_leaf", sd);
    T1(8, sd);
    HCK(hipEventRecord(v->dep_tr, sd));
    HCK(hipStreamWaitEvent(st, v->dep_tr, 0));   // k_merkle reads the leaf digests
    HCK(hipEventRecord(v->dep_p1, st));          // k_fri / the vanishing kernels read the challenges
    HCK(hipStreamWaitEvent(sd, v->dep_p1, 0));
  } else {
    HCK(hipEventRecord(v->dep_p1, st));   // the batch is ready on st (H2D, caller's stream order)
    HCK(hipStreamWaitEvent(sd, v->dep_p1, 0));
    T0(9, sd);
    if (tl == 1) k_transcript_lane<<<nt_blocks, 256, 0, sd>>>(d, tl);
    else if (tl == 2) k_transcript_pair<<<nt_blocks, 256, 0, sd>>>(d, tl);
    else k_transcript<<<nt_blocks, 256, 0, sd>>>(d, tl);
    DBG("k_transcript", sd);
    T1(9, sd);
    HCK(hipEventRecord(v->dep_tr, sd));
    T0(8, st);
    k_leaf<<<(leaf_units + 3) / 4, 256, 0, st>>>(d);
    DBG("k_leaf", st);
    T1(8, st);
    HCK(hipStreamWaitEvent(st, v->dep_tr, 0));   // k_merkle reads the query indices
  }
  HCK(hipEventRecord(v->p1_done, st));   // k_merkle's inputs are complete on st here in both forms
  v->p1_recorded.store(true, std::memory_order_release);
  // latency mode (at most 64 proofs): the Merkle paths in the row form (k_merkle_row: 16 lanes per
  // path, 4x shorter chains, 16x the lanes), one-wave work-groups for k_fri, and k_fri on a stream
  // of its own beside the vanishing kernels instead of after them.  Measured:
  // one proof 2.19 -> 1.98 ms, 64 proofs 2.18 -> 2.10 ms; at 128 proofs the row form's lanes cost more than its latency saves
  const bool lat = d.n <= v->lat_max_batch;
  const int mk_wg = lat ? 64 : 256;
  const bool fri2 = lat && sd != st;
  if (fri2 && !v->side2) HCK(hipStreamCreateWithFlags(&v->side2, hipStreamNonBlocking));
  // side-stream work-groups of k_fri / k_vanish_final (P2V_SIDE_WG, measurement)
  const int side_wg = v->side_wg;
  if (fri2) {
    HCK(hipStreamWaitEvent(v->side2, v->p1_done, 0));
    T0(3, v->side2);
    k_fri<<<(d.Q * NPB * 64 + mk_wg - 1) / mk_wg, mk_wg, 0, v->side2>>>(d);
    DBG("k_fri", v->side2);
    T1(3, v->side2);
    HCK(hipEventRecord(v->dep_fri, v->side2));
  }
  // phase 2: Merkle paths on the main stream; FRI queries and the vanishing kernel (few,
  // long-latency waves) on the side stream, concurrently
  // k_fri first: it needs only phase 1 and is the shorter chain, so the vanishing kernels
  // (longest waves, most registers) are what remains when k_merkle's waves retire
  if (v->fri_first && !fri2) {
    T0(3, sd);
    k_fri<<<(d.Q * NPB * 64 + side_wg - 1) / side_wg, side_wg, 0, sd>>>(d);
    DBG("k_fri", sd);
    T1(3, sd);
  }
  T0(7, sd);
  if (d.n_lut_pieces > 0) k_lut<<<(d.r * d.n_lut_pieces * NPB + 3) / 4, 256, 0, sd>>>(d);
  DBG("k_lut", sd);
  T1(7, sd);
  // the vanishing items in three kernels (register allocation per class), timed together
  T0(4, sd);
  // (one wave per work-group; the _r2 forms hold exactly the standard 2 challenge rounds)
  const bool r2 = d.r == 2;
  // latency mode: the coset and misc items on a stream of their own, beside the Poseidon parts
  // (each class is a handful of waves whose chain is the batch's tail)
  hipStream_t sv = sd;
  if (fri2) {
    if (!v->side3) HCK(hipStreamCreateWithFlags(&v->side3, hipStreamNonBlocking));
    HCK(hipStreamWaitEvent(v->side3, v->p1_done, 0));
    sv = v->side3;
  }
  if (d.vcls[1] > d.vcls[0]) {
    if (r2) k_vanish_poseidon_r2<<<(d.vcls[1] - d.vcls[0]) * NPB, 64, 0, sd>>>(d);
    else k_vanish_poseidon_rn<<<(d.vcls[1] - d.vcls[0]) * NPB, 64, 0, sd>>>(d);
  }
  DBG("k_vanish_poseidon", sd);
  if (d.vcls[2] > d.vcls[1]) {
    if (r2) k_vanish_coset_r2<<<(d.vcls[2] - d.vcls[1]) * NPB, 64, 0, sv>>>(d);
    else k_vanish_coset_rn<<<(d.vcls[2] - d.vcls[1]) * NPB, 64, 0, sv>>>(d);
  }
  DBG("k_vanish_coset", sv);
  if (r2) k_vanish_r2<<<(d.vcls[3] - d.vcls[2]) * NPB, 64, 0, sv>>>(d);
  else k_vanish_rn<<<(d.vcls[3] - d.vcls[2]) * NPB, 64, 0, sv>>>(d);
  DBG("k_vanish", sv);
  if (sv != sd) {
    HCK(hipEventRecord(v->dep_v3, sv));
    HCK(hipStreamWaitEvent(sd, v->dep_v3, 0));   // k_vanish_final sums every item
  }
  if (d.vcls[4] > d.vcls[3]) {
    if (r2) k_vanish_lookup_r2<<<(d.vcls[4] - d.vcls[3]) * NPB, 64, 0, sd>>>(d);
    else k_vanish_lookup_rn<<<(d.vcls[4] - d.vcls[3]) * NPB, 64, 0, sd>>>(d);
  }
  DBG("k_vanish_lookup", sd);
  T1(4, sd);
  T0(6, sd);
  k_vanish_final<<<(d.B + side_wg - 1) / side_wg, side_wg, 0, sd>>>(d);
  DBG("k_vanish_final", sd);
  T1(6, sd);
  if (!v->fri_first && !fri2) {
    T0(3, sd);
    k_fri<<<(d.Q * NPB * 64 + side_wg - 1) / side_wg, side_wg, 0, sd>>>(d);
    DBG("k_fri", sd);
    T1(3, sd);
  }
  if (sd != st) HCK(hipEventRecord(v->dep_side, sd));
  T0(2, st);
  const int merkle_units = d.Q * d.T * NPB;
  if (lat) k_merkle_row<<<(unsigned)(((int64_t)d.Q * d.T * d.n * 16 + 255) / 256), 256, 0, st>>>(d);
  else if (d.mcse) {
    // shared nodes once: plan + bucketed chains + followers' statuses (kernels.hip); the chain
    // grid covers every bucket's last partial wave
    const int ncls = 1 + d.S;
    // k_merkle_resolve zeroes the bucket counters for the next run; a run that stopped between
    // the plan and the resolve (an error return) leaves them to be zeroed here
    if (v->cse_dirty) HCK(hipMemsetAsync(v->m_count.p, 0, (size_t)(d.depth0 + 2) * 64, st));
    v->cse_dirty = true;
    k_merkle_plan<<<(ncls * d.Q * NPB + P2V_PLAN_WAVES - 1) / P2V_PLAN_WAVES, 64 * P2V_PLAN_WAVES, 0, st>>>(d);
    DBG("k_merkle_plan", st);
    const int64_t cse_waves = ((int64_t)d.T * d.Q * d.n + 63) / 64 + d.depth0 + 1;
    k_merkle_cse<<<(unsigned)((cse_waves + 31) / 32 * 8), 256, 0, st>>>(d);   // a multiple of 8 blocks (cse_wave: XCD ranges)
    DBG("k_merkle_cse", st);
    // grid-stride over the (usually empty) list: the latency form for up to 16 entries per block,
    // the lane form beyond (one wave per SIMD: a list of every follower, a garbage batch, costs about one
    // more batch); a larger grid waited ~0.5 ms per launch for free slots beside the other batch (r06e)
    k_merkle_fix<<<P2V_FIX_BLOCKS, 256, 0, st>>>(d);
    DBG("k_merkle_fix", st);
    k_merkle_resolve<<<(merkle_units + 3) / 4, 256, 0, st>>>(d);
    DBG("k_merkle_resolve", st);
    v->cse_dirty = false;
  } else k_merkle<<<(merkle_units + 3) / 4, 256, 0, st>>>(d);
  DBG("k_merkle", st);
  T1(2, st);
  if (sd != st) HCK(hipStreamWaitEvent(st, v->dep_side, 0));
  if (fri2) HCK(hipStreamWaitEvent(st, v->dep_fri, 0));
  T0(5, st);
  k_status<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(d, dres, dtrace, C.trace_words);
  DBG("k_status", st);
  T1(5, st);
  // the challenge buffer's last reader is done (a run without the flag used buffer 0: a later
  // lookahead transcript into buffer 0 must wait for it as well)
  if (la) HCK(hipEventRecord(v->chal_free[la_slot], st));
  else if (sd != st) HCK(hipEventRecord(v->chal_free[0], st));
#undef T0
#undef T1
#undef DBG
  HCK(hipGetLastError());
  if (!(flags & P2V_FLAG_RESULT_DEVICE)) {
    HCK(hipMemcpyAsync(v->h_res, dres, n, hipMemcpyDeviceToHost, st));
    if (trace) HCK(hipMemcpyAsync(trace, dtrace, (size_t)C.trace_words * n * 8, hipMemcpyDeviceToHost, st));
  }
  if (!(flags & P2V_FLAG_NO_SYNC) || !(flags & P2V_FLAG_RESULT_DEVICE)) {
    HCK(hipStreamSynchronize(st));
    if (!(flags & P2V_FLAG_RESULT_DEVICE)) memcpy(results, v->h_res, n);
    if (tm) {
      for (int k = 0; k < kNumKernels; k++) {
        float ms = 0;
        if ((timed_mask >> k) & 1u) { if (hipEventElapsedTime(&ms, v->ev[2 * k], v->ev[2 * k + 1]) == hipSuccess) v->last_ms[k] = ms; }
        else v->last_ms[k] = 0;   // not launched in this build / run
      }
      (void)hipGetLastError();   // a failed timing query must not surface as the next call's error
    }
  }
  return P2V_OK;
}

// a pipe of circuit c on `device` whose verifier holds `cap` proofs: an idle one of the pool (the
// smallest that fits), else a new one
static int pipe_acquire(const p2v_circuit* c, int device, size_t cap, HostPipe** out) {
  *out = nullptr;
  {
    std::lock_guard<std::mutex> lk(c->pool_mu);
    HostPipe* best = nullptr;
    for (HostPipe* p : c->pool)
      if (!p->busy && p->device == device && p->cap >= cap && (!best || p->cap < best->cap)) best = p;
    if (best) { best->busy = true; *out = best; return P2V_OK; }
  }
  auto* p = new HostPipe();
  p->device = device; p->cap = cap;
  int rc = P2V_OK;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&p->st, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&p->cs, hipStreamNonBlocking) != hipSuccess)
    rc = fail(P2V_E_DEVICE, "stream creation on device " + std::to_string(device));
  if (rc == P2V_OK) rc = p2v_verifier_create(c, device, cap, &p->v);
  if (rc != P2V_OK) { pipe_free(p); return rc; }
  p->busy = true;
  std::lock_guard<std::mutex> lk(c->pool_mu);
  c->pool.push_back(p);
  *out = p;
  return P2V_OK;
}

static void pipe_release(const p2v_circuit* c, HostPipe* p, bool broken) {
  HostPipe* drop = nullptr;
  {
    std::lock_guard<std::mutex> lk(c->pool_mu);
    p->busy = false;
    int idle = 0;
    for (HostPipe* q : c->pool) idle += (!q->busy && q->device == p->device) ? 1 : 0;
    if (broken || idle > kPoolIdleMax) {   // a pipe whose run failed is not reused
      c->pool.erase(std::remove(c->pool.begin(), c->pool.end(), p), c->pool.end());
      drop = p;
    }
  }
  pipe_free(drop);
}

// verify m proofs (proof-major rows in host memory) on pipe p: one run for a single chunk (the
// latency path: H2D, kernels, D2H on the pipe's stream); otherwise chunks of <= p->cap proofs
// through the ring, copies on the copy stream, verification on the compute stream, statuses
// accumulated on the device and copied back once.
static int pipe_run(HostPipe* p, const uint64_t* src, size_t m, int8_t* results, size_t W, size_t chunk) {
  HCK(hipSetDevice(p->device));
  if (m <= chunk) return p2v_verifier_run(p->v, src, m, results, nullptr, p->st, 0);
  if (!p->have_ring) {
    for (int k = 0; k < HostPipe::kRing; k++) {
      HCK(p->ring[k].alloc(p->cap * W * 8));
      HCK(hipEventCreateWithFlags(&p->copied[k], hipEventDisableTiming));
      HCK(hipEventCreateWithFlags(&p->freed[k], hipEventDisableTiming));
    }
    p->have_ring = true;
  }
  if (p->dres.bytes < m) { p->dres.free_(); HCK(p->dres.alloc(m)); }
  if (p->h_res_cap < m) {
    if (p->h_res) (void)hipHostFree(p->h_res);
    p->h_res = nullptr; p->h_res_cap = 0;
    HCK(hipHostMalloc((void**)&p->h_res, m));
    p->h_res_cap = m;
  }
  const size_t nch = (m + chunk - 1) / chunk;
  for (size_t i = 0; i < nch; i++) {
    const int b = (int)(i % HostPipe::kRing);
    const size_t off = i * chunk, len = std::min(chunk, m - off);
    if (i >= (size_t)HostPipe::kRing) HCK(hipStreamWaitEvent(p->cs, p->freed[b], 0));   // its last reader is done
    HCK(hipMemcpyAsync(p->ring[b].p, src + off * W, len * W * 8, hipMemcpyHostToDevice, p->cs));
    HCK(hipEventRecord(p->copied[b], p->cs));
    HCK(hipStreamWaitEvent(p->st, p->copied[b], 0));
    const int rc = p2v_verifier_run(p->v, (const uint64_t*)p->ring[b].p, len, (int8_t*)p->dres.p + off, nullptr, p->st,
                                    P2V_FLAG_INPUT_DEVICE | P2V_FLAG_RESULT_DEVICE | P2V_FLAG_NO_SYNC);
    if (rc != P2V_OK) return rc;
    HCK(hipEventRecord(p->freed[b], p->st));
  }
  HCK(hipMemcpyAsync(p->h_res, p->dres.p, m, hipMemcpyDeviceToHost, p->st));
  HCK(hipStreamSynchronize(p->st));
  memcpy(results, p->h_res, m);
  return P2V_OK;
}

// the chunk size of a shard of m proofs: the given one, or (0) about an eighth of the shard in
// multiples of 256 between 256 and 16384, so a batch of a few thousand proofs still has several
// chunks in flight and a large one keeps its launches large
static size_t auto_chunk(size_t m, size_t chunk) {
  if (chunk) return chunk;
  const size_t c = (m / 8 + 255) / 256 * 256;
  return std::min<size_t>(16384, std::max<size_t>(256, c));
}

int p2v_verify_batch_devices(const p2v_circuit* c, const uint64_t* proofs, size_t n, int8_t* results,
                             const int* devices, int ndevices, size_t chunk) {
  if (!c || !devices || ndevices <= 0 || (n && (!proofs || !results))) return fail(P2V_E_ARG, "null argument / no devices");
  if (n == 0) return P2V_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(P2V_E_NODEVICE, "no HIP device available: libp2v verifies on MI355X only (no CPU fallback)");
  for (int i = 0; i < ndevices; i++)
    if (devices[i] < 0 || devices[i] >= ndev) return fail(P2V_E_ARG, "bad device index " + std::to_string(devices[i]));
  const size_t W = (size_t)c->c.L.words;
  const int shards = (int)std::min<size_t>((size_t)ndevices, n);
  std::vector<int> rcs(shards, P2V_OK);
  std::vector<std::string> msgs(shards);
  auto work = [&](int s) {
    const size_t base = n / shards, extra = n % shards;   // p2v.shard_bounds
    const size_t a = s * base + std::min<size_t>(s, extra), b = a + base + ((size_t)s < extra ? 1 : 0);
    const size_t m = b - a;
    // one chunk: a verifier sized to the shard (64-proof granules, powers of two), else chunks
    const size_t ch = m <= 64 ? m : auto_chunk(m, chunk);
    size_t cap = 64;
    while (cap < std::min(m, ch)) cap <<= 1;
    if (m > ch) cap = ch;
    HostPipe* p = nullptr;
    int rc = pipe_acquire(c, devices[s], cap, &p);
    if (rc == P2V_OK) {
      rc = pipe_run(p, proofs + a * W, m, results + a, W, ch);
      pipe_release(c, p, rc != P2V_OK);
    }
    if (rc != P2V_OK) msgs[s] = g_err;   // g_err is thread-local: carry the message back
    rcs[s] = rc;
  };
  if (shards == 1) work(0);   // the calling thread (a drop-in verifyProof call starts no thread)
  else {
    std::vector<std::thread> pool;
    for (int s = 0; s < shards; s++) pool.emplace_back(work, s);
    for (auto& t : pool) t.join();
  }
  for (int s = 0; s < shards; s++)
    if (rcs[s] != P2V_OK)
      return fail(rcs[s], "shard " + std::to_string(s) + " (device " + std::to_string(devices[s]) + "): " + msgs[s]);
  return P2V_OK;
}

// JSON texts -> packed rows of v->in (device packer against the template, host reader for
// the rest); codes[i] as p2v_pack_proof_json
static int pack_json_into(p2v_verifier* v, const char* blob, const uint64_t* offsets, size_t n,
                          int32_t* codes, size_t* n_device, void* stream_) {
  if (n_device) *n_device = 0;
  if (!v || (n && (!blob || !offsets || !codes))) return fail(P2V_E_ARG, "null argument");
  if (n > v->max_batch) return fail(P2V_E_ARG, "batch larger than max_batch");
  if (n == 0) return P2V_OK;
  HCK(hipSetDevice(v->device));
  HCK(input_buf(v));
  hipStream_t st = (hipStream_t)stream_;
  const Circuit& C = v->circ->c;
  const int64_t W = C.L.words;
  auto text = [&](size_t i) { return blob + offsets[i]; };
  auto tlen = [&](size_t i) { return (size_t)(offsets[i + 1] - offsets[i]); };
  std::vector<uint64_t> row((size_t)W);
  // template: keep the current one while it packs the batch's first proof, else rebuild it
  // from the first proof the full reader accepts
  bool fresh = false;
  if (!(v->have_tmpl && v->tmpl.pack(text(0), tlen(0), row.data()))) {
    v->have_tmpl = false;
    for (size_t i = 0; i < n && !v->have_tmpl && i < 64; i++) {
      try { v->have_tmpl = v->tmpl.build(C, text(i), tlen(i), row.data()); } catch (...) { v->have_tmpl = false; }
    }
    fresh = v->have_tmpl;
  }
  std::vector<uint8_t> skel; std::vector<int32_t> tok;
  const bool dev_ok = v->have_tmpl && (!fresh || v->tmpl.device_form(skel, tok));
  if (fresh && dev_ok) {
    auto put = [&](DevBuf& b, const void* h, size_t bytes) -> hipError_t {
      if (b.bytes < bytes + 64) { b.free_(); hipError_t e = b.alloc(bytes + 64); if (e != hipSuccess) return e; }   // + vector-load slack
      return hipMemcpy(b.p, h, bytes, hipMemcpyHostToDevice);
    };
    HCK(put(v->j_skel, skel.data(), skel.size()));
    HCK(put(v->j_tok, tok.data(), tok.size() * sizeof(int32_t)));
    v->skel_len = (int64_t)skel.size(); v->ntok = (int64_t)tok.size();
  } else if (fresh || !v->have_tmpl) {
    // a new template without a device form (or none at all): drop the previous template's
    // device form, so no later batch pairs it with this host template
    v->skel_len = 0; v->ntok = 0;
  }
  std::vector<int8_t> okf(n, 0);
  if (dev_ok && v->ntok > 0) {
    const uint64_t base = offsets[0], bytes = offsets[n] - base;
    if (v->j_blob.bytes < bytes + 64) { v->j_blob.free_(); HCK(v->j_blob.alloc(bytes + 64)); }   // + vector-load slack
    if (v->j_offs.bytes < (n + 1) * 8) { v->j_offs.free_(); HCK(v->j_offs.alloc((n + 1) * 8)); }
    if (v->j_ok.bytes < n) { v->j_ok.free_(); HCK(v->j_ok.alloc(n)); }
    std::vector<uint64_t> rel(n + 1);
    for (size_t i = 0; i <= n; i++) rel[i] = offsets[i] - base;
    HCK(hipMemcpyAsync(v->j_blob.p, blob + base, bytes, hipMemcpyHostToDevice, st));
    HCK(hipMemcpyAsync(v->j_offs.p, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
    k_json_pack<<<(unsigned)n, 256, 0, st>>>((const uint8_t*)v->j_blob.p, (const uint64_t*)v->j_offs.p, (int)n, (const uint8_t*)v->j_skel.p,
                                             v->skel_len, (const int32_t*)v->j_tok.p, v->ntok, (uint64_t*)v->in.p, W, (int8_t*)v->j_ok.p);
    HCK(hipGetLastError());
    HCK(hipMemcpyAsync(v->h_res, v->j_ok.p, n, hipMemcpyDeviceToHost, st));
    HCK(hipStreamSynchronize(st));
    memcpy(okf.data(), v->h_res, n);
  }
  if (n_device) for (size_t i = 0; i < n; i++) *n_device += okf[i] ? 1 : 0;
  // the rest (other formatting, exotic numbers, errors): the host reader, as p2v_pack_proof_json
  for (size_t i = 0; i < n; i++) {
    codes[i] = P2V_OK;
    if (okf[i]) continue;
    try {
      JVal pj = parse_json(text(i), tlen(i));
      pack_proof(C, pj, row.data());
      HCK(hipMemcpyAsync((uint64_t*)v->in.p + i * W, row.data(), (size_t)W * 8, hipMemcpyHostToDevice, st));
      HCK(hipStreamSynchronize(st));   // row is reused
    } catch (const ShapeError&) { codes[i] = P2V_E_SHAPE; }
    catch (...) { codes[i] = P2V_E_PARSE; }
  }
  return P2V_OK;
}

// the circuit's byte map (circuit.cpp bytes_map) on the verifier's device, made once
static int ensure_bytes_map(p2v_verifier* v) {
  if (v->have_bmap) return P2V_OK;
  const BytesMap m = bytes_map(v->circ->c);
  auto put = [&](DevBuf& b, const void* h, size_t bytes) -> hipError_t {
    hipError_t e = b.alloc(bytes + 16);
    if (e == hipSuccess && bytes) e = hipMemcpy(b.p, h, bytes, hipMemcpyHostToDevice);
    return e;
  };
  HCK(put(v->b_rsrc, m.run_src.data(), m.run_src.size() * 8));
  HCK(put(v->b_rdst, m.run_dst.data(), m.run_dst.size() * 8));
  HCK(put(v->b_rlen, m.run_len.data(), m.run_len.size() * 8));
  HCK(put(v->b_coff, m.chk_off.data(), m.chk_off.size() * 8));
  HCK(put(v->b_cval, m.chk_val.data(), m.chk_val.size()));
  v->nruns = (int)m.run_len.size(); v->nchk = (int)m.chk_off.size(); v->bfixed = m.fixed;
  v->have_bmap = true;
  return P2V_OK;
}

// plonky2 binary proofs -> packed rows of v->in (k_bytes_pack against the circuit's byte map,
// the host reader for any proof that fails a check); codes[i] as p2v_pack_proof_bytes
static int pack_bytes_into(p2v_verifier* v, const uint8_t* blob, const uint64_t* offsets, size_t n,
                           int32_t* codes, size_t* n_device, void* stream_) {
  if (n_device) *n_device = 0;
  if (!v || (n && (!blob || !offsets || !codes))) return fail(P2V_E_ARG, "null argument");
  if (n > v->max_batch) return fail(P2V_E_ARG, "batch larger than max_batch");
  if (n == 0) return P2V_OK;
  HCK(hipSetDevice(v->device));
  HCK(input_buf(v));
  hipStream_t st = (hipStream_t)stream_;
  const Circuit& C = v->circ->c;
  const int64_t W = C.L.words;
  { const int rc = ensure_bytes_map(v); if (rc != P2V_OK) return rc; }
  const uint64_t base = offsets[0], bytes = offsets[n] - base;
  if (v->j_blob.bytes < bytes + 64) { v->j_blob.free_(); HCK(v->j_blob.alloc(bytes + 64)); }   // + unaligned-load slack
  if (v->j_offs.bytes < (n + 1) * 8) { v->j_offs.free_(); HCK(v->j_offs.alloc((n + 1) * 8)); }
  if (v->j_ok.bytes < n) { v->j_ok.free_(); HCK(v->j_ok.alloc(n)); }
  std::vector<uint64_t> rel(n + 1);
  for (size_t i = 0; i <= n; i++) rel[i] = offsets[i] - base;
  HCK(hipMemcpyAsync(v->j_blob.p, blob + base, bytes, hipMemcpyHostToDevice, st));
  HCK(hipMemcpyAsync(v->j_offs.p, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, st));
  k_bytes_pack<<<(unsigned)n, 256, 0, st>>>((const uint8_t*)v->j_blob.p, (const uint64_t*)v->j_offs.p, (int)n, (const int64_t*)v->b_rsrc.p,
                                            (const int64_t*)v->b_rdst.p, (const int64_t*)v->b_rlen.p, v->nruns, (const int64_t*)v->b_coff.p,
                                            (const uint8_t*)v->b_cval.p, v->nchk, v->bfixed, (int64_t)C.num_pis, C.L.pis,
                                            (uint64_t*)v->in.p, W, (int8_t*)v->j_ok.p);
  HCK(hipGetLastError());
  HCK(hipMemcpyAsync(v->h_res, v->j_ok.p, n, hipMemcpyDeviceToHost, st));
  HCK(hipStreamSynchronize(st));
  std::vector<int8_t> okf(v->h_res, v->h_res + n);
  std::vector<uint64_t> row((size_t)W);
  for (size_t i = 0; i < n; i++) {
    codes[i] = P2V_OK;
    if (okf[i]) { if (n_device) (*n_device)++; continue; }
    try {
      pack_proof_bytes(C, blob + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), row.data());
      HCK(hipMemcpyAsync((uint64_t*)v->in.p + i * W, row.data(), (size_t)W * 8, hipMemcpyHostToDevice, st));
      HCK(hipStreamSynchronize(st));   // row is reused
    } catch (const ShapeError&) { codes[i] = P2V_E_SHAPE; }
    catch (...) { codes[i] = P2V_E_PARSE; }
  }
  return P2V_OK;
}

// plonky2 binary proofs in host memory, verified through the circuit's pooled pipe: per chunk the
// bytes are copied on the copy stream, packed on the device (k_bytes_pack into a ring slot) and
// verified on the compute stream, up to kRing chunks in flight.  Proofs the device packer flags
// are packed by the host reader afterwards and verified in one more run (or get the reader's
// code), so results and codes equal p2v_verifier_run_bytes'.
int p2v_verify_batch_bytes(const p2v_circuit* c, const uint8_t* blob, const uint64_t* offsets, size_t n,
                           int8_t* results, int32_t* codes, size_t* n_device, int device, size_t chunk) {
  if (n_device) *n_device = 0;
  if (!c || (n && (!blob || !offsets || !results || !codes))) return fail(P2V_E_ARG, "null argument");
  if (n == 0) return P2V_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(P2V_E_NODEVICE, "no HIP device available: libp2v verifies on MI355X only (no CPU fallback)");
  if (device < 0 || device >= ndev) return fail(P2V_E_ARG, "bad device index");
  const Circuit& C = c->c;
  const size_t W = (size_t)C.L.words;
  const size_t ch = auto_chunk(n, chunk);
  size_t cap = 64;
  while (cap < std::min(n, ch)) cap <<= 1;
  if (n > ch) cap = ch;
  HostPipe* p = nullptr;
  int rc = pipe_acquire(c, device, cap, &p);
  if (rc != P2V_OK) return rc;
  auto body = [&]() -> int {
    HCK(hipSetDevice(device));
    { const int r = ensure_bytes_map(p->v); if (r != P2V_OK) return r; }
    if (!p->have_ring) {
      for (int k = 0; k < HostPipe::kRing; k++) {
        HCK(p->ring[k].alloc(p->cap * W * 8));
        HCK(hipEventCreateWithFlags(&p->copied[k], hipEventDisableTiming));
        HCK(hipEventCreateWithFlags(&p->freed[k], hipEventDisableTiming));
      }
      p->have_ring = true;
    }
    if (p->dres.bytes < n) { p->dres.free_(); HCK(p->dres.alloc(n)); }
    if (p->dok.bytes < n) { p->dok.free_(); HCK(p->dok.alloc(n)); }
    if (p->h_res_cap < n) {
      if (p->h_res) (void)hipHostFree(p->h_res);
      p->h_res = nullptr; p->h_res_cap = 0;
      HCK(hipHostMalloc((void**)&p->h_res, n));
      p->h_res_cap = n;
    }
    if (p->h_ok_cap < n) {
      if (p->h_ok) (void)hipHostFree(p->h_ok);
      p->h_ok = nullptr; p->h_ok_cap = 0;
      HCK(hipHostMalloc((void**)&p->h_ok, n));
      p->h_ok_cap = n;
    }
    p2v_verifier* v = p->v;
    const size_t nch = (n + ch - 1) / ch;
    for (size_t i = 0; i < nch; i++) {
      const int b = (int)(i % HostPipe::kRing);
      const size_t off = i * ch, len = std::min(ch, n - off);
      const uint64_t base = offsets[off], bytes = offsets[off + len] - base;
      if (i >= (size_t)HostPipe::kRing) {
        HCK(hipEventSynchronize(p->copied[b]));              // the slot's host offsets are no longer read
        HCK(hipStreamWaitEvent(p->cs, p->freed[b], 0));      // its device buffers' last reader is done
      }
      if (p->bbytes[b].bytes < bytes + 64) { p->bbytes[b].free_(); HCK(p->bbytes[b].alloc(bytes + 64)); }   // + unaligned-load slack
      if (p->boffs[b].bytes < (len + 1) * 8) { p->boffs[b].free_(); HCK(p->boffs[b].alloc((p->cap + 1) * 8)); }
      auto& ho = p->hoffs[b];
      ho.resize(len + 1);
      for (size_t k = 0; k <= len; k++) ho[k] = offsets[off + k] - base;
      HCK(hipMemcpyAsync(p->bbytes[b].p, blob + base, bytes, hipMemcpyHostToDevice, p->cs));
      HCK(hipMemcpyAsync(p->boffs[b].p, ho.data(), (len + 1) * 8, hipMemcpyHostToDevice, p->cs));
      HCK(hipEventRecord(p->copied[b], p->cs));
      HCK(hipStreamWaitEvent(p->st, p->copied[b], 0));
      k_bytes_pack<<<(unsigned)len, 256, 0, p->st>>>((const uint8_t*)p->bbytes[b].p, (const uint64_t*)p->boffs[b].p, (int)len,
                                                      (const int64_t*)v->b_rsrc.p, (const int64_t*)v->b_rdst.p, (const int64_t*)v->b_rlen.p,
                                                      v->nruns, (const int64_t*)v->b_coff.p, (const uint8_t*)v->b_cval.p, v->nchk, v->bfixed,
                                                      (int64_t)C.num_pis, C.L.pis, (uint64_t*)p->ring[b].p, (int64_t)W,
                                                      (int8_t*)p->dok.p + off);
      HCK(hipGetLastError());
      const int r = p2v_verifier_run(v, (const uint64_t*)p->ring[b].p, len, (int8_t*)p->dres.p + off, nullptr, p->st,
                                     P2V_FLAG_INPUT_DEVICE | P2V_FLAG_RESULT_DEVICE | P2V_FLAG_NO_SYNC);
      if (r != P2V_OK) return r;
      HCK(hipEventRecord(p->freed[b], p->st));
    }
    HCK(hipMemcpyAsync(p->h_res, p->dres.p, n, hipMemcpyDeviceToHost, p->st));
    HCK(hipMemcpyAsync(p->h_ok, p->dok.p, n, hipMemcpyDeviceToHost, p->st));
    HCK(hipStreamSynchronize(p->st));
    memcpy(results, p->h_res, n);
    // the proofs the device packer did not take: the host reader, then one more run for those it packs
    std::vector<size_t> redo;
    std::vector<uint64_t> rows;
    for (size_t i = 0; i < n; i++) {
      codes[i] = P2V_OK;
      if (p->h_ok[i]) { if (n_device) (*n_device)++; continue; }
      rows.resize((redo.size() + 1) * W);
      try {
        pack_proof_bytes(C, blob + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), rows.data() + redo.size() * W);
        redo.push_back(i);
      } catch (const ShapeError&) { codes[i] = P2V_E_SHAPE; results[i] = P2V_ERR_SHAPE; }
      catch (...) { codes[i] = P2V_E_PARSE; results[i] = P2V_ERR_PARSE; }
    }
    if (!redo.empty()) {
      std::vector<int8_t> rr(redo.size());
      const int r = pipe_run(p, rows.data(), redo.size(), rr.data(), W, p->cap);
      if (r != P2V_OK) return r;
      for (size_t k = 0; k < redo.size(); k++) results[redo[k]] = rr[k];
    }
    return P2V_OK;
  };
  rc = body();
  pipe_release(c, p, rc != P2V_OK);
  return rc;
}

int p2v_verifier_pack_bytes(p2v_verifier* v, const uint8_t* blob, const uint64_t* offsets, size_t n,
                            int32_t* codes, size_t* n_device, uint64_t* words, void* stream_) {
  int rc = pack_bytes_into(v, blob, offsets, n, codes, n_device, stream_);
  if (rc != P2V_OK || n == 0 || !words) return rc;
  hipStream_t st = (hipStream_t)stream_;
  const size_t W = (size_t)v->circ->c.L.words;
  HCK(hipMemcpyAsync(words, v->in.p, n * W * 8, hipMemcpyDeviceToHost, st));
  HCK(hipStreamSynchronize(st));
  for (size_t i = 0; i < n; i++)
    if (codes[i] != P2V_OK) memset(words + i * W, 0, W * 8);
  return P2V_OK;
}

int p2v_verifier_run_bytes(p2v_verifier* v, const uint8_t* blob, const uint64_t* offsets, size_t n,
                           int8_t* results, int32_t* codes, size_t* n_device, void* stream_) {
  if (n && !results) return fail(P2V_E_ARG, "null argument");
  int rc = pack_bytes_into(v, blob, offsets, n, codes, n_device, stream_);
  if (rc != P2V_OK || n == 0) return rc;
  rc = p2v_verifier_run(v, (const uint64_t*)v->in.p, n, results, nullptr, stream_, P2V_FLAG_INPUT_DEVICE);
  if (rc != P2V_OK) return rc;
  for (size_t i = 0; i < n; i++)
    if (codes[i] != P2V_OK) results[i] = codes[i] == P2V_E_SHAPE ? P2V_ERR_SHAPE : P2V_ERR_PARSE;
  return P2V_OK;
}

int p2v_verifier_pack_json(p2v_verifier* v, const char* blob, const uint64_t* offsets, size_t n,
                           int32_t* codes, size_t* n_device, uint64_t* words, void* stream_) {
  int rc = pack_json_into(v, blob, offsets, n, codes, n_device, stream_);
  if (rc != P2V_OK || n == 0 || !words) return rc;
  hipStream_t st = (hipStream_t)stream_;
  const size_t W = (size_t)v->circ->c.L.words;
  HCK(hipMemcpyAsync(words, v->in.p, n * W * 8, hipMemcpyDeviceToHost, st));
  HCK(hipStreamSynchronize(st));
  for (size_t i = 0; i < n; i++)
    if (codes[i] != P2V_OK) memset(words + i * W, 0, W * 8);
  return P2V_OK;
}

int p2v_verifier_run_json(p2v_verifier* v, const char* blob, const uint64_t* offsets, size_t n,
                          int8_t* results, int32_t* codes, size_t* n_device, void* stream_) {
  if (n && !results) return fail(P2V_E_ARG, "null argument");
  int rc = pack_json_into(v, blob, offsets, n, codes, n_device, stream_);
  if (rc != P2V_OK || n == 0) return rc;
  rc = p2v_verifier_run(v, (const uint64_t*)v->in.p, n, results, nullptr, stream_, P2V_FLAG_INPUT_DEVICE);
  if (rc != P2V_OK) return rc;
  for (size_t i = 0; i < n; i++)
    if (codes[i] != P2V_OK) results[i] = codes[i] == P2V_E_SHAPE ? P2V_ERR_SHAPE : P2V_ERR_PARSE;
  return P2V_OK;
}

int p2v_selftest(int device, int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n) {
  const bool needs_b = op == 0 || op == 3 || op == 4 || op == 6;
  if (op < 0 || op > 11 || (n && (!a || !out || (needs_b && !b)))) return fail(P2V_E_ARG, "bad op / null argument");
  const int ndev = p2v_device_count();
  if (ndev == 0) return fail(P2V_E_NODEVICE, "no HIP device");
  if (device < 0 || device >= ndev) return fail(P2V_E_ARG, "bad device index");
  if (n == 0) return P2V_OK;
  HCK(hipSetDevice(device));
  // words per item of a / b and of out
  const bool scalar = op == 0 || op == 3 || op == 5 || op == 6 || op == 7 || op == 8;
  const size_t w = scalar ? 1 : 12, wo = op == 6 ? 2 : w;
  const size_t bw = op == 4 ? 24 : scalar && needs_b ? n : 2;
  DevBuf da, db, dout;
  auto cleanup = [&]() { da.free_(); db.free_(); dout.free_(); };
  hipError_t e = da.alloc(n * w * 8);
  if (e == hipSuccess) e = db.alloc(bw * 8);
  if (e == hipSuccess) e = dout.alloc(n * wo * 8);
  if (e == hipSuccess) e = hipMemcpy(da.p, a, n * w * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess && needs_b) e = hipMemcpy(db.p, b, bw * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    if (op >= 9) {
      const int lanes = op == 9 ? 16 : op == 10 ? 4 : 2;
      hipLaunchKernelGGL(k_selftest_forms, dim3((unsigned)((n * lanes + 255) / 256)), dim3(256), 0, 0, op, (const uint64_t*)da.p,
                         (uint64_t*)dout.p, (int64_t)n);
    } else {
      hipLaunchKernelGGL(k_selftest, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, op, (const uint64_t*)da.p,
                         (const uint64_t*)db.p, (uint64_t*)dout.p, (int64_t)n);
    }
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, dout.p, n * wo * 8, hipMemcpyDeviceToHost);
  cleanup();
  if (e != hipSuccess) return fail(P2V_E_DEVICE, std::string("p2v_selftest: ") + hipGetErrorString(e));
  return P2V_OK;
}

int p2v_count_mismatches(const int8_t* results, const int8_t* expect, size_t n, uint64_t* counters, void* stream) {
  if (!counters || (n && (!results || !expect))) return fail(P2V_E_ARG, "null argument");
  const unsigned blocks = n ? (unsigned)((n + 255) / 256) : 1;
  hipLaunchKernelGGL(k_count_mismatches, dim3(blocks), dim3(256), 0, (hipStream_t)stream, results, expect, (int64_t)n,
                     (unsigned long long*)counters);
  HCK(hipGetLastError());
  return P2V_OK;
}

int p2v_clock_probe(uint64_t* stamps, int nblocks, void* stream) {
  if (!stamps || nblocks <= 0) return fail(P2V_E_ARG, "null argument / no blocks");
  hipLaunchKernelGGL(k_clock_probe, dim3((unsigned)nblocks), dim3(64), 0, (hipStream_t)stream, (unsigned long long*)stamps);
  HCK(hipGetLastError());
  return P2V_OK;
}

int p2v_verifier_last_timings(const p2v_verifier* v, float* out, int max) {
  if (!v || !out) return 0;
  int k = 0;
  for (; k < kNumKernels && k < max; k++) out[k] = v->last_ms[k];
  return k;
}

int p2v_verify_batch(const p2v_circuit* c, const uint64_t* proofs, size_t n, int8_t* results, int device) {
  if (!c || (n && (!proofs || !results))) return fail(P2V_E_ARG, "null argument");
  return p2v_verify_batch_devices(c, proofs, n, results, &device, 1, 0);
}

}  // extern "C"
