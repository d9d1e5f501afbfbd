// kernels.hip — gfx950 kernels of the batch verifier (everything except the vanishing /
// gate-constraint kernel, which lives in vanish.hip).
//
// Data layout: the caller's proof-major batch ([n][words]) is read in place (devcommon.h ld();
// P2V_PROOF_MAJOR=0 builds the older transposed [word][B] form).  In every kernel lane i of a
// wave handles proof (64*pb + i) and all other indices (query, tree, step, word) are
// wave-uniform: control flow never diverges and the Poseidon round constants are scalar operands.
//
//   k_transpose   proof-major -> SoA (P2V_PROOF_MAJOR=0 only)
//   k_phase1      transcript waves (a row or quad of lanes per proof, ~115 sequential permutations,
//                 Challenge/Verifier.hs:58-103 + Challenge/FRI.hs:65-104) run in the SAME
//                 launch as the leaf-hash waves (one lane per (proof, query, tree) sponge,
//                 Hash/Sponge.hs:26-31) which do not depend on the challenges
//   k_merkle      path compression (Hash/Merkle.hs:27-42) for the 4 initial trees and every
//                 FRI step tree, one lane per (proof, query, tree)
//   k_fri         combineInitial + folding steps + final polynomial, one lane per
//                 (proof, query)  (Plonk/FRI.hs:151-407)
//   k_status      reference evaluation order -> int8 status (+ optional trace)
#include "devcommon.h"
#include "qposeidon.h"
#include "rposeidon.h"
#include "pposeidon.h"
#include "lposeidon.h"

using namespace p2d;
using gl::E;

// ------------------------------------------------------------------------ transpose
extern "C" __global__ void __launch_bounds__(256) k_transpose(const uint64_t* __restrict__ in, int64_t words, int n,
                                                              uint64_t* __restrict__ out, int B) {
  __shared__ uint64_t tile[64][65];
  const int64_t w0 = (int64_t)blockIdx.x * 64;
  const int p0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
  for (int k = ty; k < 64; k += 4) {
    int p = p0 + k; int64_t w = w0 + tx;
    tile[k][tx] = (p < n && w < words) ? in[(int64_t)p * words + w] : 0;
  }
  __syncthreads();
  for (int k = ty; k < 64; k += 4) {
    int64_t w = w0 + k; int p = p0 + tx;
    if (w < words) out[w * B + p] = tile[tx][k];
  }
}

// ------------------------------------------------------------------------ helpers
#ifndef P2V_LEAF_PREFETCH
#define P2V_LEAF_PREFETCH 1   // leaf sponges: each block's words loaded one permutation ahead (0: two blocks per trip, round 5)
#endif
#ifndef P2V_LEAF_FOLD
#define P2V_LEAF_FOLD 1   // the folded zh round 0 (poseidon.h P2V_ZH_FOLD) on each leaf's first block
#endif
__device__ __forceinline__ void leaf_hash_unit(const DevCircuit& c, int unit, int lane) {
  const int NPB = c.B >> 6;
  const int pb = unit % NPB, qt = unit / NPB;   // (position, query)-major: costly trees first
  const int q = qt % c.Q, t = c.leaf_order[qt / c.Q];
  const int p = pb * 64 + lane;
  const int64_t base = c.q0 + (int64_t)q * c.qstride;
  int64_t off; int len;
  if (t < 4) { off = base + c.leaf[t]; len = c.lwidth[t]; }
  else { int s = t - 4; off = base + c.step_evals[s]; len = 2 << c.arity[s]; }
  uint64_t st[12];
#pragma unroll
  for (int i = 0; i < 12; i++) st[i] = 0;
  if (c.noop_leaves && len <= 4) {   // P2V_EXT_HASH_OR_NOOP: plonky2 hash_or_noop, the leaf zero-padded
#pragma unroll
    for (int j = 0; j < 4; j++) if (j < len) st[j] = ld(c, off + j, p);
    len = 0;
  }
#if P2V_LEAF_PREFETCH
  // sponge, overwrite mode, no padding.  One 8-word block per trip, its words loaded one
  // permutation ahead (during the previous block's permutation, into the registers that block has
  // just been copied out of), so no wave waits for its row at the top of a trip; one permutation
  // call site (round 6)
  uint64_t nb[8];
#pragma unroll
  for (int j = 0; j < 8; j++) nb[j] = j < len ? ld(c, off + j, p) : 0;
  for (int i = 0; i < len; i += 8) {
    const int k = len - i;
#pragma unroll
    for (int j = 0; j < 8; j++) if (j < k) st[j] = nb[j];
#pragma unroll
    for (int j = 0; j < 8; j++) nb[j] = 8 + j < k ? ld(c, off + i + 8 + j, p) : 0;
    // words the rest of the sponge reads: the digest (0..3) after the last block, else the
    // words the next block does not overwrite (nx.. 11); state words 8..11 are 0 in block 0
    const int nx = k - 8;
    p2::permute_dev<P2V_LEAF_FOLD != 0>(st, i == 0, nx <= 0 ? 1 : (nx >= 8 ? 4 : ((7 << (nx >> 2)) & 7)));
  }
#else
  // sponge, overwrite mode, no padding.  Two 8-word blocks per trip, both loaded up front: each
  // lane streams its own proof's row, so the loads of one trip cover a whole 128-B line while
  // it is resident in L2 (one block per load left half of every line to be fetched again after
  // the permutation, profiles/r02_fetch_calibration.json)
  for (int i = 0; i < len; i += 16) {
    const int k = len - i;
    uint64_t nb[8];
#pragma unroll
    for (int j = 0; j < 8; j++) if (j < k) st[j] = ld(c, off + i + j, p);
#pragma unroll
    for (int j = 0; j < 8; j++) nb[j] = 8 + j < k ? ld(c, off + i + 8 + j, p) : 0;
    // words the rest of the sponge reads: the digest (0..3) after the last block, else the
    // words the next block does not overwrite (nx.. 11); state words 8..11 are 0 in block 0
    int nx = k - 8;
    p2::permute_dev<P2V_LEAF_FOLD != 0>(st, i == 0, nx <= 0 ? 1 : (nx >= 8 ? 4 : ((7 << (nx >> 2)) & 7)));
    if (k > 8) {
#pragma unroll
      for (int j = 0; j < 8; j++) if (8 + j < k) st[j] = nb[j];
      nx = k - 16;
      p2::permute_dev<false>(st, false, nx <= 0 ? 1 : (nx >= 8 ? 4 : ((7 << (nx >> 2)) & 7)));
    }
  }
#endif
  uint64_t* dst = c.leafdig + ((int64_t)(q * c.T + t) * 4) * c.B + p;
#pragma unroll
  for (int i = 0; i < 4; i++) dst[(int64_t)i * c.B] = st[i];
}

// The transcript (Challenge/Verifier.hs:58-103, Challenge/FRI.hs:65-104) is a fixed
// sequence of absorbs and squeezes for a given circuit; the host compiles it into an op
// program and this loop interprets it with ONE permutation call site.  Each proof's duplex
// state is spread over a 16-lane row (rposeidon.h): the ~115 permutations form a strictly
// serial chain, so per-permutation latency, not throughput, is what counts.  Lane L owns
// state word L, so an absorbed chunk is one load per lane, issued before the pending
// permutation so that its latency hides behind it.
template <int D>
__device__ __forceinline__ uint64_t row_up(uint64_t v, bool plus) {   // value of lane L + D (mod 16)
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  const uint32_t l = plus ? rp::ror32<D>(lo) : rp::ror32<16 - D>(lo);
  const uint32_t h = plus ? rp::ror32<D>(hi) : rp::ror32<16 - D>(hi);
  return ((uint64_t)h << 32) | l;
}
template <int D>
__device__ __forceinline__ E row_fold(E h, E ad, bool plus) {   // h_L + alpha^D h_{L+D}
  return gl::eadd(h, gl::emul(ad, E{row_up<D>(h.a, plus), row_up<D>(h.b, plus)}));
}

// sum_m y_{S m + lane} * as^m over the F^2 openings at `off` (n of them), Horner from the top;
// eight terms' loads are issued ahead of their multiply-adds so the HBM latency overlaps the chain
template <int S>
__device__ __forceinline__ E horner_strided(const DevCircuit& c, int64_t off, int64_t n, int lane, int p, E as) {
  const int64_t M = (n + S - 1) / S;
  E h = gl::e0();
  for (int64_t m0 = M - 1; m0 >= 0; m0 -= 8) {
    E ys[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int64_t i = S * (m0 - u) + lane;
      ys[u] = (m0 - u >= 0 && i < n) ? lde(c, off + 2 * i, p) : gl::e0();
    }
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (m0 - u >= 0) h = gl::eadd(gl::emul(h, as), ys[u]);
  }
  return h;
}

// the row form's permutation: lposeidon.h (round 5: LDS exchange, merged partial blocks; 8.1-8.6 us
// per dependent permutation against 11.7-12.3 us for the DPP form of rposeidon.h,
// profiles/r05e_lrow_chain.txt; round 6: chain rows on the idle lanes, 6.6-6.8 us,
// profiles/r06p_row_par.txt); P2V_ROW_LAT=0 rebuilds the DPP form
#ifndef P2V_ROW_LAT
#define P2V_ROW_LAT 1
#endif
#if P2V_ROW_LAT
#define ROW_PERMUTE(x) lp::permute((x), LR, TL)
#else
#define ROW_PERMUTE(x) rp::permute((x), R, TQ)
#endif
__device__ __forceinline__ void transcript_row(const DevCircuit& c, int p, const rp::Row& R, const lp::Row& LR, const qp::TLds& TQ,
                                               const lp::TLdsL& TL) {
  (void)LR; (void)TQ; (void)TL;
  const int L = R.L;
  // public inputs hash, Hash/Sponge.hs:26-31 (sponge [] = zero digest)
  uint64_t x = 0;
  for (int i = 0; i < c.num_pis; i += 8) {
    const int k = c.num_pis - i;
    if (L < 8 && L < k) x = ld(c, c.pis + i + L, p);
    x = ROW_PERMUTE(x);
  }
  uint64_t pih[4];
#pragma unroll
  for (int w = 0; w < 4; w++) {
    pih[w] = rp::get_word(x, w);
    if (L == 0) chal(c, CH_PI(c) + w, p) = pih[w];
  }
  x = 0;
  int nbuf = 0, outpos = -1;
  bool absorbing = true;
  const uint64_t qmask = (1ULL << c.lde_bits) - 1;
  uint64_t fa0 = 0, fa1 = 0;   // FRI alpha, kept in registers for the reduced openings below
  for (int o = 0; o < c.ntops; o++) {
    const int type = c.tops[3 * o], a = c.tops[3 * o + 1], n = c.tops[3 * o + 2];
    if (type == TOP_COPY) {   // mkLookupDeltaList (betas ++ gammas ++ ...), Challenge/Verifier.hs:36-40,82-86
      if (L == 0) for (int k = 0; k < n; k++) chal(c, a + k, p) = chal(c, a - 3 * c.r + k, p);
      continue;
    }
    if (type == TOP_ZERO) {
      if (L == 0) for (int k = 0; k < n; k++) chal(c, a + k, p) = 0;
      continue;
    }
    if (type <= TOP_ABSORB_DIGEST) {   // absorb n words, chunk by chunk (lazy duplex, Challenge/Pure.hs:38-69)
      if (!absorbing) { absorbing = true; nbuf = 0; }
      for (int k = 0; k < n;) {
        const int start = nbuf == 8 ? 0 : nbuf;
        const int take = (8 - start) < (n - k) ? (8 - start) : (n - k);
        const int j = k + L - start;   // this lane's word of the chunk
        const bool mine = L >= start && L < start + take;
        uint64_t v = 0;
        if (type == TOP_ABSORB_SOA) { if (mine) v = ld(c, (int64_t)a + j, p); }
        else if (type == TOP_ABSORB_PIH) { const int w = j & 3; v = w == 0 ? pih[0] : w == 1 ? pih[1] : w == 2 ? pih[2] : pih[3]; }
        else v = c.digest[j & 3];
        if (nbuf == 8) { x = ROW_PERMUTE(x); nbuf = 0; }   // overwrite mode: the rate part is replaced
        if (mine) x = v;
        nbuf += take;
        k += take;
      }
      continue;
    }
    for (int k = 0; k < n; k++) {   // squeeze: output order state[7], state[6], ... (reverse of take 8)
      if (absorbing || outpos < 0) { x = ROW_PERMUTE(x); absorbing = false; outpos = 7; }
      uint64_t w = rp::get_word(x, outpos);
      outpos--;
      if (type == TOP_SQUEEZE_IDX) w &= qmask;
      if (a + k == CH_FRI_ALPHA(c)) fa0 = w;
      if (a + k == CH_FRI_ALPHA(c) + 1) fa1 = w;
      if (L == 0) chal(c, a + k, p) = w;
    }
  }
  // precomputeReducedOpenings, Plonk/FRI.hs:128-134: Y = sum alpha^i y_i.  Split over the
  // row: lane L sums the terms i = L (mod 16) in powers of alpha^16, then a 4-level DPP tree
  // forms sum_L alpha^L H_L in lane 0.
  const E alpha{fa0, fa1};
  const E a2 = gl::emul(alpha, alpha), a4 = gl::emul(a2, a2), a8 = gl::emul(a4, a4), a16 = gl::emul(a8, a8);
#pragma unroll
  for (int b = 0; b < 2; b++) {
    const int64_t n = b == 0 ? c.n_this : c.n_next, off = b == 0 ? c.o_const : c.o_zs_next;
    E h = horner_strided<16>(c, off, n, L, p, a16);
    h = row_fold<1>(h, alpha, R.plus);
    h = row_fold<2>(h, a2, R.plus);
    h = row_fold<4>(h, a4, R.plus);
    h = row_fold<8>(h, a8, R.plus);
    if (L == 0) { chal(c, (b == 0 ? CH_Y0(c) : CH_Y1(c)), p) = h.a; chal(c, (b == 0 ? CH_Y0(c) : CH_Y1(c)) + 1, p) = h.b; }
  }
}

// Quad form of the same transcript (qposeidon.h: 4 lanes per proof, 3 state words per
// lane).  Higher per-permutation latency than the row form but ~2.3x fewer issue slots in
// total, which is what matters once the batch is large enough that the transcript hides
// behind the leaf hashing sharing its launch (the host picks the form, see api.cpp).
__device__ __forceinline__ void transcript_quad(const DevCircuit& c, int p, int t, const qp::TLds& T) {
  // public inputs hash, Hash/Sponge.hs:26-31 (sponge [] = zero digest)
  uint64_t x[3] = {0, 0, 0};
  for (int i = 0; i < c.num_pis; i += 8) {
    const int k = c.num_pis - i;
    for (int j = 0; j < 8 && j < k; j++) qp::set_word(x, t, j, ld(c, c.pis + i + j, p));
    qp::permute(x, t, T);
  }
  uint64_t pih[4];
#pragma unroll
  for (int w = 0; w < 4; w++) {
    pih[w] = qp::get_word(x, w);
    if (t == 0) chal(c, CH_PI(c) + w, p) = pih[w];
  }
  x[0] = x[1] = x[2] = 0;
  int nbuf = 0, outpos = -1;
  bool absorbing = true;
  const uint64_t qmask = (1ULL << c.lde_bits) - 1;
  uint64_t fa0 = 0, fa1 = 0;   // FRI alpha, kept in registers for the reduced openings below
  for (int o = 0; o < c.ntops; o++) {
    const int type = c.tops[3 * o], a = c.tops[3 * o + 1], n = c.tops[3 * o + 2];
    if (type == TOP_COPY) {   // mkLookupDeltaList (betas ++ gammas ++ ...), Challenge/Verifier.hs:36-40,82-86
      if (t == 0) for (int k = 0; k < n; k++) chal(c, a + k, p) = chal(c, a - 3 * c.r + k, p);
      continue;
    }
    if (type == TOP_ZERO) {
      if (t == 0) for (int k = 0; k < n; k++) chal(c, a + k, p) = 0;
      continue;
    }
    if (type <= TOP_ABSORB_DIGEST) {   // absorb n words, chunk by chunk (lazy duplex, Challenge/Pure.hs:38-69)
      if (!absorbing) { absorbing = true; nbuf = 0; }
      for (int k = 0; k < n;) {
        const int start = nbuf == 8 ? 0 : nbuf;
        const int take = (8 - start) < (n - k) ? (8 - start) : (n - k);
        // lane t owns rate positions 3t..3t+2 (qposeidon.h); the chunk's loads are issued
        // before the permutation so their HBM latency hides under it
        uint64_t v[3];
        bool mine[3];
#pragma unroll
        for (int j = 0; j < 3; j++) {
          const int pos = 3 * t + j, w = k + pos - start;
          mine[j] = pos >= start && pos < start + take;
          v[j] = 0;
          if (type == TOP_ABSORB_SOA) { const uint64_t u = ld(c, (int64_t)a + (mine[j] ? w : 0), p); v[j] = mine[j] ? u : 0; }
          else if (type == TOP_ABSORB_PIH) { const int q = w & 3; v[j] = q == 0 ? pih[0] : q == 1 ? pih[1] : q == 2 ? pih[2] : pih[3]; }
          else v[j] = c.digest[w & 3];
        }
        if (nbuf == 8) { qp::permute(x, t, T); nbuf = 0; }   // overwrite mode: the rate part is replaced
#pragma unroll
        for (int j = 0; j < 3; j++) x[j] = mine[j] ? v[j] : x[j];
        nbuf += take;
        k += take;
      }
      continue;
    }
    for (int k = 0; k < n; k++) {   // squeeze
      const bool need = absorbing || outpos < 0;
      if (need) { qp::permute(x, t, T); absorbing = false; outpos = 7; }   // duplex / re-permute, Challenge/Pure.hs:38-69
      uint64_t w = qp::get_word(x, outpos);   // output order state[7], state[6], ... (reverse of take 8)
      outpos--;
      if (type == TOP_SQUEEZE_IDX) w &= qmask;
      if (a + k == CH_FRI_ALPHA(c)) fa0 = w;
      if (a + k == CH_FRI_ALPHA(c) + 1) fa1 = w;
      if (t == 0) chal(c, a + k, p) = w;
    }
  }
  // precomputeReducedOpenings, Plonk/FRI.hs:128-134: Y = sum alpha^i y_i.  Split over the
  // quad: lane t sums the terms i = t (mod 4) in powers of alpha^4, then Y = sum_t alpha^t H_t.
  const E alpha{fa0, fa1};
  const E al2 = gl::emul(alpha, alpha), al4 = gl::emul(al2, al2);
  E H[2];
#pragma unroll
  for (int b = 0; b < 2; b++) {
    const int64_t n = b == 0 ? c.n_this : c.n_next, off = b == 0 ? c.o_const : c.o_zs_next;
    H[b] = horner_strided<4>(c, off, n, t, p, al4);
  }
#pragma unroll
  for (int b = 0; b < 2; b++) {
    E h1{qp::bcast64(H[b].a, 1), qp::bcast64(H[b].b, 1)};
    E h2{qp::bcast64(H[b].a, 2), qp::bcast64(H[b].b, 2)};
    E h3{qp::bcast64(H[b].a, 3), qp::bcast64(H[b].b, 3)};
    E h0{qp::bcast64(H[b].a, 0), qp::bcast64(H[b].b, 0)};
    const E y = gl::eadd(h0, gl::emul(alpha, gl::eadd(h1, gl::emul(alpha, gl::eadd(h2, gl::emul(alpha, h3))))));
    if (t == 0) { chal(c, (b == 0 ? CH_Y0(c) : CH_Y1(c)), p) = y.a; chal(c, (b == 0 ? CH_Y0(c) : CH_Y1(c)) + 1, p) = y.b; }
  }
}

// Lane form of the same transcript: one lane per proof, the whole state in its registers, the
// throughput permutation (p2::permute_dev).  About half of the quad form's VALU instructions per
// proof (85.9 M against 169.4 M per 4096 proofs), but a chain ~3.5x longer (a lone wave issues its dependent permutation at its own
// latency): for pipelines with enough batches in flight to hide it (round 4, P2V_TRANSCRIPT=lane).
__device__ __forceinline__ void transcript_lane(const DevCircuit& c, int p) {
  uint64_t x[12];
#pragma unroll
  for (int i = 0; i < 12; i++) x[i] = 0;
  for (int i = 0; i < c.num_pis; i += 8) {   // public inputs hash, Hash/Sponge.hs:26-31
    const int k = c.num_pis - i;
#pragma unroll
    for (int j = 0; j < 8; j++) if (j < k) x[j] = ld(c, c.pis + i + j, p);
    p2::permute_dev<false>(x);
  }
  uint64_t pih[4];
#pragma unroll
  for (int w = 0; w < 4; w++) { pih[w] = x[w]; chal(c, CH_PI(c) + w, p) = pih[w]; }
#pragma unroll
  for (int i = 0; i < 12; i++) x[i] = 0;
  int nbuf = 0, outpos = -1;
  bool absorbing = true;
  const uint64_t qmask = (1ULL << c.lde_bits) - 1;
  uint64_t fa0 = 0, fa1 = 0;
  for (int o = 0; o < c.ntops; o++) {
    const int type = c.tops[3 * o], a = c.tops[3 * o + 1], n = c.tops[3 * o + 2];
    if (type == TOP_COPY) { for (int k = 0; k < n; k++) chal(c, a + k, p) = chal(c, a - 3 * c.r + k, p); continue; }
    if (type == TOP_ZERO) { for (int k = 0; k < n; k++) chal(c, a + k, p) = 0; continue; }
    if (type <= TOP_ABSORB_DIGEST) {   // absorb n words, chunk by chunk (lazy duplex, Challenge/Pure.hs:38-69)
      if (!absorbing) { absorbing = true; nbuf = 0; }
      for (int k = 0; k < n;) {
        const int start = nbuf == 8 ? 0 : nbuf;
        const int take = (8 - start) < (n - k) ? (8 - start) : (n - k);
        if (nbuf == 8) { p2::permute_dev<false>(x); nbuf = 0; }   // overwrite mode: the rate part is replaced
#pragma unroll
        for (int j = 0; j < 8; j++) {   // (loaded after the permutation: no registers held across it)
          const int w = k + j - start;
          if (j < start || j >= start + take) continue;
          if (type == TOP_ABSORB_SOA) x[j] = ld(c, (int64_t)a + w, p);
          else if (type == TOP_ABSORB_PIH) { const int q = w & 3; x[j] = q == 0 ? pih[0] : q == 1 ? pih[1] : q == 2 ? pih[2] : pih[3]; }
          else x[j] = c.digest[w & 3];
        }
        nbuf += take;
        k += take;
      }
      continue;
    }
    for (int k = 0; k < n; k++) {   // squeeze: output order state[7], state[6], ...
      if (absorbing || outpos < 0) { p2::permute_dev<false>(x); absorbing = false; outpos = 7; }
      uint64_t w;
      switch (outpos) {   // uniform: a switch, not a dynamically indexed (scratch) array
        case 0: w = x[0]; break;
        case 1: w = x[1]; break;
        case 2: w = x[2]; break;
        case 3: w = x[3]; break;
        case 4: w = x[4]; break;
        case 5: w = x[5]; break;
        case 6: w = x[6]; break;
        default: w = x[7]; break;
      }
      outpos--;
      if (type == TOP_SQUEEZE_IDX) w &= qmask;
      if (a + k == CH_FRI_ALPHA(c)) fa0 = w;
      if (a + k == CH_FRI_ALPHA(c) + 1) fa1 = w;
      chal(c, a + k, p) = w;
    }
  }
  // precomputeReducedOpenings, Plonk/FRI.hs:128-134: Y = sum alpha^i y_i, Horner from the top
  const E alpha{fa0, fa1};
#pragma unroll
  for (int b = 0; b < 2; b++) {
    const int64_t n = b == 0 ? c.n_this : c.n_next, off = b == 0 ? c.o_const : c.o_zs_next;
    const E y = horner_strided<1>(c, off, n, 0, p, alpha);
    chal(c, (b == 0 ? CH_Y0(c) : CH_Y1(c)), p) = y.a;
    chal(c, (b == 0 ? CH_Y0(c) : CH_Y1(c)) + 1, p) = y.b;
  }
}

// Pair form (pposeidon.h: 2 lanes per proof, 6 state words per lane): about half of the quad's
// instructions per proof at a shorter chain (round 4)
__device__ __forceinline__ void transcript_pair(const DevCircuit& c, int p, int t, const pp::TLdsP& T) {
  uint64_t x[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < c.num_pis; i += 8) {   // public inputs hash, Hash/Sponge.hs:26-31
    const int k = c.num_pis - i;
#pragma unroll
    for (int j = 0; j < 6; j++) {   // selects, not divergent stores: x stays in registers
      const int pos = 6 * t + j;
      const bool mine = pos < 8 && pos < k;
      const uint64_t v = ld(c, c.pis + i + (mine ? pos : 0), p);
      x[j] = mine ? v : x[j];
    }
    pp::permute(x, t, T);
  }
  uint64_t pih[4];
#pragma unroll
  for (int w = 0; w < 4; w++) {
    pih[w] = pp::get_word(x, w);
    if (t == 0) chal(c, CH_PI(c) + w, p) = pih[w];
  }
#pragma unroll
  for (int j = 0; j < 6; j++) x[j] = 0;
  int nbuf = 0, outpos = -1;
  bool absorbing = true;
  const uint64_t qmask = (1ULL << c.lde_bits) - 1;
  uint64_t fa0 = 0, fa1 = 0;
  for (int o = 0; o < c.ntops; o++) {
    const int type = c.tops[3 * o], a = c.tops[3 * o + 1], n = c.tops[3 * o + 2];
    if (type == TOP_COPY) { if (t == 0) for (int k = 0; k < n; k++) chal(c, a + k, p) = chal(c, a - 3 * c.r + k, p); continue; }
    if (type == TOP_ZERO) { if (t == 0) for (int k = 0; k < n; k++) chal(c, a + k, p) = 0; continue; }
    if (type <= TOP_ABSORB_DIGEST) {   // absorb n words, chunk by chunk (lazy duplex, Challenge/Pure.hs:38-69)
      if (!absorbing) { absorbing = true; nbuf = 0; }
      for (int k = 0; k < n;) {
        const int start = nbuf == 8 ? 0 : nbuf;
        const int take = (8 - start) < (n - k) ? (8 - start) : (n - k);
        // lane t owns rate positions 6t .. 6t+5 (lane 1: 6, 7); the chunk's loads before the
        // permutation so their latency hides under it
        uint64_t v[6];
        bool mine[6];
#pragma unroll
        for (int j = 0; j < 6; j++) {
          const int pos = 6 * t + j, w = k + pos - start;
          mine[j] = pos >= start && pos < start + take;
          v[j] = 0;
          if (type == TOP_ABSORB_SOA) { const uint64_t u = ld(c, (int64_t)a + (mine[j] ? w : 0), p); v[j] = mine[j] ? u : 0; }
          else if (type == TOP_ABSORB_PIH) { const int q = w & 3; v[j] = q == 0 ? pih[0] : q == 1 ? pih[1] : q == 2 ? pih[2] : pih[3]; }
          else v[j] = c.digest[w & 3];
        }
        if (nbuf == 8) { pp::permute(x, t, T); nbuf = 0; }   // overwrite mode: the rate part is replaced
#pragma unroll
        for (int j = 0; j < 6; j++) x[j] = mine[j] ? v[j] : x[j];
        nbuf += take;
        k += take;
      }
      continue;
    }
    for (int k = 0; k < n; k++) {   // squeeze: output order state[7], state[6], ...
      if (absorbing || outpos < 0) { pp::permute(x, t, T); absorbing = false; outpos = 7; }
      uint64_t w = pp::get_word(x, outpos);
      outpos--;
      if (type == TOP_SQUEEZE_IDX) w &= qmask;
      if (a + k == CH_FRI_ALPHA(c)) fa0 = w;
      if (a + k == CH_FRI_ALPHA(c) + 1) fa1 = w;
      if (t == 0) chal(c, a + k, p) = w;
    }
  }
  // precomputeReducedOpenings, Plonk/FRI.hs:128-134: lane t sums the terms i = t (mod 2) in
  // powers of alpha^2, then Y = H_0 + alpha H_1
  const E alpha{fa0, fa1};
  const E al2 = gl::emul(alpha, alpha);
#pragma unroll
  for (int b = 0; b < 2; b++) {
    const int64_t n = b == 0 ? c.n_this : c.n_next, off = b == 0 ? c.o_const : c.o_zs_next;
    const E h = horner_strided<2>(c, off, n, t, p, al2);
    const E h0{pp::bcast64(h.a, 0), pp::bcast64(h.b, 0)}, h1{pp::bcast64(h.a, 1), pp::bcast64(h.b, 1)};
    const E y = gl::eadd(h0, gl::emul(alpha, h1));
    if (t == 0) { chal(c, (b == 0 ? CH_Y0(c) : CH_Y1(c)), p) = y.a; chal(c, (b == 0 ? CH_Y0(c) : CH_Y1(c)) + 1, p) = y.b; }
  }
}

// the constant tables of the transcript forms, in LDS (qposeidon.h TLds, pposeidon.h TLdsP)
union TLdsAny { qp::TLds q; pp::TLdsP p; lp::TLdsL l; };

// one workgroup of transcripts: `tl` lanes per proof (16: row form, 4: quad form); FORM 1: the
// lane form, FORM 2: the pair form (kernels of their own, so that their register demand does
// not touch the others')
template <int FORM = 0>
__device__ __forceinline__ void transcript_block(const DevCircuit& c, int tl, TLdsAny& U) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  const qp::TLds& T = U.q;
  if constexpr (FORM == 1) {
    (void)tl; (void)T;
    if (g < c.B) transcript_lane(c, g);
  } else if constexpr (FORM == 2) {
    (void)tl;
    if ((g >> 1) < c.B) transcript_pair(c, g >> 1, g & 1, U.p);
  } else if (tl == 16) {
    rp::Row R;
    rp::init(R, threadIdx.x);
    lp::Row LR;
    lp::init(LR, U.l, threadIdx.x);
    if ((g >> 4) < c.B) transcript_row(c, g >> 4, R, LR, T, U.l);
  } else {
    if ((g >> 2) < c.B) transcript_quad(c, g >> 2, g & 3, T);
  }
}

// the constant tables of the transcript form in use (tl uniform: 16 the row form, else quad)
__device__ __forceinline__ void tlds_fill_form(TLdsAny& T, int tl) {
  if (P2V_ROW_LAT && tl == 16) lp::tlds_fill(T.l, threadIdx.x, 256);
  else qp::tlds_fill(T.q, threadIdx.x, 256);
}

// ------------------------------------------------------------------------ phase 1
// blocks [0, nt_blocks): transcripts, `tl` lanes per proof (16: row form, 4: quad form) at
// raised wave priority so co-resident leaf waves do not stretch the serial chain; the
// rest: leaf hashing, 4 units per block.  Transcript blocks come first so they start first.
template <int FORM>
__device__ __forceinline__ void phase1_body(const DevCircuit& c, int nt_blocks, int tl) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ TLdsAny T;
  if ((int)blockIdx.x < nt_blocks) {   // block-uniform branch: the whole workgroup fills T
    __builtin_amdgcn_s_setprio(3);
    if constexpr (FORM == 0) tlds_fill_form(T, tl);
    if constexpr (FORM == 2) pp::tlds_fill(T.p, threadIdx.x, 256);
    transcript_block<FORM>(c, tl, T);
    return;
  }
  const int unit = ((int)blockIdx.x - nt_blocks) * 4 + wave;
  const int units = c.Q * c.T * (c.B >> 6);
  if (unit < units) leaf_hash_unit(c, unit, lane);
}
extern "C" __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_phase1(DevCircuit c, int nt_blocks, int tl) {
  phase1_body<0>(c, nt_blocks, tl);
}
// the lane-form transcript (P2V_TRANSCRIPT=lane) with the leaf hashing
extern "C" __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_phase1_lane(DevCircuit c, int nt_blocks, int tl) {
  phase1_body<1>(c, nt_blocks, tl);
}
// the pair-form transcript (P2V_TRANSCRIPT=pair) with the leaf hashing
extern "C" __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_phase1_pair(DevCircuit c, int nt_blocks, int tl) {
  phase1_body<2>(c, nt_blocks, tl);
}

// The same two halves as separate launches (env P2V_PHASE1=split, api.cpp): on their own the leaf
// waves run at the permutation's 72 VGPRs (7 waves/SIMD) instead of inheriting the transcript's
// 123 (4 waves/SIMD), the transcript on the side stream beside them.  Measured slower (serial
// 0.94x): the transcript chains then stretch to the leaf kernel's length; kept for measurement.
extern "C" __global__ void __launch_bounds__(256) k_transcript(DevCircuit c, int tl) {
  __builtin_amdgcn_s_setprio(3);
  __shared__ TLdsAny T;
  tlds_fill_form(T, tl);
  transcript_block(c, tl, T);
}
// the lane and pair forms on their own (the lookahead / split launches, api.cpp)
extern "C" __global__ void __launch_bounds__(256) k_transcript_lane(DevCircuit c, int tl) {
  __builtin_amdgcn_s_setprio(3);
  __shared__ TLdsAny T;
  transcript_block<1>(c, tl, T);
}
extern "C" __global__ void __launch_bounds__(256) k_transcript_pair(DevCircuit c, int tl) {
  __builtin_amdgcn_s_setprio(3);
  __shared__ TLdsAny T;
  pp::tlds_fill(T.p, threadIdx.x, 256);
  transcript_block<2>(c, tl, T);
}
// k_transcript with SIMDs of its own: the clobbers below make the kernel allocate the whole
// register file (256 VGPRs + 256 AGPRs), so each transcript wave is alone on its SIMD and issues
// at the single-wave latency (lat.hip) instead of sharing issue with co-resident leaf waves.
extern "C" __global__ void __launch_bounds__(256) k_transcript_x(DevCircuit c, int tl) {
  asm volatile("" ::: "v255", "a255");
  __shared__ TLdsAny T;
  tlds_fill_form(T, tl);
  transcript_block(c, tl, T);
}
extern "C" __global__ void __launch_bounds__(256) k_leaf(DevCircuit c) {
  const int unit = (int)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (unit < c.Q * c.T * (c.B >> 6)) leaf_hash_unit(c, unit, threadIdx.x & 63);
}

// ------------------------------------------------------------------------ Merkle paths
#ifndef P2V_MERKLE_WAVES
#define P2V_MERKLE_WAVES 6   // amdgpu_waves_per_eu on k_merkle: 77-79 VGPRs, 6 waves/SIMD, no scratch (serial +4.7 %, pipelined unchanged; 0 = compiler default, 5 waves)
#endif
#if P2V_MERKLE_WAVES > 0
#define P2V_MERKLE_ATTR __attribute__((amdgpu_waves_per_eu(P2V_MERKLE_WAVES)))
#else
#define P2V_MERKLE_ATTR
#endif
// Tree t of query q (lane proof p): path length, word offset of its siblings in the proof, and the
// query's leaf index in that tree (FRI step trees: the index shifted by the earlier arities)
__device__ __forceinline__ void tree_path(const DevCircuit& c, int t, int q, int p, int& depth, int64_t& poff, uint32_t& idx) {
  const int64_t base = c.q0 + (int64_t)q * c.qstride;
  idx = (uint32_t)chal(c, CH_QIDX(c) + q, p);
  if (t < 4) { depth = c.depth0; poff = base + c.path[t]; }
  else {
    const int s = t - 4;
    int sh = 0;
    for (int j = 0; j <= s; j++) sh += c.arity[j];
    idx >>= sh; depth = c.step_depth[s]; poff = base + c.step_path[s];
  }
}
__device__ __forceinline__ void load_leafdig(const DevCircuit& c, int t, int q, int p, uint64_t (&cur)[4]) {
  const uint64_t* src = c.leafdig + ((int64_t)(q * c.T + t) * 4) * c.B + p;
#pragma unroll
  for (int i = 0; i < 4; i++) cur[i] = src[(int64_t)i * c.B];
}
// One level of a path (Hash/Merkle.hs:27-42): even index compress(cur, sib), odd compress(sib, cur)
__device__ __forceinline__ void merkle_level(uint64_t (&cur)[4], const uint64_t (&sib)[4], bool odd) {
  uint64_t st[12];
#pragma unroll
  for (int i = 0; i < 4; i++) { st[i] = odd ? sib[i] : cur[i]; st[4 + i] = odd ? cur[i] : sib[i]; st[8 + i] = 0; }
  p2::permute_dev(st, true, 1);   // compress: words 8..11 enter as 0, only 0..3 are read
#pragma unroll
  for (int i = 0; i < 4; i++) cur[i] = st[i];
}
// merkle_level, and the next level's siblings (when `more`, wave-uniform) loaded into sib before
// the compression runs, so their latency hides behind it
__device__ __forceinline__ void merkle_level_next(const DevCircuit& c, uint64_t (&cur)[4], uint64_t (&sib)[4], bool odd,
                                                  bool more, int64_t nxt, int p) {
  uint64_t st[12];
#pragma unroll
  for (int i = 0; i < 4; i++) { st[i] = odd ? sib[i] : cur[i]; st[4 + i] = odd ? cur[i] : sib[i]; st[8 + i] = 0; }
  if (more) {
#pragma unroll
    for (int i = 0; i < 4; i++) sib[i] = ld(c, nxt + i, p);
  }
  p2::permute_dev(st, true, 1);
#pragma unroll
  for (int i = 0; i < 4; i++) cur[i] = st[i];
}
// cap_roots !! (idx >> depth) == the path's root
__device__ __forceinline__ bool cap_ok(const DevCircuit& c, int t, uint32_t idx, const uint64_t (&cur)[4], int p) {
  bool ok = idx < (uint32_t)c.cap_len;
  const uint32_t ci = ok ? idx : 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint64_t root;
    if (t == 0) root = c.cs_cap[ci * 4 + i];
    else if (t == 1) root = ld(c, c.wcap + ci * 4 + i, p);
    else if (t == 2) root = ld(c, c.zcap + ci * 4 + i, p);
    else if (t == 3) root = ld(c, c.qcap + ci * 4 + i, p);
    else root = ld(c, c.ccaps + (int64_t)(t - 4) * 4 * c.cap_len + ci * 4 + i, p);
    ok = ok && (root == cur[i]);
  }
  return ok;
}
// The whole path of (tree t, query q, proof p) against its cap entry
__device__ __forceinline__ bool path_ok(const DevCircuit& c, int t, int q, int p) {
  int depth; int64_t poff; uint32_t idx;
  tree_path(c, t, q, p, depth, poff, idx);
  uint64_t cur[4];
  load_leafdig(c, t, q, p, cur);
  for (int l = 0; l < depth; l++) {
    uint64_t sib[4];
    // one level's 32 B of siblings per load (proof-major: the line re-fetches this leaves hit
    // the Infinity Cache; tiled: whole 512-B rows per wave)
#pragma unroll
    for (int i = 0; i < 4; i++) sib[i] = ld(c, poff + 4 * l + i, p);
    merkle_level(cur, sib, idx & 1u);
    idx >>= 1;
  }
  return cap_ok(c, t, idx, cur, p);
}
__device__ __forceinline__ void merkle_unit(const DevCircuit& c) {
  const int lane = threadIdx.x & 63;
  const int unit = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int NPB = c.B >> 6;
  if (unit >= c.Q * c.T * NPB) return;
  const int pb = unit % NPB, qt = unit / NPB;   // (position, query)-major: deepest paths first
  const int q = qt % c.Q, t = c.merkle_order[qt / c.Q];
  const int p = pb * 64 + lane;
  c.mk_ok[(int64_t)(q * c.T + t) * c.B + p] = path_ok(c, t, q, p) ? 1 : 0;
}
extern "C" __global__ void __launch_bounds__(256) P2V_MERKLE_ATTR k_merkle(DevCircuit c) { merkle_unit(c); }

// ------------------------------------------------------------------------ Merkle paths, shared nodes once
// The Q queries of a proof open paths in the same trees, and two queries whose leaf indices agree
// above bit l hash the same parent at level l and everything above it: with 28 queries and cap 16
// a third of the top-level compressions repeat (13.4 % of all compressions of the standard proof).
// Each parent is hashed once, by its OWNER, the lowest query under it.  Query q owns the levels
// 0 .. e_q - 1 (a prefix: ownership only shrinks going up), so its work is one chain of e_q
// compressions; at level e_q < depth it meets its owner o (a lower query) and stops.
// Exact, whatever the proof holds.  q's reference path equals o's above level e_q when both
// compress the same pair there and read the same siblings above it, so for every follower q
//   (A) o's sibling at level e_q is q's node (same leaf, e_q = 0: the leaf digests are equal),
//   (B) q's sibling at level e_q is o's node (checked by o's chain, which knows its follower there),
//   (C) q's and o's siblings above level e_q are equal (same leaf: from level 0 on),
// and then q's status is o's.  A follower that fails a check is flagged and re-run from its own
// node at level e_q (k_merkle_fix), unless its root (the lowest query under its cap entry, whose
// chain is a whole path) failed: then k_status stops at that lower query whatever q's status is
// (Plonk/FRI.hs:105-117, queries in order).  Statuses and codes are the plain k_merkle's bit for
// bit; honest proofs fail no check.
//   k_merkle_plan     one lane per (tree class, query, proof): e, owner, followers, root; appends
//                     the chains to buckets by length, one global atomic per (work-group, bucket)
//                     (the 4 initial trees share the leaf index, each FRI step tree shifts it)
//   k_merkle_cse      one lane per chain, longest bucket first: waves of equal-length chains
//   k_merkle_fix      the flagged followers (a compact list; none for honest proofs)
//   k_merkle_resolve  one lane per (tree, query, proof): a follower takes the status of its
//                     first flagged or root ancestor
#ifndef P2V_CSE_PREFETCH
#define P2V_CSE_PREFETCH 0   // k_merkle_cse: 1 loads each level's siblings one compression ahead (96 VGPRs; measured no gain, profiles/r06l_prefetch.txt)
#endif
#ifndef P2V_CSE_ORDER
#define P2V_CSE_ORDER 0   // k_merkle_cse wave order: 0 bucket-major, longest first; 1 tile order merged over the buckets, XCD ranges (round 6, measured slower: see cse_wave)
#endif
#define P2V_CSE_CSTRIDE 16   // counters 64 B apart: atomics on one line serialise
__device__ __forceinline__ void class_shape(const DevCircuit& c, int cls, int& sh, int& depth) {
  sh = 0; depth = c.depth0;
  if (cls > 0) { for (int j = 0; j < cls; j++) sh += c.arity[j]; depth = c.step_depth[cls - 1]; }
}
__device__ __forceinline__ int tree_class(int t) { return t < 4 ? 0 : t - 3; }
#ifndef P2V_PLAN_WAVES
#define P2V_PLAN_WAVES 16   // waves per k_merkle_plan work-group (one global atomic per work-group and bucket)
#endif
extern "C" __global__ void __launch_bounds__(64 * P2V_PLAN_WAVES) k_merkle_plan(DevCircuit c) {
  __shared__ int hist[P2V_CSE_MAX_DEPTH + 1], gbase[P2V_CSE_MAX_DEPTH + 1];
  const int lane = threadIdx.x & 63;
  const int unit = blockIdx.x * P2V_PLAN_WAVES + (threadIdx.x >> 6);
  const int NPB = c.B >> 6, ncls = 1 + c.S;
  const int nb = c.depth0 + 1;
  if (threadIdx.x < (unsigned)nb) hist[threadIdx.x] = 0;
  __syncthreads();
  const bool unit_live = unit < ncls * c.Q * NPB;   // wave-uniform
  // tile-major (P2V_CSE_ORDER 1): a work-group's units are (tree class, query) pairs of one or two
  // 64-proof tiles, so the buckets fill tile by tile and k_merkle_cse's merged order follows the tiles
#if P2V_CSE_ORDER
  const int cq = unit % (ncls * c.Q), pb = unit / (ncls * c.Q);
#else
  const int pb = unit % NPB, cq = unit / NPB;
#endif
  const int q = cq % c.Q, cls = unit_live ? cq / c.Q : 0;
  const int p = pb * 64 + lane;
  const bool live = unit_live && p < c.n;
  int sh, depth;
  class_shape(c, cls, sh, depth);
  const int ntr = cls == 0 ? 4 : 1, t0 = cls == 0 ? 0 : 3 + cls;
  int e = 0, loc = 0, cnt = 0;
  if (live) {
    const uint64_t* qi = c.chal + (int64_t)CH_QIDX(c) * c.B + p;
    const uint32_t me = (uint32_t)qi[(int64_t)q * c.B] >> sh;
    // b = bit length of (index xor other's index): the two paths first share a parent at level b - 1
    int minb = 64, owner = q, root = q;
    bool have_root = false;
    uint64_t fol = ~0ULL;
    for (int k0 = 0; k0 < c.Q; k0 += 4) {
      uint32_t ik[4];
#pragma unroll
      for (int u = 0; u < 4; u++) ik[u] = k0 + u < c.Q ? (uint32_t)qi[(int64_t)(k0 + u) * c.B] >> sh : me;
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int k = k0 + u;
        if (k >= c.Q) break;
        const uint32_t x = me ^ ik[u];
        const int b = x ? 32 - __clz(x) : 0;
        if (!have_root && b <= depth) { root = k; have_root = true; }   // lowest query under the cap entry
        if (k < q) {
          if (b < minb) { minb = b; owner = k; }   // the lowest query sharing q's lowest shared parent
        } else if (k > q && b >= 1 && b <= depth) {
          // the lowest query in the sibling subtree at level b - 1 meets q there (if q owns that level)
          const int sl = 5 * (b - 1);
          if (((fol >> sl) & 31) == 31) fol ^= (uint64_t)(31 ^ k) << sl;
        }
      }
    }
    e = minb - 1 >= depth ? depth : (minb >= 1 ? minb - 1 : 0);
    if (e < depth) fol |= ~0ULL << (5 * e);   // levels q does not own: their owner checks the follower
    const int64_t pi = ((int64_t)cls * c.Q + q) * c.B + p;
    c.mplan[pi] = (uint32_t)e | (uint32_t)owner << 4 | (uint32_t)(minb == 0) << 9 | (uint32_t)root << 10;
    c.mfol[pi] = fol;
    for (int tt = 0; tt < ntr; tt++) {
      c.mbadq[((int64_t)(t0 + tt) * c.Q + q) * c.B + p] = 0;
      c.mk_ok[(int64_t)(q * c.T + t0 + tt) * c.B + p] = 0;   // written again by its chain, k_merkle_fix or k_merkle_resolve
    }
  }
  // the wave's lanes of one length: one run of that bucket, tree-major; a work-group's runs are
  // packed in LDS, then one global atomic per (work-group, bucket) places them
  uint64_t todo = __ballot(live);
  while (todo) {
    const int lead = __ffsll((unsigned long long)todo) - 1;
    const int eb = __shfl(e, lead);
    const uint64_t grp = __ballot(live && e == eb);
    const int n = __popcll(grp);
    int off = 0;
    if (lane == lead) off = atomicAdd(&hist[eb], n * ntr);
    off = __shfl(off, lead);
    if (live && e == eb) { loc = off + __popcll(grp & ((1ULL << lane) - 1)); cnt = n; }
    todo &= ~grp;
  }
  __syncthreads();
  if (threadIdx.x < (unsigned)nb) {
    const int h = hist[threadIdx.x];
    gbase[threadIdx.x] = h ? atomicAdd(&c.mcount[threadIdx.x * P2V_CSE_CSTRIDE], h) : 0;
  }
  __syncthreads();
  if (live) {
    uint32_t* dst = c.mchain + (int64_t)e * c.mcap;
    const int64_t base = (int64_t)gbase[e] + loc;
    for (int tt = 0; tt < ntr; tt++) {
      const int64_t pos = base + (int64_t)tt * cnt;
      if (pos < c.mcap) dst[pos] = (uint32_t)(t0 + tt) << 27 | (uint32_t)q << 22 | (uint32_t)p;   // (always: T Q B slots)
    }
  }
}
// Set the re-run flag of (t, q, p); true for the one caller that set it first.  A follower can fail
// two checks, its owner's (B) and its own (A)/(C), so the flag is one bit set by an atomic OR on the
// flag byte's 32-bit word (the flag array is [T][Q][B], B a multiple of 64: the word is in bounds).
__device__ __forceinline__ bool cse_flag_once(const DevCircuit& c, int t, int q, int p) {
  const size_t at = ((size_t)t * c.Q + q) * c.B + p;
  uint32_t* w = (uint32_t*)(c.mbadq + (at & ~(size_t)3));
  const uint32_t bit = 1u << (8 * (at & 3));
  return !(atomicOr(w, bit) & bit);
}
// a follower to re-run from its own node (k_merkle_fix): flag + one list entry.  Each (t, q, p) is
// listed at most once, so the list (capacity T Q B) cannot overflow; the guard below is therefore
// unreachable, and fails safe: an entry that could not be listed is rejected, never left to a stale
// status (k_merkle_plan also clears every status byte of the run)
__device__ __forceinline__ void cse_flag(const DevCircuit& c, int t, int q, int p) {
  if (!cse_flag_once(c, t, q, p)) return;
  const int at = atomicAdd(c.mfixn, 1);
  if (at < c.mcap) c.mfix[at] = (uint32_t)t << 27 | (uint32_t)q << 22 | (uint32_t)p;
  else c.mk_ok[(int64_t)(q * c.T + t) * c.B + p] = 0;
}
#ifndef P2V_CSE_INLINE
#define P2V_CSE_INLINE 0   // 1: a follower failing (A) / (C) re-runs its path in k_merkle_cse, not k_merkle_fix
#endif
// Which chains a wave of k_merkle_cse runs: bucket b (the chain length) and wave w of that bucket.
// P2V_CSE_ORDER 0 (round 5): bucket-major, longest first.  The 64 lanes of a wave are then runs of
// a few proofs from many 64-proof tiles, and the other proofs of every 128-B line they read sit in
// other buckets, read long after the line has left the XCD's L2: 6.6x the algorithmic bytes
// (profiles/r05z_pmc_traffic.json).  P2V_CSE_ORDER 1: the waves of all buckets
// merged in the order of the plan's tiles (the plan appends tile by tile), so every chain that
// reads a tile's rows -- all lengths, the owners' and followers' checks -- runs at about the same
// time, and each XCD takes one contiguous range of that order (blocks i, i + 8, ... share an XCD,
// MI355X_MICROARCH.md "Workgroup dispatch"), so those reads meet in one L2.  The merge is fraction
// r of every bucket in turn: waves [r nw_b / R, (r + 1) nw_b / R) of bucket b, longest first within
// a fraction; fraction r starts at sum_b floor(r nw_b / R), found by bisection.  Scalar work only.
#define P2V_CSE_LR 12   // R = 4096 fractions
__device__ __forceinline__ bool cse_wave(const DevCircuit& c, int& b, int64_t& w) {
  const int nbk = c.depth0 + 1;
  uint64_t nw[P2V_CSE_MAX_DEPTH + 1];
  uint64_t total = 0;
#pragma unroll
  for (int k = 0; k <= P2V_CSE_MAX_DEPTH; k++) {
    nw[k] = k < nbk ? ((uint64_t)min((int64_t)c.mcount[k * P2V_CSE_CSTRIDE], c.mcap) + 63) >> 6 : 0;
    total += nw[k];
  }
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
#if P2V_CSE_ORDER
  const uint64_t nblk = gridDim.x >> 3;   // the grid is a multiple of 8
  const uint64_t g = ((uint64_t)(blockIdx.x & 7) * nblk + (blockIdx.x >> 3)) * 4 + wv;
  if (g >= total) return false;
  auto start = [&](uint64_t r) {
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k <= P2V_CSE_MAX_DEPTH; k++) s += (r * nw[k]) >> P2V_CSE_LR;
    return s;
  };
  uint64_t r = 0;
  for (int step = P2V_CSE_LR - 1; step >= 0; step--) {
    const uint64_t rr = r | (1ull << step);
    if (start(rr) <= g) r = rr;
  }
  uint64_t off = g - start(r);   // < start(r + 1) - start(r): fraction r holds wave g
  b = -1;
#pragma unroll
  for (int k = P2V_CSE_MAX_DEPTH; k >= 0; k--) {
    const uint64_t lo = (r * nw[k]) >> P2V_CSE_LR, len = (((r + 1) * nw[k]) >> P2V_CSE_LR) - lo;
    if (b < 0) {
      if (off < len) { b = k; w = (int64_t)(lo + off); }
      else off -= len;
    }
  }
  return b >= 0;
#else
  int64_t g = (int64_t)blockIdx.x * 4 + wv;
#pragma unroll
  for (int k = P2V_CSE_MAX_DEPTH; k >= 0; k--) {   // longest chains first
    if (g >= 0 && g < (int64_t)nw[k]) { b = k; w = g; }
    g -= (int64_t)nw[k];
  }
  return g < 0;
#endif
}
__device__ __forceinline__ void merkle_chain(const DevCircuit& c) {
  const int lane = threadIdx.x & 63;
  int b = -1;
  int64_t w = 0;
  if (!cse_wave(c, b, w)) return;
  const int64_t cnt = min((int64_t)c.mcount[b * P2V_CSE_CSTRIDE], c.mcap);
  const int64_t slot = w * 64 + lane;
  if (slot >= cnt) return;
  const uint32_t id = c.mchain[(int64_t)b * c.mcap + slot];
  const int t = (int)(id >> 27), q = (int)((id >> 22) & 31), p = (int)(id & 0x3FFFFFu);
  const int64_t pi = ((int64_t)tree_class(t) * c.Q + q) * c.B + p;
  const uint32_t pw = c.mplan[pi];
  const uint64_t fol = c.mfol[pi];
  const int e = b;   // == pw & 15: the bucket is the chain length (wave-uniform)
  int depth; int64_t poff; uint32_t idx;
  tree_path(c, t, q, p, depth, poff, idx);
  uint64_t cur[4];
  load_leafdig(c, t, q, p, cur);
#if P2V_CSE_PREFETCH
  // each level's siblings are loaded one compression ahead, into the registers the compression
  // has just consumed, so no wave waits for them at the top of a level
  uint64_t sib[4];
  if (e > 0) {
#pragma unroll
    for (int i = 0; i < 4; i++) sib[i] = ld(c, poff + i, p);
  }
#endif
  for (int l = 0; l < e; l++) {
#if !P2V_CSE_PREFETCH
    uint64_t sib[4];
#pragma unroll
    for (int i = 0; i < 4; i++) sib[i] = ld(c, poff + 4 * l + i, p);
#endif
    const int f = (int)((fol >> (5 * l)) & 31);
    if (f != 31) {   // (B): the follower meeting this path here holds this node as its sibling
      const int64_t fo = poff + (int64_t)(f - q) * c.qstride + 4 * l;
      bool bad = false;
#pragma unroll
      for (int i = 0; i < 4; i++) bad |= ld(c, fo + i, p) != cur[i];
      if (bad) cse_flag(c, t, f, p);
    }
#if P2V_CSE_PREFETCH
    merkle_level_next(c, cur, sib, idx & 1u, l + 1 < e, poff + 4 * (l + 1), p);
#else
    merkle_level(cur, sib, idx & 1u);
#endif
    idx >>= 1;
  }
  if (e == depth) {
    c.mk_ok[(int64_t)(q * c.T + t) * c.B + p] = cap_ok(c, t, idx, cur, p) ? 1 : 0;
    return;
  }
  uint64_t* nd = c.mnode + ((int64_t)(t * c.Q + q) * 4) * c.B + p;   // k_merkle_fix resumes here
#pragma unroll
  for (int i = 0; i < 4; i++) nd[(int64_t)i * c.B] = cur[i];
  const int owner = (int)((pw >> 4) & 31);
  const int64_t oo = poff + (int64_t)(owner - q) * c.qstride;   // the owner's siblings in this tree
  bool bad = false;
  int l0 = e + 1;
  if ((pw >> 9) & 1) {   // same leaf: equal digests, and (C) from level 0
    uint64_t od[4];
    load_leafdig(c, t, owner, p, od);
#pragma unroll
    for (int i = 0; i < 4; i++) bad |= od[i] != cur[i];
    l0 = 0;
  } else {   // (A)
#pragma unroll
    for (int i = 0; i < 4; i++) bad |= ld(c, oo + 4 * e + i, p) != cur[i];
  }
  for (int l = l0; l < depth; l++)   // (C)
#pragma unroll
    for (int i = 0; i < 4; i++) bad |= ld(c, poff + 4 * l + i, p) != ld(c, oo + 4 * l + i, p);
#if P2V_CSE_INLINE
  if (bad) {   // this lane's own data disagrees: its own path to the cap, here (k_merkle_resolve skips it)
    (void)cse_flag_once(c, t, q, p);   // (an entry (B) listed first re-runs the same path in k_merkle_fix)
    for (int l = e; l < depth; l++) {
      uint64_t sib[4];
#pragma unroll
      for (int i = 0; i < 4; i++) sib[i] = ld(c, poff + 4 * l + i, p);
      merkle_level(cur, sib, idx & 1u);
      idx >>= 1;
    }
    c.mk_ok[(int64_t)(q * c.T + t) * c.B + p] = cap_ok(c, t, idx, cur, p) ? 1 : 0;
  }
#else
  if (bad) cse_flag(c, t, q, p);
#endif
}
#ifndef P2V_CSE_WAVES
#define P2V_CSE_WAVES 5   // amdgpu_waves_per_eu on k_merkle_cse: 90 VGPRs, no spills; 6 (80 VGPRs, 40 B of spills
                          // outside the chain loop) measured 0.7-1.4 % slower pipelined (profiles/r05v_cse_waves.txt)
#endif
extern "C" __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(P2V_CSE_WAVES))) k_merkle_cse(DevCircuit c) { merkle_chain(c); }
// The flagged followers, each from its own node at its meeting level to its cap entry: a short
// list (none for honest proofs) on the batch's critical path, so in the row form of the
// permutation (lposeidon.h: 16 lanes per path, ~8.5 us per dependent compression against ~20 us
// for one lane), grid-stride over the list rows (the list length is read once)
// One listed follower in the lane form (one lane per entry): a long list (adversarial batches of
// garbage proofs flag about half of all paths) costs about one k_merkle, not list/rows passes of
// the latency form
__device__ __forceinline__ void merkle_fix_lane(const DevCircuit& c, int64_t k) {
  const uint32_t id = c.mfix[k];
  const int t = (int)(id >> 27), q = (int)((id >> 22) & 31), p = (int)(id & 0x3FFFFFu);
  const uint32_t pw = c.mplan[((int64_t)tree_class(t) * c.Q + q) * c.B + p];
  uint8_t* mk = c.mk_ok + (int64_t)t * c.B + p;
  const int64_t qs = (int64_t)c.T * c.B;
  if (!mk[(int64_t)((pw >> 10) & 31) * qs]) { mk[q * qs] = 0; return; }   // a lower query fails first
  const int e = (int)(pw & 15);
  int depth; int64_t poff; uint32_t idx;
  tree_path(c, t, q, p, depth, poff, idx);
  uint64_t cur[4];
  const uint64_t* nd = c.mnode + ((int64_t)(t * c.Q + q) * 4) * c.B + p;
#pragma unroll
  for (int i = 0; i < 4; i++) cur[i] = nd[(int64_t)i * c.B];
  idx >>= e;
  for (int l = e; l < depth; l++) {
    uint64_t sib[4];
#pragma unroll
    for (int i = 0; i < 4; i++) sib[i] = ld(c, poff + 4 * l + i, p);
    merkle_level(cur, sib, idx & 1u);
    idx >>= 1;
  }
  mk[q * qs] = cap_ok(c, t, idx, cur, p) ? 1 : 0;
}
extern "C" __global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) k_merkle_fix(DevCircuit c) {
  __shared__ TLdsAny T;
  const int64_t nfix = min((int64_t)*c.mfixn, c.mcap);
  if (nfix > (int64_t)gridDim.x * 16) {   // more entries than latency rows: one lane per entry (grid-uniform)
    const int64_t lanes = (int64_t)gridDim.x * 256;
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < nfix; k += lanes) merkle_fix_lane(c, k);
    return;
  }
  if ((int64_t)blockIdx.x * 16 >= nfix) return;   // block-uniform: no entry for this block's rows (honest batches: all)
  tlds_fill_form(T, 16);
  __builtin_amdgcn_s_setprio(3);
  rp::Row R;
  rp::init(R, threadIdx.x);
  lp::Row LR;
  lp::init(LR, T.l, threadIdx.x);
  const qp::TLds& TQ = T.q;
  const lp::TLdsL& TL = T.l;
  (void)LR; (void)TQ; (void)TL;
  const int L = R.L;
  const int64_t rows = (int64_t)gridDim.x * 16;
  for (int64_t k = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4; k < nfix; k += rows) {   // row-uniform
    const uint32_t id = c.mfix[k];
    const int t = (int)(id >> 27), q = (int)((id >> 22) & 31), p = (int)(id & 0x3FFFFFu);
    const uint32_t pw = c.mplan[((int64_t)tree_class(t) * c.Q + q) * c.B + p];
    uint8_t* mk = c.mk_ok + (int64_t)t * c.B + p;
    const int64_t qs = (int64_t)c.T * c.B;
    if (!mk[(int64_t)((pw >> 10) & 31) * qs]) {   // a lower query fails first
      if (L == 0) mk[q * qs] = 0;
      continue;
    }
    const int e = (int)(pw & 15);
    int depth; int64_t poff; uint32_t idx;
    tree_path(c, t, q, p, depth, poff, idx);
    uint64_t cur = L < 4 ? c.mnode[((int64_t)(t * c.Q + q) * 4 + L) * c.B + p] : 0;
    idx >>= e;
    for (int l = e; l < depth; l++) {   // as k_merkle_row
      const uint64_t sib = L < 8 ? ld(c, poff + 4 * l + (L & 3), p) : 0;
      const uint64_t c0 = rp::get_word(cur, 0), c1 = rp::get_word(cur, 1), c2 = rp::get_word(cur, 2), c3 = rp::get_word(cur, 3);
      const uint64_t cb = L == 4 ? c0 : L == 5 ? c1 : L == 6 ? c2 : c3;
      const bool odd = idx & 1u;
      const uint64_t x = L < 4 ? (odd ? sib : cur) : L < 8 ? (odd ? cb : sib) : 0;
      cur = ROW_PERMUTE(x);
      idx >>= 1;
    }
    bool ok = idx < (uint32_t)c.cap_len;
    const uint32_t ci = ok ? idx : 0;
    uint64_t root = 0;
    if (L < 4) {
      if (t == 0) root = c.cs_cap[ci * 4 + L];
      else if (t == 1) root = ld(c, c.wcap + ci * 4 + L, p);
      else if (t == 2) root = ld(c, c.zcap + ci * 4 + L, p);
      else if (t == 3) root = ld(c, c.qcap + ci * 4 + L, p);
      else root = ld(c, c.ccaps + (int64_t)(t - 4) * 4 * c.cap_len + ci * 4 + L, p);
    }
    const uint64_t eq = (L >= 4 || root == cur) ? 1 : 0;
    ok = ok && (rp::get_word(eq, 0) & rp::get_word(eq, 1) & rp::get_word(eq, 2) & rp::get_word(eq, 3));
    if (L == 0) mk[q * qs] = ok ? 1 : 0;
  }
}
extern "C" __global__ void __launch_bounds__(256) k_merkle_resolve(DevCircuit c) {
  if (blockIdx.x == 0 && threadIdx.x <= (unsigned)c.depth0) c.mcount[threadIdx.x * P2V_CSE_CSTRIDE] = 0;   // the next run's
  if (blockIdx.x == 0 && threadIdx.x == 0) *c.mfixn = 0;
  const int lane = threadIdx.x & 63;
  const int unit = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int NPB = c.B >> 6;
  if (unit >= c.Q * c.T * NPB) return;
  const int pb = unit % NPB, qt = unit / NPB;
  const int q = qt % c.Q, t = qt / c.Q;
  const int p = pb * 64 + lane;
  if (p >= c.n) return;
  const int cls = tree_class(t);
  int sh, depth;
  class_shape(c, cls, sh, depth);
  const uint32_t* plan = c.mplan + (int64_t)cls * c.Q * c.B + p;
  const uint8_t* badq = c.mbadq + (int64_t)t * c.Q * c.B + p;
  uint32_t pw = plan[(int64_t)q * c.B];
  if ((int)(pw & 15) == depth || badq[(int64_t)q * c.B]) return;   // a root or a re-run follower: written
  // the first ancestor whose status is its own: a root chain or a re-run follower
  int a = (int)((pw >> 4) & 31);
  for (int hop = 0; hop < c.Q; hop++) {
    pw = plan[(int64_t)a * c.B];
    if ((int)(pw & 15) == depth || badq[(int64_t)a * c.B]) break;
    a = (int)((pw >> 4) & 31);
  }
  uint8_t* mk = c.mk_ok + (int64_t)t * c.B + p;
  const int64_t qs = (int64_t)c.T * c.B;
  mk[q * qs] = mk[a * qs];
}

// Latency mode (small batches, api.cpp): the same paths in the row form of the permutation
// (lposeidon.h: 16 lanes per path, lane L < 12 holding word L), four paths per wave.  A path is a
// chain of dependent compressions; one lane per path issues at the single-wave latency (~53 us
// per compression, lat.hip), the row form at ~14 us.  Row = path (tree position, query, proof),
// proofs fastest; lanes 0..3 hold the path value, lanes 4..7 the other half of the input.
extern "C" __global__ void __launch_bounds__(256) k_merkle_row(DevCircuit c) {
  __shared__ TLdsAny T;
  tlds_fill_form(T, 16);
  __builtin_amdgcn_s_setprio(3);   // the batch's critical path in this mode
  rp::Row R;
  rp::init(R, threadIdx.x);
  lp::Row LR;
  lp::init(LR, T.l, threadIdx.x);
  const qp::TLds& TQ = T.q;
  const lp::TLdsL& TL = T.l;
  (void)LR; (void)TQ; (void)TL;
  const int L = R.L;
  const int path = (int)((blockIdx.x * 256 + threadIdx.x) >> 4);
  const int npaths = c.Q * c.T * c.n;
  const bool live = path < npaths;   // idle rows still run the permutation (its DPP ops span the row)
  const int pp = live ? path : 0;
  const int p = pp % c.n, qt = pp / c.n;
  const int q = qt % c.Q, t = c.merkle_order[qt / c.Q];
  const int64_t base = c.q0 + (int64_t)q * c.qstride;
  uint32_t idx = (uint32_t)chal(c, CH_QIDX(c) + q, p);
  int depth; int64_t poff;
  if (t < 4) { depth = c.depth0; poff = base + c.path[t]; }
  else {
    const int s = t - 4;
    int sh = 0;
    for (int j = 0; j <= s; j++) sh += c.arity[j];
    idx >>= sh; depth = c.step_depth[s]; poff = base + c.step_path[s];
  }
  uint64_t cur = L < 4 ? c.leafdig[((int64_t)(q * c.T + t) * 4 + L) * c.B + p] : 0;
  for (int l = 0; l < depth; l++) {   // even index: compress(cur, sib), odd: compress(sib, cur)
    const uint64_t sib = L < 8 ? ld(c, poff + 4 * l + (L & 3), p) : 0;
    const uint64_t c0 = rp::get_word(cur, 0), c1 = rp::get_word(cur, 1), c2 = rp::get_word(cur, 2), c3 = rp::get_word(cur, 3);
    const uint64_t cb = L == 4 ? c0 : L == 5 ? c1 : L == 6 ? c2 : c3;
    const bool odd = idx & 1u;
    const uint64_t x = L < 4 ? (odd ? sib : cur) : L < 8 ? (odd ? cb : sib) : 0;
    cur = ROW_PERMUTE(x);   // lanes 0..3: the compression's output
    idx >>= 1;
  }
  bool ok = idx < (uint32_t)c.cap_len;
  const uint32_t ci = ok ? idx : 0;
  uint64_t root = 0;
  if (L < 4) {
    if (t == 0) root = c.cs_cap[ci * 4 + L];
    else if (t == 1) root = ld(c, c.wcap + ci * 4 + L, p);
    else if (t == 2) root = ld(c, c.zcap + ci * 4 + L, p);
    else if (t == 3) root = ld(c, c.qcap + ci * 4 + L, p);
    else root = ld(c, c.ccaps + (int64_t)(t - 4) * 4 * c.cap_len + ci * 4 + L, p);
  }
  const uint64_t eq = (L >= 4 || root == cur) ? 1 : 0;
  ok = ok && (rp::get_word(eq, 0) & rp::get_word(eq, 1) & rp::get_word(eq, 2) & rp::get_word(eq, 3));
  if (live && L == 0) c.mk_ok[(int64_t)(q * c.T + t) * c.B + p] = ok ? 1 : 0;
}

// ------------------------------------------------------------------------ FRI query
// foldCosetWith (Plonk/FRI.hs:263-279) for arity 2^AB: the coset values (received order v,
// bit-reversed coset order vals[rev k] = v[k]) are interpolated and evaluated at beta.
// c_k = sum_j vals_j w^{-jk} is a DIT FFT applied to v directly (v is already the
// bit-reversal of vals); P(beta) = (1/2^AB) sum_k c_k (beta/ofs)^k.
template <int AB>
__device__ __forceinline__ E fold_regs(const DevCircuit& c, int s, int64_t off, int p, E beta_over_ofs) {
  constexpr int AR = 1 << AB;
  E a[AR];
#pragma unroll
  for (int k = 0; k < AR; k++) a[k] = lde(c, off + 2 * k, p);
  const uint64_t* tw = c.twiddles + 256 * s;   // omega^{-j}
#pragma unroll
  for (int len = 2; len <= AR; len <<= 1) {
#pragma unroll
    for (int i = 0; i < AR; i += len) {
#pragma unroll
      for (int k = 0; k < len / 2; k++) {
        E u = a[i + k], v = a[i + k + len / 2];
        if (k != 0) v = gl::escale(tw[k * (AR / len)], v);
        a[i + k] = gl::eadd(u, v);
        a[i + k + len / 2] = gl::esub(u, v);
      }
    }
  }
  E acc = gl::e0();
#pragma unroll
  for (int k = AR - 1; k >= 0; k--) acc = gl::eadd(gl::emul(acc, beta_over_ofs), a[k]);
  return gl::escale(c.inv_arity[s], acc);
}
// Arity 16 in two halves, so that only 8 F^2 values are live (k_fri's 96-VGPR budget held all 16
// with 152 B/lane of scratch).  The DIT's first three stages act on v[0..7] and v[8..15] alone,
// giving the 8-point transforms E, O (twiddles w^{-2jk}); the last stage is c_k = E_k + w^{-k} O_k,
// c_{k+8} = E_k - w^{-k} O_k.  With b = beta/ofs:
//   sum_{k<16} c_k b^k = (1 + b^8) sum_{k<8} E_k b^k + (1 - b^8) sum_{k<8} O_k (w^{-1} b)^k.
template <int AR>
__device__ __forceinline__ E dft8_horner(const DevCircuit& c, const uint64_t* tw, int64_t off, int p, E b) {
  E a[8];
#pragma unroll
  for (int k = 0; k < 8; k++) a[k] = lde(c, off + 2 * k, p);
#pragma unroll
  for (int len = 2; len <= 8; len <<= 1) {
#pragma unroll
    for (int i = 0; i < 8; i += len) {
#pragma unroll
      for (int k = 0; k < len / 2; k++) {
        E u = a[i + k], v = a[i + k + len / 2];
        if (k != 0) v = gl::escale(tw[k * (AR / len)], v);
        a[i + k] = gl::eadd(u, v);
        a[i + k + len / 2] = gl::esub(u, v);
      }
    }
  }
  E acc = gl::e0();
#pragma unroll
  for (int k = 7; k >= 0; k--) acc = gl::eadd(gl::emul(acc, b), a[k]);
  return acc;
}
__device__ __forceinline__ E fold16_halves(const DevCircuit& c, int s, int64_t off, int p, E b) {
  const uint64_t* tw = c.twiddles + 256 * s;
  const E lo = dft8_horner<16>(c, tw, off, p, b);
  __builtin_amdgcn_sched_barrier(0);   // keep the halves apart: one half's 8 values live at a time
  const E hi = dft8_horner<16>(c, tw, off + 16, p, gl::escale(tw[1], b));
  const E b2 = gl::emul(b, b), b4 = gl::emul(b2, b2), b8 = gl::emul(b4, b4);
  const E one = gl::eb(1);
  const E acc = gl::eadd(gl::emul(gl::eadd(one, b8), lo), gl::emul(gl::esub(one, b8), hi));
  return gl::escale(c.inv_arity[s], acc);
}
// generic arity: direct O(arity^2) evaluation of the same interpolant
__device__ E fold_generic(const DevCircuit& c, int s, int ab, int64_t off, int p, E beta_over_ofs) {
  const int ar = 1 << ab;
  const uint64_t* tw = c.twiddles + 256 * s;
  E acc = gl::e0();
  for (int k = ar - 1; k >= 0; k--) {
    E ck = gl::e0();
    for (int j = 0; j < ar; j++) {
      const int jj = (int)gl::rev_bits(ab, (uint32_t)j);   // vals[j] = v[rev j]
      ck = gl::eadd(ck, gl::escale(tw[(j * k) & (ar - 1)], lde(c, off + 2 * jj, p)));
    }
    acc = gl::eadd(gl::emul(acc, beta_over_ofs), ck);
  }
  return gl::escale(c.inv_arity[s], acc);
}

// ---- combineInitial's reduceWithPowers (Goldilocks.hs:180-183, Plonk/FRI.hs:151-207):
// sum_v alpha^v y_v over a list of base-field leaf words (up to 5 contiguous segments of the
// query's leaves, ascending), alpha in F^2.  Round 4 ran one F^2 Horner step per word (a full
// emul, ~100 VALU).  Round 5: Horner in chunks of 8, g <- g alpha^8 + sum_{k<8} y_{j+k} alpha^k,
// with alpha^1..alpha^8 in registers; the inner sum's base-field products y alpha^k (2 per word,
// one per component) are accumulated unreduced in 128 + 3 bits and reduced once per chunk and
// component.  The same field element (exact arithmetic).
struct Acc3 { uint64_t lo, hi; uint32_t top; };   // lo + hi 2^64 + top 2^128
__device__ __forceinline__ void acc_mul(Acc3& A, uint64_t y, uint64_t c) {
  uint64_t h, l;
  gl::mul128(y, c, h, l);
  const uint64_t lo2 = A.lo + l;
  const uint64_t c0 = lo2 < l ? 1 : 0;
  const uint64_t hi2 = A.hi + h;
  const uint32_t c1 = hi2 < h ? 1u : 0u;
  const uint64_t hi3 = hi2 + c0;
  const uint32_t c2 = hi3 < c0 ? 1u : 0u;
  A.lo = lo2; A.hi = hi3; A.top += c1 + c2;
}
// lo + hi 2^64 + top 2^128 mod p, canonical: 2^128 == (2^32 - 1)^2 == -2^32 (mod p), top <= 8
__device__ __forceinline__ uint64_t acc_reduce(const Acc3& A) {
  return gl::sub(gl::reduce128(A.hi, A.lo), (uint64_t)A.top << 32);
}
struct Segs { int64_t off[5]; int n[5]; int ns; };
__device__ __forceinline__ int64_t seg_addr(const Segs& S, int v) {   // v wave-uniform: scalar code
  for (int s = 0; s < S.ns; s++) {
    if (v < S.n[s]) return S.off[s] + v;
    v -= S.n[s];
  }
  return S.off[0];
}
__device__ __forceinline__ E reduce_powers(const DevCircuit& c, const Segs& S, int p, E alpha, const E* ap) {
  int N = 0;
  for (int s = 0; s < S.ns; s++) N += S.n[s];
  E g = gl::e0();
  const int rem = N & 7;
  for (int v = N - 1; v >= N - rem; v--) g = gl::eadd(gl::emul(g, alpha), gl::eb(ld(c, seg_addr(S, v), p)));
  for (int j = N - rem - 8; j >= 0; j -= 8) {
    uint64_t y[8];
#pragma unroll
    for (int k = 0; k < 8; k++) y[k] = ld(c, seg_addr(S, j + k), p);
    Acc3 A{y[0], 0, 0}, B{0, 0, 0};   // alpha^0 = 1
#pragma unroll
    for (int k = 1; k < 8; k++) { acc_mul(A, y[k], ap[k].a); acc_mul(B, y[k], ap[k].b); }
    g = gl::eadd(gl::emul(g, ap[8]), E{acc_reduce(A), acc_reduce(B)});
  }
  return g;
}

// k_fri runs on the side stream beside k_merkle (see vanish.hip P2V_SIDE_WAVES): 5 waves per SIMD
// caps it at 96 VGPRs, so a wave fits where one k_merkle wave retired (0: compiler default, 122)
#ifndef P2V_FOLD16_HALVES
#define P2V_FOLD16_HALVES 1
#endif
#ifndef P2V_FRI_CHUNKED
#define P2V_FRI_CHUNKED 1   // combineInitial in chunks of 8 with unreduced product sums (round 5, above)
#endif
#ifndef P2V_FRI_WAVES
#define P2V_FRI_WAVES 5
#endif
#if P2V_FRI_WAVES > 0
#define P2V_FRI_ATTR __attribute__((amdgpu_waves_per_eu(P2V_FRI_WAVES)))
#else
#define P2V_FRI_ATTR
#endif
extern "C" __global__ void __launch_bounds__(256) P2V_FRI_ATTR k_fri(DevCircuit c) {
  const int lane = threadIdx.x & 63;
  const int unit = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int NPB = c.B >> 6;
  if (unit >= c.Q * NPB) return;
  __builtin_amdgcn_s_setprio(2);   // side stream, concurrent with k_merkle (see k_vanish)
  const int pb = unit % NPB, q = unit / NPB;
  const int p = pb * 64 + lane;
  const int64_t base = c.q0 + (int64_t)q * c.qstride;
  const int r = c.r;
  uint32_t idx = (uint32_t)chal(c, CH_QIDX(c) + q, p);
  const E alpha = chal_e(c, CH_FRI_ALPHA(c), p);
  const E zeta = chal_e(c, CH_ZETA(c), p);
  // combineInitial, Plonk/FRI.hs:151-207.  firstBatch = consts|sigmas, wires, pp part,
  // quotient, lookup part; secondBatch = first r of the pp part, lookup part.
  const int npp_all = r * ((c.num_routed + c.qdf - 1) / c.qdf);
  const int64_t l0 = base + c.leaf[0], l1 = base + c.leaf[1], l2 = base + c.leaf[2], l3 = base + c.leaf[3];
#if P2V_FRI_CHUNKED
  // ascending lists (the Horner of round 4 below walks them from the top): firstBatch =
  // leaf0 | leaf1 | leaf2[0, npp_all) | leaf3 | leaf2[npp_all, w2); secondBatch = leaf2[0, r') |
  // leaf2[npp_all, w2)
  E ap[9];
  ap[0] = gl::eb(1); ap[1] = alpha;
#pragma unroll
  for (int k = 2; k <= 8; k++) ap[k] = gl::emul(ap[k - 1], alpha);
  const int rr = r < npp_all ? r : npp_all;
  Segs s0{{l0, l1, l2, l3, l2 + npp_all}, {c.width[0], c.width[1], npp_all, c.width[3], c.width[2] - npp_all}, 5};
  Segs s1{{l2, l2 + npp_all, 0, 0, 0}, {rr, c.width[2] - npp_all, 0, 0, 0}, 2};
  const E g0 = reduce_powers(c, s0, p, alpha, ap);
  const E g1 = reduce_powers(c, s1, p, alpha, ap);
#else
  E g0 = gl::e0(), g1 = gl::e0();
  for (int i = c.width[2] - 1; i >= npp_all; i--) g0 = gl::eadd(gl::emul(g0, alpha), gl::eb(ld(c, l2 + i, p)));
  for (int i = c.width[3] - 1; i >= 0; i--) g0 = gl::eadd(gl::emul(g0, alpha), gl::eb(ld(c, l3 + i, p)));
  for (int i = npp_all - 1; i >= 0; i--) g0 = gl::eadd(gl::emul(g0, alpha), gl::eb(ld(c, l2 + i, p)));
  for (int i = c.width[1] - 1; i >= 0; i--) g0 = gl::eadd(gl::emul(g0, alpha), gl::eb(ld(c, l1 + i, p)));
  for (int i = c.width[0] - 1; i >= 0; i--) g0 = gl::eadd(gl::emul(g0, alpha), gl::eb(ld(c, l0 + i, p)));
  for (int i = c.width[2] - 1; i >= npp_all; i--) g1 = gl::eadd(gl::emul(g1, alpha), gl::eb(ld(c, l2 + i, p)));
  for (int i = (r < npp_all ? r : npp_all) - 1; i >= 0; i--) g1 = gl::eadd(gl::emul(g1, alpha), gl::eb(ld(c, l2 + i, p)));
#endif
  const int len2 = (r < npp_all ? r : npp_all) + (c.width[2] - npp_all);
  const uint64_t px = gl::mul(gl::MULT_GEN, pow_root(c, c.lde_bits, gl::rev_bits(c.lde_bits, idx)));
  const uint64_t omega = c.root_pow2[32 - c.degree_bits];
  E d0 = gl::esub(gl::eb(px), zeta), d1 = gl::esub(gl::eb(px), gl::escale(omega, zeta));
  E i0, i1; einv2(d0, d1, i0, i1);
  const E one = gl::emul(gl::esub(g0, chal_e(c, CH_Y0(c), p)), i0);
  const E two = gl::emul(gl::esub(g1, chal_e(c, CH_Y1(c), p)), i1);
  E cur = gl::eadd(gl::emul(epow_u(alpha, (uint32_t)len2), one), two);
  uint64_t* qv = c.qvals + (int64_t)q * 6 * c.B + p;
  qv[0] = cur.a; qv[(int64_t)c.B] = cur.b;
  // folding steps, Plonk/FRI.hs:306-323
  uint32_t bits = 0;
  int logn = c.lde_bits;
  for (int s = 0; s < c.S; s++) {
    const int ab = c.arity[s];
    const int64_t eoff = base + c.step_evals[s];
    const uint32_t pos = idx & ((1u << ab) - 1);
    const E at = lde(c, eoff + 2 * pos, p);   // evals !! (idx mod arity)
    if (gl::eeq(at, cur)) bits |= 1u << s;
    // coset offset shift * eta^{rev((idx >> a) << a)}, and its inverse without an inversion
    const uint32_t start = gl::rev_bits(logn, (idx >> ab) << ab);
    const uint32_t nmask = (logn >= 32) ? 0xFFFFFFFFu : ((1u << logn) - 1);
    const uint64_t ofs_inv = gl::mul(c.step_shift_inv[s], pow_root(c, logn, (0u - start) & nmask));
    const E beta = chal_e(c, CH_FRI_BETA(c) + 2 * s, p);
    const E bo = gl::escale(ofs_inv, beta);
    E nv;
    switch (ab) {
      case 1: nv = fold_regs<1>(c, s, eoff, p, bo); break;
      case 2: nv = fold_regs<2>(c, s, eoff, p, bo); break;
      case 3: nv = fold_regs<3>(c, s, eoff, p, bo); break;
      case 4: nv = P2V_FOLD16_HALVES ? fold16_halves(c, s, eoff, p, bo) : fold_regs<4>(c, s, eoff, p, bo); break;
      default: nv = fold_generic(c, s, ab, eoff, p, bo); break;
    }
    cur = nv;
    idx >>= ab; logn -= ab;
  }
  qv[2 * (int64_t)c.B] = cur.a; qv[3 * (int64_t)c.B] = cur.b;
  // final polynomial at x = shift * eta^{rev idx}, Plonk/FRI.hs:288-291,325-327
  const uint64_t xf = gl::mul(c.step_shift[c.S], pow_root(c, logn, gl::rev_bits(logn, idx)));
  E acc = gl::e0();
  for (int k = c.final_len - 1; k >= 0; k--) acc = gl::eadd(gl::escale(xf, acc), lde(c, c.final_poly + 2 * k, p));
  qv[4 * (int64_t)c.B] = acc.a; qv[5 * (int64_t)c.B] = acc.b;
  if (gl::eeq(acc, cur)) bits |= 1u << 31;
  c.fri_bits[(int64_t)q * c.B + p] = bits;
}

// ------------------------------------------------------------------------ status
// verifyProof = eqs_ok && (pow_ok && and [rounds in order]) with the reference's error
// precedence inside a round (Plonk/Verifier.hs:62, Plonk/FRI.hs:370-407, 105-117, 306-313).
extern "C" __global__ void __launch_bounds__(256) k_status(DevCircuit c, int8_t* __restrict__ results, uint64_t* __restrict__ trace,
                                                           int64_t trace_words) {
  // a few short waves that gate the workspace's next batch: ahead of co-resident phase-1 waves
  __builtin_amdgcn_s_setprio(3);
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= c.n) return;
  const bool eqs_ok = c.van[p] != 0;
  const uint64_t resp = chal(c, CH_POW(c), p);
  const int pb = c.pow_bits;
  const uint64_t mask = pb <= 0 ? 0ULL : (pb >= 64 ? ~0ULL : (((1ULL << pb) - 1) << (64 - pb)));
  const bool pow_ok = (resp & mask) == 0;
  int8_t st = 1;
  if (!eqs_ok || !pow_ok) st = 0;
  else {
    for (int q = 0; q < c.Q && st == 1; q++) {
      const uint8_t* mk = c.mk_ok + (int64_t)q * c.T * c.B + p;
      bool init_ok = mk[0] && mk[c.B] && mk[2 * (int64_t)c.B] && mk[3 * (int64_t)c.B];
      if (!init_ok) { st = -1; break; }
      const uint32_t bits = c.fri_bits[(int64_t)q * c.B + p];
      for (int s = 0; s < c.S; s++) {
        if (!mk[(int64_t)(4 + s) * c.B]) { st = -2; break; }
        if (!((bits >> s) & 1u)) { st = -3; break; }
      }
      if (st != 1) break;
      if (!((bits >> 31) & 1u)) st = 0;
    }
  }
  results[p] = st;
  if (trace) {
    uint64_t* tr = trace + (int64_t)p * trace_words;
    const int r = c.r, S = c.S, Q = c.Q;
    int64_t k = 0;
    for (int64_t w = 0; w < CH_QIDX(c) + Q; w++) tr[k++] = chal(c, w, p);
    for (int i = 0; i < 4 * r; i++) tr[k++] = c.van[(int64_t)(1 + i) * c.B + p];   // C_i then quotient_i
    for (int j = 0; j < 3; j++)
      for (int q = 0; q < Q; q++) {
        const uint64_t* qv = c.qvals + (int64_t)q * 6 * c.B + p;
        tr[k++] = qv[(int64_t)(2 * j) * c.B];
        tr[k++] = qv[(int64_t)(2 * j + 1) * c.B];
      }
    tr[k++] = (uint64_t)(eqs_ok ? 1 : 0) | ((uint64_t)(pow_ok ? 1 : 0) << 1);
    for (int i = 0; i < r * c.nluts; i++) tr[k++] = c.lutre[(int64_t)i * c.B + p];
    (void)S;
  }
}

// Self-test of the device field and hash primitives the verifier kernels are built from
// (p2v_selftest): op 0 gl::mul (canonical a b mod p, Goldilocks.hs:126-133), op 3 the S-box
// multiply form (gl::mul_nc_dev_v<2>, canonicalised), op 1 the
// Poseidon permutation (permute_dev, Hash/Poseidon.hs:42-46; a = n states of 12 words),
// op 2 the 2-to-1 compression form (permute_dev(s, zh, gm = words 0..3), Hash/Merkle.hs:21-24;
// a = n states whose words 8..11 are ignored and taken as 0), op 4 one MDS layer + constants
// (the permutation's row reduction with its grouped carry fix-up).  One lane per item.
// ops 5-8: the S-box forms x -> x^7 (Hash/Poseidon.hs:92-96) with their rare -2^64 fix-ups
// (ADVICE r4): 5 sbox_n<1> (throughput permutation, partial rounds), 6 sbox_n<2> on the pair
// (a[i], b[i]) (full rounds; out[2i], out[2i+1]), 7 sbox_lat_br (row form), 8 sbox_lat (quad /
// pair forms); canonical outputs.
extern "C" __global__ void __launch_bounds__(256) k_selftest(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (op >= 5 && op <= 8) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (op == 5) { uint64_t x = a[i]; p2::dv::sbox_n<1>(&x); out[i] = gl::canon(x); }
    else if (op == 6) { uint64_t x[2] = {a[i], b[i]}; p2::dv::sbox_n<2>(x); out[2 * i] = gl::canon(x[0]); out[2 * i + 1] = gl::canon(x[1]); }
    else if (op == 7) out[i] = gl::canon(p2::sbox_lat_br(a[i]));
    else out[i] = gl::canon(p2::sbox_lat(a[i]));
#endif
  } else if (op == 0) {
    out[i] = gl::mul(a[i], b[i]);
  } else if (op == 3) {
#if defined(__HIP_DEVICE_COMPILE__)
    out[i] = gl::canon(gl::mul_nc_dev_v<2>(a[i], b[i]));
#endif
  } else if (op == 4) {
    // one MDS layer plus the next round's constants, exactly as the permutation runs it
    // (poseidon.h: 32-bit-half accumulators, the rare carry fix-up in one uniform branch per
    // group of 4 rows); b = the constants' halves kl[12], kh[12], shared by every item
#if defined(__HIP_DEVICE_COMPILE__)
    uint64_t st[12], t[12], kl[12], kh[12];
#pragma unroll
    for (int k = 0; k < 12; k++) { st[k] = a[12 * i + k]; kl[k] = b[k]; kh[k] = b[12 + k]; }
#if P2V_MDS_BRANCH == 2
    p2::dv::mds_group<0>(st, t, kl, kh);
    p2::dv::mds_group<4>(st, t, kl, kh);
    p2::dv::mds_group<8>(st, t, kl, kh);
#else
    p2::dv::mds_rows<0, 12>(st, t, kl, kh);
#endif
#pragma unroll
    for (int k = 0; k < 12; k++) out[12 * i + k] = t[k];
#endif
  } else {
    uint64_t s[12];
#pragma unroll
    for (int k = 0; k < 12; k++) s[k] = op == 2 && k >= 8 ? 0 : a[12 * i + k];
    if (op == 1) p2::permute_dev(s);
    else p2::permute_dev(s, true, 1);
#pragma unroll
    for (int k = 0; k < 12; k++) out[12 * i + k] = op == 2 && k >= 4 ? 0 : s[k];
  }
}

// The latency forms of the permutation on caller-chosen states (p2v_selftest ops 9-11; ADVICE
// r4): 9 the row form (lposeidon.h, or rposeidon.h with P2V_ROW_LAT=0; 16 lanes per state), 10 the quad form (qposeidon.h, 4 lanes),
// 11 the pair form (pposeidon.h, 2 lanes).  Every lane of a group takes part in the DPP moves, so
// lanes past n compute on a copy of state n - 1 and store nothing.  a, out: n states of 12 words.
extern "C" __global__ void __launch_bounds__(256) k_selftest_forms(int op, const uint64_t* a, uint64_t* out, int64_t n) {
  __shared__ TLdsAny T;
  if (op == 11) pp::tlds_fill(T.p, threadIdx.x, 256);
  else tlds_fill_form(T, op == 9 ? 16 : 4);
  const int lanes = op == 9 ? 16 : op == 10 ? 4 : 2;
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t item = g / lanes, src = item < n ? item : n - 1;
  const int t = (int)(g % lanes);
  const uint64_t* s = a + 12 * src;
  uint64_t* o = out + 12 * item;
  if (op == 9) {
    rp::Row R;
    rp::init(R, threadIdx.x);
    lp::Row LR;
    lp::init(LR, T.l, threadIdx.x);
    const qp::TLds& TQ = T.q;
    const lp::TLdsL& TL = T.l;
    (void)LR; (void)TQ; (void)TL;
    const uint64_t x = ROW_PERMUTE(R.L < 12 ? s[R.L] : 0);
    if (item < n && R.L < 12) o[R.L] = x;
  } else if (op == 10) {
    uint64_t x[3] = {s[3 * t], s[3 * t + 1], s[3 * t + 2]};
    qp::permute(x, t, T.q);
    if (item < n) for (int k = 0; k < 3; k++) o[3 * t + k] = x[k];
  } else {
    uint64_t x[6];
#pragma unroll
    for (int k = 0; k < 6; k++) x[k] = s[6 * t + k];
    pp::permute(x, t, T.p);
    if (item < n)
#pragma unroll
      for (int k = 0; k < 6; k++) o[6 * t + k] = x[k];
  }
}
