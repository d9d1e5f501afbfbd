// json_pack.hip — ProofWithPublicInputs JSON (Types.hs:245-279) -> packed words, on the GPU.
//
// Template-guided, like the host batch packer (circuit.cpp ProofTemplate): the proofs of one
// circuit, written by one producer, differ only in their numbers.  The host derives from one
// proof the skeleton (every byte outside the number tokens) and the packed word of each
// token; one workgroup per proof then checks the proof's own skeleton against it byte for
// byte and parses its tokens straight into the packed layout.  A proof whose bytes do not fit
// (other whitespace or key order, fractions / exponents, malformed text) is flagged and the
// host packs it with the full reader instead, so the words and error codes are always those of
// p2v_pack_proof_json.  Numbers: optional '-', decimal digits, reduced mod p
// (Goldilocks.hs:101-102: aeson integers of any size), negatives as p - (|x| mod p).
//
// Byte work, one workgroup per proof, lane per aligned 16-byte block.  Each 4 KB step:
//  1. the 256 threads read the text with coalesced 16-byte loads and classify the bytes
//     (number character or skeleton; SWAR per dword);
//  2. a workgroup prefix count (wave shuffle scan, wave totals through LDS; barrier 1) gives
//     every thread its skeleton and token offsets;
//  3. LDS staging (barrier 2): the step's slice of the template skeleton, the step's text
//     (+ 48 bytes of token tails) and its token starts in token order;
//  4. each thread compares its own skeleton bytes (16 independent LDS byte reads), then the
//     step's tokens are dealt round-robin over the threads (a run of short numbers does not
//     serialise one lane) and each is parsed from a 24-byte LDS window (7 dword reads,
//     funnel-shifted, unrolled over 21 digit positions).
// Tokens longer than 20 digits go to the host reader.
#include "devcommon.h"

namespace {
// 4-bit mask of the bytes of x that are '0'..'9' or '-' (exact for every byte value)
__device__ __forceinline__ uint32_t numc4(uint32_t x) {
  const uint32_t y = x ^ 0x30303030u;
  const uint32_t nondig = (((y | 0x80808080u) - 0x0A0A0A0Au) | y) & 0x80808080u;   // high bit: y >= 10
  const uint32_t z = x ^ 0x2D2D2D2Du;
  const uint32_t nzero = (((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;     // high bit: z != 0
  const uint32_t num = ~(nondig & nzero) & 0x80808080u;
  return ((num >> 7) * 0x01020408u) >> 24 & 15u;   // bytes 0..3 -> bits 0..3
}
__device__ __forceinline__ uint32_t word_of(const uint4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
}  // namespace

// one workgroup per proof; okf[p] = 1 when proof p was packed here, 0 when the host must
extern "C" __global__ void __launch_bounds__(256) k_json_pack(const uint8_t* __restrict__ blob, const uint64_t* __restrict__ offs, int n,
                                                              const uint8_t* __restrict__ skel, int64_t skel_len,
                                                              const int32_t* __restrict__ tok_dst, int64_t ntok,
                                                              uint64_t* __restrict__ out, int64_t W, int8_t* __restrict__ okf) {
  __shared__ uint32_t s_tot[2][4];   // per wave and step parity: skeleton bytes | tokens << 16 | bad << 31
  __shared__ int s_bad;
  __shared__ uint4 s_sk[258];        // expected skeleton bytes of the step (+ alignment slack)
  __shared__ uint4 s_tx[259];        // the step's text blocks + the 3 that follow (token tails)
  __shared__ uint16_t s_tpos[2048];  // the step's token starts (offsets in s_tx), in token order
  const int p = blockIdx.x;
  if (p >= n) return;   // uniform over the block
  const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
  const uint4* SK = (const uint4*)skel;   // 16-byte aligned, 64 bytes of slack
  const uint8_t* s = blob + offs[p];
  const int64_t len = (int64_t)(offs[p + 1] - offs[p]);
  const uint4* A = (const uint4*)((uintptr_t)s & ~(uintptr_t)15);   // the host pads the blob
  const int o = (int)((uintptr_t)s & 15);
  const int64_t nb = (o + len + 15) >> 4;
  const int64_t nsteps = (nb + 255) >> 8;
  if (t == 0) s_bad = 0;
  int64_t csk = 0, ctk = 0;   // skeleton bytes / tokens before this step
  bool bad = false;
  for (int64_t st = 0; st < nsteps; st++) {
    const int64_t j = (st << 8) + t;
    const int64_t b0 = (j << 4) - o;   // text index of the block's byte 0
    const uint4 w = j < nb ? A[j] : uint4{0, 0, 0, 0};
    const bool has_prev = b0 >= 1 && b0 <= len;
    const uint32_t wp = has_prev ? ((const uint32_t*)A)[4 * j - 1] : 0u;   // the byte before
    const int lo = (int)max((int64_t)0, min((int64_t)16, -b0)), hi = (int)max((int64_t)0, min((int64_t)16, len - b0));
    const uint32_t inr = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
    const uint32_t m = (numc4(w.x) | numc4(w.y) << 4 | numc4(w.z) << 8 | numc4(w.w) << 12) & inr;
    const uint32_t pnum = has_prev ? numc4(wp) >> 3 : 0u;
    const uint32_t starts = m & ~((m << 1) | pnum);
    const uint32_t skm = inr & ~m;
    // workgroup prefix count of (skeleton bytes | tokens << 16)
    const uint32_t cnt = (uint32_t)__popc(skm) | ((uint32_t)__popc(starts) << 16);
    uint32_t inc = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d);
      inc += lane >= d ? y : 0u;
    }
    const bool wbad = __ballot(bad) != 0;
    if (lane == 63) s_tot[st & 1][wv] = inc | ((uint32_t)wbad << 31);
    __syncthreads();
    uint32_t before = 0, all = 0, any_bad = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t x = s_tot[st & 1][u];
      before += u < wv ? (x & 0x7FFFFFFFu) : 0u;
      all += x & 0x7FFFFFFFu;
      any_bad |= x >> 31;
    }
    if (any_bad) break;   // uniform: every thread read the same four words
    const uint32_t ex = before + inc - cnt;
    const int64_t sk = csk + (ex & 0xFFFF);
    const int64_t tk0 = ctk;
    const uint32_t step_tk = all >> 16;
    // stage in LDS: the step's slice of the template skeleton, skel[csk, csk + <= 4096); the
    // step's text (+ 48 bytes of token tails); and the step's token starts in token order
    {
      const int64_t sb = csk >> 4;
      for (int i = t; i < 258; i += 256) s_sk[i] = ((sb + i) << 4) < skel_len ? SK[sb + i] : uint4{0, 0, 0, 0};
      s_tx[t] = w;
      if (t < 3) s_tx[256 + t] = j + 256 < nb ? A[j + 256] : uint4{0, 0, 0, 0};
      uint32_t rem = starts, q = ex >> 16;
      while (rem) {
        s_tpos[q++] = (uint16_t)(16 * t + __builtin_ctz(rem));
        rem &= rem - 1;
      }
    }
    __syncthreads();
    const uint8_t* E = (const uint8_t*)s_sk + (csk & 15) + (sk - csk);
    csk += all & 0xFFFF; ctk += step_tk;
    if (sk + __popc(skm) > skel_len) bad = true;
    else {
      uint32_t mis = 0, r = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) {   // branch-free: 16 independent LDS byte reads
        const uint32_t bit = (skm >> k) & 1;
        const uint32_t e = E[r];
        mis |= bit ? (e ^ ((word_of(w, k >> 2) >> (8 * (k & 3))) & 255)) : 0u;
        r += bit;
      }
      bad = bad || mis != 0;
    }
    // the step's tokens, dealt round-robin over the threads (about 190 per 4 KB step)
    for (uint32_t q = t; q < step_tk && !bad; q += 256) {
      const int64_t tk = tk0 + q;
      if (tk >= ntok) { bad = true; break; }
      const int ls = s_tpos[q];
      const bool neg = ((const uint8_t*)s_tx)[ls] == '-';
      const int lp = ls + (neg ? 1 : 0);   // first digit, in the staged text
      const uint32_t* D = (const uint32_t*)s_tx + (lp >> 2);
      const uint32_t sh = (uint32_t)(lp & 3) * 8;
      uint32_t rw[7], e[6];
#pragma unroll
      for (int i = 0; i < 7; i++) rw[i] = D[i];
#pragma unroll
      for (int i = 0; i < 6; i++) e[i] = (uint32_t)((((uint64_t)rw[i + 1] << 32) | rw[i]) >> sh);
      uint64_t acc = 0;
      bool live = true;
      int nd = 0;
      uint32_t term = 0;
#pragma unroll
      for (int i = 0; i < 21; i++) {
        const uint32_t c = (e[i >> 2] >> (8 * (i & 3))) & 255;
        const uint32_t dg = c - '0';
        const bool isd = dg < 10u;
        if (live && !isd) term = c;
        live = live && isd;
        if (i < 19) acc = live ? acc * 10 + dg : acc;
        else if (i == 19) { if (live) acc = gl::add(gl::mul(acc, 10), dg); }   // 10^19 <= acc*10+d < 2^67
        nd += live;
      }
      if (live || nd == 0 || term == '-') { bad = true; break; }   // > 20 digits, "-" alone, "1-2"
      const uint64_t v = neg ? (acc ? gl::P - acc : 0) : acc;
      const int32_t wo = tok_dst[tk];
      if (wo >= 0) out[(int64_t)p * W + wo] = v;
    }
  }
  if (bad || csk != skel_len || ctk != ntok) s_bad = 1;   // benign race: every writer stores 1
  __syncthreads();
  if (t == 0) okf[p] = s_bad ? 0 : 1;
}

// ------------------------------------------------------------------ plonky2 binary proofs
// plonky2's byte serialization (circuit.cpp pack_proof_bytes) has a fixed layout for a given
// circuit: runs of little-endian u64 words at fixed byte offsets, u8 sibling counts at fixed
// offsets, then the public inputs (raw, or after a u64 count).  The host turns it into a map
// (circuit.cpp bytes_map: runs of (source byte, packed word, count), count bytes and their values);
// one workgroup per proof checks the length, the count bytes and the PI form, then copies every
// run into the packed row with coalesced loads and stores, reducing mod p.  A proof that fails
// any check is flagged and packed by the host reader (the exact error code).  Words after a count
// byte sit at odd byte offsets: each is assembled from three aligned dwords with v_alignbyte
// (the blob has 64 bytes of slack past its end).
__device__ __forceinline__ uint64_t ld_u64_any(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t w0 = q[0], w1 = q[1], w2 = q[2];
  const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh), hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t modp(uint64_t x) { return x >= gl::P ? x - gl::P : x; }

extern "C" __global__ void __launch_bounds__(256) k_bytes_pack(const uint8_t* __restrict__ blob, const uint64_t* __restrict__ offs, int n,
                                                               const int64_t* __restrict__ rsrc, const int64_t* __restrict__ rdst,
                                                               const int64_t* __restrict__ rlen, int nruns,
                                                               const int64_t* __restrict__ coff, const uint8_t* __restrict__ cval, int nchk,
                                                               int64_t fixed, int64_t npis, int64_t pis_dst,
                                                               uint64_t* __restrict__ dst, int64_t W, int8_t* __restrict__ ok) {
  const int i = blockIdx.x;
  if (i >= n) return;
  const uint8_t* s = blob + offs[i];
  const int64_t L = (int64_t)(offs[i + 1] - offs[i]);
  int64_t pis_src = -1;
  if (L == fixed + 8 * npis) pis_src = fixed;
  else if (L == fixed + 8 + 8 * npis && ld_u64_any(s + fixed) == (uint64_t)npis) pis_src = fixed + 8;
  int good = pis_src >= 0;
  if (good)
    for (int k = threadIdx.x; k < nchk; k += blockDim.x) good &= s[coff[k]] == cval[k];
  good = __syncthreads_and(good);
  if (!good) {
    if (threadIdx.x == 0) ok[i] = 0;
    return;
  }
  uint64_t* d = dst + (int64_t)i * W;
  for (int r = 0; r < nruns; r++) {
    const uint8_t* src = s + rsrc[r];
    uint64_t* out = d + rdst[r];
    const int64_t len = rlen[r];
    for (int64_t k = threadIdx.x; k < len; k += blockDim.x) out[k] = modp(ld_u64_any(src + 8 * k));
  }
  for (int64_t k = threadIdx.x; k < npis; k += blockDim.x) d[pis_dst + k] = modp(ld_u64_any(s + pis_src + 8 * k));
  if (threadIdx.x == 0) ok[i] = 1;
}
