// lposeidon.h — Poseidon-12 over a 16-lane row for the LATENCY paths (device only): the
// transcript of small batches (~115 strictly dependent permutations per proof,
// Challenge/Pure.hs:50-69) and the small-batch Merkle paths (Hash/Merkle.hs:27-42).
//
// Same layout and interface as rposeidon.h (lane L < 12 of the row holds state word L), built
// for a lone wave: on a dependent chain a wave issues about one instruction per 4-cycle slot
// whatever their independence, so its time is its instruction count, s_nop padding included
// (DESIGN.md §5.2).  Round 5 cut that count:
//   * no DPP rotations: after its S-box each lane writes its word to LDS and reads the row's 12
//     words back (a wave's LDS operations are processed in order), so every lane holds the
//     whole state and computes its own MDS row from 12 terms (24 MADs) instead of 16 rotations
//     x 2 halves (30 DPP moves + 32 MADs);
//   * the 22 partial rounds as the merged blocks of poseidon.h (PBlock, D = 4,4,4,4,4,2): with
//     the whole state in every lane, each lane runs the block's S-box chain itself (y_1..y_D
//     through the chain rows) and then its own output row: one exchange per block instead of D;
//     round 6 (pblock_par) moves the chain rows' dot products onto the idle lanes 12-14, off the
//     serial path: 8.2-8.5 -> 6.6-6.8 us per dependent permutation (profiles/r06p_row_par.txt),
//     and splits their S-boxes' x^3 / x^4 over lane pairs (sbox_u): 6.2-6.4 us (r06u_row_sbox2.txt);
//   * the S-box multiply and the row reductions as single inline-asm statements (the compiler
//     pads an s_nop after every inline-asm statement with an SGPR output, an issue slot of the
//     lone wave each time); the MADs are plain C with coefficients in registers (no asm, no
//     padding, no strength reduction of constant coefficients).
// Same function as Hash/Poseidon.hs:42-101 (the block algebra: poseidon.h PBlock); held to the
// KAT and the oracle by test_gpu_permutation_forms_first_round_wrap (p2v_selftest op 9) and by
// every transcript trace of the small-batch tests.
#pragma once
#include "gl.h"
#include "poseidon.h"

namespace lp {

constexpr int kXbStride = 17;   // u64 per row's exchange slots: 136 B apart, so the four rows of
                                // a wave read distinct LDS banks in the same broadcast read

// The permutation's tables and the rows' exchange slots in LDS, filled once per workgroup.
struct TLdsL {
  p2::RcSplit rc;                // round constants as 32-bit halves, rows 0..30 (30 = 0)
  uint64_t rc0[12];              // round 0's constants (added before the first S-box)
  uint32_t m[12][16];            // the MDS matrix M[i][j] (Hash/Constants.hs:19-25), rows padded
  p2::PBlock pm[p2::PM_NB];      // the merged partial-round blocks (poseidon.h make_pm)
  uint64_t xb[16 * kXbStride];   // per 16-lane row of a 256-thread workgroup: the state words
};

// cooperative fill by the n threads of the workgroup; ends with a barrier
__device__ __forceinline__ void tlds_fill(TLdsL& T, int tid, int n) {
  const uint64_t* rs = (const uint64_t*)&p2::c_rc_split;
  uint64_t* rd = (uint64_t*)&T.rc;
  for (int i = tid; i < (int)(sizeof(p2::RcSplit) / 8); i += n) rd[i] = rs[i];
  if (tid < 12) T.rc0[tid] = p2::c_round_constants[tid];
  for (int i = tid; i < 192; i += n) T.m[i / 16][i % 16] = (i % 16) < 12 ? p2::mds_coeff(i / 16, i % 16) : 0u;
  const uint32_t* qs = (const uint32_t*)&p2::c_pm;
  uint32_t* qd = (uint32_t*)T.pm;
  for (int i = tid; i < (int)(sizeof(p2::PMTab) / 4); i += n) qd[i] = qs[i];
  __syncthreads();
}

// A lane's row context: its word index (idle lanes 12..15 compute on word 11's coefficients and
// are never read) and its exchange slots.
struct Row {
  int L, Lc;
  uint64_t* xb;
};
__device__ __forceinline__ void init(Row& R, TLdsL& T, int tid) {
  R.L = tid & 15;
  R.Lc = R.L < 12 ? R.L : 11;
  R.xb = T.xb + (tid >> 4) * kXbStride;
}

#if defined(__HIP_DEVICE_COMPILE__)
// a b mod p (a, b < 2^64; result in [0, 2^64)) as one asm statement: 14 VALU + 2 SALU, the
// branch-free net-wrap fix-up of gl::mul_nc_dev_v<1>.  Scratch: v[4:9], s[88:95].
//   P = a0 b0;  X = a0 b1 + hi(P);  Y = a1 b0 + X (carry cm, weight 2^96);  H = a1 b1 + hi(Y)
//   lo = lo(P) + lo(Y) 2^32;  T = lo + h0 (2^32 - 1) (carry ct);  U = T - h1 - cm (borrow bw)
//   r = U + (ct & ~bw) (2^32 - 1) + (bw & ~ct) p   (2^64 == 2^32 - 1, 2^96 == -1 mod p)
__device__ __forceinline__ uint64_t mul_lat(uint64_t a, uint64_t b) {
  uint64_t r;
  asm("v_mad_u64_u32 v[4:5], s[94:95], %[a0], %[b0], 0\n\t"
      "v_lshrrev_b64 v[6:7], 32, v[4:5]\n\t"
      "v_mad_u64_u32 v[6:7], s[94:95], %[a0], %[b1], v[6:7]\n\t"
      "v_mad_u64_u32 v[6:7], s[92:93], %[a1], %[b0], v[6:7]\n\t"
      "v_lshrrev_b64 v[8:9], 32, v[6:7]\n\t"
      "v_mad_u64_u32 v[8:9], s[94:95], %[a1], %[b1], v[8:9]\n\t"
      "v_mov_b32_e32 v5, v6\n\t"
      "v_mad_u64_u32 v[4:5], s[90:91], v8, -1, v[4:5]\n\t"
      "v_subb_co_u32_e64 v4, s[88:89], v4, v9, s[92:93]\n\t"
      "v_subb_co_u32_e64 v5, s[88:89], v5, 0, s[88:89]\n\t"
      "s_andn2_b64 s[92:93], s[90:91], s[88:89]\n\t"
      "s_andn2_b64 s[94:95], s[88:89], s[90:91]\n\t"
      "v_cndmask_b32_e64 v6, 0, 1, s[94:95]\n\t"
      "v_cndmask_b32_e64 v6, v6, -1, s[92:93]\n\t"
      "v_cndmask_b32_e64 v7, 0, -1, s[94:95]\n\t"
      "v_lshl_add_u64 %[r], v[4:5], 0, v[6:7]"
      : [r] "=&v"(r)
      : [a0] "v"((uint32_t)a), [a1] "v"((uint32_t)(a >> 32)), [b0] "v"((uint32_t)b), [b1] "v"((uint32_t)(b >> 32))
      : "v4", "v5", "v6", "v7", "v8", "v9", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95", "scc");
  return r;
}
__device__ __forceinline__ uint64_t sbox(uint64_t x) {   // x^7 (Hash/Poseidon.hs:92-96)
  const uint64_t x2 = mul_lat(x, x), x3 = mul_lat(x, x2), x4 = mul_lat(x2, x2);
  return mul_lat(x3, x4);
}

// al + 2^32 ah -> [0, 2^64), congruent mod p, for al < 2^63 and ah < 2^62 (every MDS and
// chain row, and the output rows of blocks with D <= 3: row sums < 2^24): t = al + ah_hi
// (2^32 - 1) cannot carry; ah_lo joins t's high word (carry c, weight 2^64 == 2^32 - 1), and
// the wrapped sum is small enough that adding c (2^32 - 1) cannot carry again.  4 VALU.
__device__ __forceinline__ uint64_t red_small(uint64_t al, uint64_t ah) {
  uint64_t r;
  asm("v_mad_u64_u32 v[4:5], s[94:95], %[ahh], -1, %[al]\n\t"
      "v_add_co_u32_e64 v5, s[92:93], v5, %[ahl]\n\t"
      "v_cndmask_b32_e64 v6, 0, 1, s[92:93]\n\t"
      "v_mad_u64_u32 %[r], s[94:95], v6, -1, v[4:5]"
      : [r] "=&v"(r)
      : [al] "v"(al), [ahh] "v"((uint32_t)(ah >> 32)), [ahl] "v"((uint32_t)ah)
      : "v4", "v5", "v6", "s92", "s93", "s94", "s95");
  return r;
}
// the same for al, ah < 2^64 with ah < 2^63.8 (the output rows of D = 4 blocks: poseidon.h
// reduce_w): lo = al + ah_lo 2^32 (carry c0), hi = ah_hi + c0 < 2^32, lo + hi (2^32 - 1) with one
// wrap fix-up (the wrapped sum is < hi 2^32: no second wrap).  6 VALU.
__device__ __forceinline__ uint64_t red_wide(uint64_t al, uint64_t ah) {
  uint64_t r;
  asm("v_mov_b32_e32 v4, %[all]\n\t"
      "v_add_co_u32_e64 v5, s[92:93], %[alh], %[ahl]\n\t"
      "v_addc_co_u32_e64 v6, s[94:95], %[ahh], 0, s[92:93]\n\t"
      "v_mad_u64_u32 v[4:5], s[92:93], v6, -1, v[4:5]\n\t"
      "v_cndmask_b32_e64 v6, 0, 1, s[92:93]\n\t"
      "v_mad_u64_u32 %[r], s[94:95], v6, -1, v[4:5]"
      : [r] "=&v"(r)
      : [all] "v"((uint32_t)al), [alh] "v"((uint32_t)(al >> 32)), [ahh] "v"((uint32_t)(ah >> 32)), [ahl] "v"((uint32_t)ah)
      : "v4", "v5", "v6", "s92", "s93", "s94", "s95");
  return r;
}

// acc + a c with a register coefficient: one v_mad_u64_u32, no asm
__device__ __forceinline__ uint64_t madr(uint32_t a, uint32_t c, uint64_t acc) { return (uint64_t)a * c + acc; }

// (al, ah) += sum_j c[j] s[j] over the 32-bit halves (c: 12 coefficients, 16-B aligned in LDS)
__device__ __forceinline__ void dot12(const uint32_t* c, const uint64_t* s, uint64_t& al, uint64_t& ah) {
  const uint4* c4 = (const uint4*)c;
#pragma unroll
  for (int q = 0; q < 3; q++) {
    const uint4 k = c4[q];
    al = madr((uint32_t)s[4 * q], k.x, al);         ah = madr((uint32_t)(s[4 * q] >> 32), k.x, ah);
    al = madr((uint32_t)s[4 * q + 1], k.y, al);     ah = madr((uint32_t)(s[4 * q + 1] >> 32), k.y, ah);
    al = madr((uint32_t)s[4 * q + 2], k.z, al);     ah = madr((uint32_t)(s[4 * q + 2] >> 32), k.z, ah);
    al = madr((uint32_t)s[4 * q + 3], k.w, al);     ah = madr((uint32_t)(s[4 * q + 3] >> 32), k.w, ah);
  }
}

// the row's state into every lane: lane L writes its word, then reads all 12 (a wave's LDS
// operations are processed in order, so the reads see the writes of the row's other lanes; the
// compiler fences stop it from moving the reads above the write)
__device__ __forceinline__ void exchange(uint64_t x, uint64_t* xb, int L, uint64_t s[12]) {
  xb[L] = x;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int j = 0; j < 12; j++) s[j] = xb[j];
}

// full round r: S-box, exchange, MDS row Lc + the constants of round r + 1
__device__ __forceinline__ uint64_t full_round(uint64_t x, int r, const Row& R, const TLdsL& T) {
  uint64_t s[12];
  exchange(sbox(x), R.xb, R.L, s);
  uint64_t al = T.rc.lo[12 * (r + 1) + R.Lc], ah = T.rc.hi[12 * (r + 1) + R.Lc];
  dot12(T.m[R.Lc], s, al, ah);
  return red_small(al, ah);
}

// D merged partial rounds (poseidon.h PBlock / dv::pblock): x = this lane's word of the state
// entering the block (its constants included) -> its word of the state after the block
template <int D>
__device__ __forceinline__ uint64_t pblock(uint64_t x, const p2::PBlock& B, const Row& R, const TLdsL& T) {
  uint64_t s[12], y[D + 1];
  exchange(x, R.xb, R.L, s);
  s[0] = sbox(s[0]);   // y_1, word 0 of s'
  const uint32_t m00 = T.m[0][0];
  {   // chain row 1: row 0 of M s' + d_1
    uint64_t al = B.dlo[0], ah = B.dhi[0];
    dot12(T.m[0], s, al, ah);
    y[2] = sbox(red_small(al, ah));
  }
  if constexpr (D >= 3) {   // chain row 2: G_2 row 0 . s' + M00 y_2 + d_2
    uint64_t al = madr((uint32_t)y[2], m00, B.dlo[1]), ah = madr((uint32_t)(y[2] >> 32), m00, B.dhi[1]);
    dot12(B.cf[0], s, al, ah);
    y[3] = sbox(red_small(al, ah));
  }
  if constexpr (D >= 4) {   // chain row 3: G_3 row 0 . s' + H_3[0][2] y_2 + M00 y_3 + d_3
    uint64_t al = madr((uint32_t)y[3], m00, B.dlo[2]), ah = madr((uint32_t)(y[3] >> 32), m00, B.dhi[2]);
    dot12(B.cf[1], s, al, ah);
    al = madr((uint32_t)y[2], B.cf[1][12], al);
    ah = madr((uint32_t)(y[2] >> 32), B.cf[1][12], ah);
    y[4] = sbox(red_small(al, ah));
  }
  // this lane's output row: G_D row Lc . s' + sum_m H_D[Lc][m] y_m + M[Lc][0] y_D + d_D
  const uint32_t* cf = B.cf[2 + R.Lc];
  const uint32_t c0 = T.m[R.Lc][0];
  uint64_t al = madr((uint32_t)y[D], c0, B.dlo[4 + R.Lc]), ah = madr((uint32_t)(y[D] >> 32), c0, B.dhi[4 + R.Lc]);
  dot12(cf, s, al, ah);
#pragma unroll
  for (int m = 2; m < D; m++) {
    al = madr((uint32_t)y[m], cf[12 + m - 2], al);
    ah = madr((uint32_t)(y[m] >> 32), cf[12 + m - 2], ah);
  }
  return D == 4 ? red_wide(al, ah) : red_small(al, ah);
}

// Round 6: the same block with its chain rows on the row's idle lanes.  pblock above evaluates
// chain row k (a 12-term dot product over s') between S-box k and S-box k + 1, so three dot
// products sit on the lone wave's serial path per block.  None of them depends on the chain
// except through its y terms.  Here every lane of the row evaluates one row's s'-part in the same
// dot product: lanes 0..11 their output rows, lanes 12, 13, 14 chain rows 1, 2, 3.  Then the
// chain is, per S-box, one reduction in every lane, a broadcast of the chain lane's value to its
// row (DPP row_newbcast) and the S-box.  Each lane adds y_m times its own row's coefficient:
//   output row L: H_D[L][m] (cf[12 + m - 2]) for m < D, M[L][0] for m = D;
//   chain row 2 (lane 13): M[0][0] for y_2;  chain row 3 (lane 14): H_3[0][2] (cf[12]) for y_2,
//   M[0][0] for y_3.
// A lane's sum is read only at the step where it is complete (lane 12 at S-box 2, 13 at 3, 14 at
// 4, the output rows after the block).  That sum has the same non-negative terms as pblock's, so
// the same reduction bounds hold.  The other lanes' reductions of partial sums are never read.
// Lane 15 repeats lane 13's row and is never read.
#ifndef P2V_ROW_PAR
#define P2V_ROW_PAR 1   // 0: pblock (round 5), the chain rows between the S-boxes
#endif
// lane S of each 16-lane row, to the whole row (DPP row_newbcast: a VALU move, no LDS round trip)
template <int S>
__device__ __forceinline__ uint64_t row_bcast(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x150 + S, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x150 + S, 0xf, 0xf, false);
  return (uint64_t)hi << 32 | lo;
}
// x^7 of a value every lane of the row holds (the partial rounds' S-box inputs): x^3 and x^4 are
// independent, so even lanes form x^3 = x x^2 and odd lanes x^4 = x^2 x^2 in one multiply, swap
// them with their neighbour (DPP quad_perm [1,0,3,2]) and multiply: three multiplies on the
// serial path instead of four.  Bit-identical to sbox(): mul_lat's result is a function of the
// 128-bit product alone (the cross terms a0 b1 + a1 b0 enter as one sum), so x^3 x^4 and x^4 x^3
// agree.
#ifndef P2V_ROW_SBOX2
#define P2V_ROW_SBOX2 1   // 0: sbox() for the uniform S-box inputs too
#endif
__device__ __forceinline__ uint64_t sbox_u(uint64_t x, int L) {
#if P2V_ROW_SBOX2
  const uint64_t x2 = mul_lat(x, x);
  const uint64_t h = mul_lat((L & 1) ? x2 : x, x2);
  constexpr int kSwap = 1 | (0 << 2) | (3 << 4) | (2 << 6);
  const uint32_t olo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)h, kSwap, 0xf, 0xf, false);
  const uint32_t ohi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(h >> 32), kSwap, 0xf, 0xf, false);
  return mul_lat(h, (uint64_t)ohi << 32 | olo);
#else
  (void)L;
  return sbox(x);
#endif
}
template <int D>
__device__ __forceinline__ uint64_t pblock_par(uint64_t x, const p2::PBlock& B, const Row& R, const TLdsL& T, uint32_t c0) {
  uint64_t s[12];
  exchange(x, R.xb, R.L, s);
  const int L = R.L;
  const uint32_t* cf = L < 12 ? B.cf[2 + L] : (L == 12 ? T.m[0] : B.cf[L == 14 ? 1 : 0]);
  const int di = L < 12 ? 4 + L : (L == 15 ? 1 : L - 12);
  uint64_t al = B.dlo[di], ah = B.dhi[di];
  const uint4 hk = *(const uint4*)(cf + 12);   // H coefficients (zero where the row has none)
  const uint32_t m00 = T.m[0][0];
  s[0] = sbox_u(s[0], L);   // y_1, word 0 of s'
  dot12(cf, s, al, ah);
  uint64_t y = sbox_u(row_bcast<12>(red_small(al, ah)), L);   // y_2
  {
    const uint32_t k = D == 2 ? c0 : (L == 13 ? m00 : hk.x);
    al = madr((uint32_t)y, k, al); ah = madr((uint32_t)(y >> 32), k, ah);
  }
  if constexpr (D >= 3) {
    y = sbox_u(row_bcast<13>(red_small(al, ah)), L);   // y_3
    const uint32_t k = D == 3 ? c0 : (L == 14 ? m00 : hk.y);
    al = madr((uint32_t)y, k, al); ah = madr((uint32_t)(y >> 32), k, ah);
  }
  if constexpr (D >= 4) {
    y = sbox_u(row_bcast<14>(red_small(al, ah)), L);   // y_4
    al = madr((uint32_t)y, c0, al); ah = madr((uint32_t)(y >> 32), c0, ah);
  }
  return D == 4 ? red_wide(al, ah) : red_small(al, ah);
}

// the row's permutation; x = this lane's word (inputs < 2^64, outputs canonical)
__device__ __forceinline__ uint64_t permute(uint64_t x, const Row& R, const TLdsL& T) {
  x = p2::add_nc(x, T.rc0[R.Lc]);
#pragma unroll 1
  for (int r = 0; r < 4; r++) x = full_round(x, r, R, T);
#if P2V_PMERGE == 4 && P2V_ROW_PAR
  const uint32_t c0 = T.m[R.Lc][0];   // M[L][0]: the output row's y_D coefficient
#pragma unroll 1
  for (int b = 0; b < 5; b++) x = pblock_par<4>(x, T.pm[b], R, T, c0);
  x = pblock_par<2>(x, T.pm[5], R, T, c0);
#elif P2V_PMERGE == 4
#pragma unroll 1
  for (int b = 0; b < 5; b++) x = pblock<4>(x, T.pm[b], R, T);
  x = pblock<2>(x, T.pm[5], R, T);
#else
#error "lposeidon.h follows the D = 4,4,4,4,4,2 merge schedule (P2V_PMERGE 4)"
#endif
#pragma unroll 1
  for (int r = 26; r < 30; r++) x = full_round(x, r, R, T);
  return gl::canon(x);
}
#elif defined(__HIPCC__)
__device__ uint64_t permute(uint64_t x, const Row& R, const TLdsL& T);   // device-only
#endif

}  // namespace lp
