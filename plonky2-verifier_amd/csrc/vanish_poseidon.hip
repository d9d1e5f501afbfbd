// vanish_poseidon.hip — the PoseidonGate constraint program (Gate/Custom/Poseidon.hs:63-150,
// fast partial rounds), split into 8 independent vanishing items, and its kernels.
//
// Within a full round the state is replaced by the S-box witness wires, so the state entering
// full round r >= 2 (and the gate output) is MDS(sbox(wires of round r-1)): every full-round
// constraint block is evaluated from the wires alone and only the partial rounds form a chain.
//   part 0: swap constraints + round 1 (terms [0,17))     part 1, 2: rounds 2, 3
//   part 3: partial rounds + round 26 ([41,75))           part 4..6: rounds 27..29
//   part 7: output ([111,123))
// Term numbering is the gate's own (Acc starts at alpha^first_term of the part).
//
// Register budget: these waves run beside k_merkle (6 waves per SIMD at 80
// VGPRs), so a wave must fit the 112 VGPRs one retiring k_merkle wave leaves.  The MDS output is
// therefore never materialised: each row is reduced and pushed as a constraint term as soon as
// it is formed, from the 12 S-box outputs (48 VGPRs); and part 3's state entering the partial
// rounds, A'(M sb + rc) with the fast-partial initial matrix A' (Poseidon.hs:92-104), is one
// 12 x 12 product W sb + k (W = A'M, k = A' rc, exact mod p, host-built, DevCircuit::pos_w)
// whose S-box inputs wait in LDS instead of registers.
#include "vanish.h"

using namespace p2d;
using gl::E;

namespace {

constexpr int POS_SB1 = 29, POS_SBP = 29 + 36, POS_SBF = 29 + 36 + 22;

// The S-box outputs of a full round as two coordinate arrays (x = a + b X), 48 VGPRs.
struct SB { uint64_t a[12], b[12]; };
__device__ __forceinline__ void pin_sb(SB& x, int i) {
  asm volatile("" : "+v"(x.a[i]), "+v"(x.b[i]));
  __builtin_amdgcn_sched_barrier(0);
}

// the 12 constraints of a full round from the S-box outputs of the round before: MDS row i over
// F^2 acts on the two coordinates separately, each the hashing MDS row (p2asm::mds_row: one asm
// block of 24 v_mad_u64_u32 over the 32-bit halves and one reduction, the same element as
// p2::mds), canonicalised; round r >= 0 adds its constants (st_i = MDS(sb)_i + rc_r,i against
// wires w0..w0+11), r < 0 (the output part) compares st_i with wires w0..
template <int R>
__device__ __forceinline__ void full_rows(const Vars& V, Acc<R>& A, const SB& sb, int r, int w0) {
  sfor<0, 12>([&](auto i) {
    constexpr int I = decltype(i)::value;
#if defined(__HIP_DEVICE_COMPILE__)
    E st = E{gl::canon(p2asm::mds_row<I>(sb.a, 0, 0)), gl::canon(p2asm::mds_row<I>(sb.b, 0, 0))};
#else
    E st = gl::e0();   // (host pass of a device-only program)
#endif
    if (r >= 0) st = gl::eadd(st, lit(p2::c_round_constants[12 * r + I]));
    A.push(gl::esub(st, V.w(w0 + I)));
    sfor<0, R>([&](auto k) { pin(A.h[k]); });   // one row at a time: its accumulators are the only live extras
  });
}
// S-box outputs of the 12 wires starting at w0: the 24 words are loaded first (into the outputs'
// own registers), then the S-boxes are applied in place one at a time
__device__ __forceinline__ void sbox_in_place(SB& sb) {
  sfor<0, 12>([&](auto i) { const E y = esbox(E{sb.a[i], sb.b[i]}); sb.a[i] = y.a; sb.b[i] = y.b; pin_sb(sb, i); });
}
__device__ __forceinline__ void sbox_wires(const Vars& V, int w0, SB& sb) {
  sfor<0, 12>([&](auto i) { const E x = V.w(w0 + i); sb.a[i] = x.a; sb.b[i] = x.b; });
  sbox_in_place(sb);
}

template <int part, int R>
__device__ __forceinline__ void gate_poseidon_part(const Vars& V, Acc<R>& A) {
  SB sb;
  if constexpr (part == 0) {
    const E one = gl::eb(1);
    const E swap = V.w(24);
    A.push(gl::emul(swap, gl::esub(swap, one)));
    for (int i = 0; i < 4; i++) A.push(gl::esub(gl::emul(swap, gl::esub(V.w(i + 4), V.w(i))), V.w(25 + i)));
    sfor<0, 12>([&](auto i) {
      E s;
      if constexpr (decltype(i)::value < 4) s = gl::eadd(V.w(i), V.w(25 + i));
      else if constexpr (decltype(i)::value < 8) s = gl::esub(V.w(i), V.w(25 + i - 4));
      else s = V.w(i);
      s = gl::eadd(s, lit(p2::c_round_constants[i]));
      sb.a[i] = s.a; sb.b[i] = s.b;
    });
    sbox_in_place(sb);
    full_rows(V, A, sb, 1, POS_SB1);
  }
  else if constexpr (part <= 2) {   // rounds 2, 3
    constexpr int r = part + 1;
    sbox_wires(V, POS_SB1 + 12 * (r - 2), sb);
    full_rows(V, A, sb, r, POS_SB1 + 12 * (r - 1));
  }
  else if constexpr (part == 3) {   // partial rounds (fast form) + the round-26 constraint
    // S-box outputs of round 3's wires into LDS (one wave per work-group, lane-major)
    __shared__ uint64_t lsb[12][2][64];
    const int lane = threadIdx.x & 63;
    sbox_wires(V, POS_SB1 + 24, sb);
    sfor<0, 12>([&](auto i) { lsb[i][0][lane] = sb.a[i]; lsb[i][1][lane] = sb.b[i]; });
    // st = A'(M sb + rc_fast_first) = W sb + k  (mdsLayer, fastPartialFirstConstant, mdsInitPartial)
    const uint64_t* W = V.c->pos_w;
    E st[12];
    sfor<0, 12>([&](auto i) {
      uint64_t xa = W[144 + i], xb = 0;
#pragma unroll
      for (int j = 0; j < 12; j++) {
        const uint64_t w = W[12 * i + j];
        xa = gl::add(xa, gl::mul(w, lsb[j][0][lane]));
        xb = gl::add(xb, gl::mul(w, lsb[j][1][lane]));
      }
      st[i] = E{xa, xb};
      asm volatile("" : "+v"(st[i].a), "+v"(st[i].b) : : "memory");   // row by row: the next row's LDS reads stay below
      __builtin_amdgcn_sched_barrier(0);
    });
#pragma unroll 1
    for (int r = 0; r < 22; r++) {
      const E sbw = V.w(POS_SBP + r);
      A.push(gl::esub(st[0], sbw));
      E z = esbox(sbw);
      if (r < 21) z = gl::eadd(z, lit(p2::c_fast_rc[r]));
      // mdsFastPartial r
      E d = E{gl::mul_small(z.a, p2::mds_coeff(0, 0)), gl::mul_small(z.b, p2::mds_coeff(0, 0))};
      sfor<0, 11>([&](auto j) {
        d = gl::eadd(d, gl::escale(p2::c_fast_w_hats[11 * r + j], st[1 + j]));
        if constexpr (decltype(j)::value % 4 == 3) pin(d);   // a few products in flight, not eleven
      });
      sfor<0, 11>([&](auto j) {
        st[1 + j] = gl::eadd(st[1 + j], gl::escale(p2::c_fast_vs[11 * r + j], z));
        if constexpr (decltype(j)::value % 4 == 3) pin(st[1 + j]);
      });
      st[0] = d;
    }
    sfor<0, 12>([&](auto i) {
      A.push(gl::esub(gl::eadd(st[i], lit(p2::c_round_constants[12 * 26 + i])), V.w(POS_SBF + i)));
      sfor<0, R>([&](auto k) { pin(A.h[k]); });
    });
  }
  else if constexpr (part <= 6) {   // rounds 27..29
    constexpr int r = 26 + part - 3;
    sbox_wires(V, POS_SBF + 12 * (r - 27), sb);
    full_rows(V, A, sb, r, POS_SBF + 12 * (r - 26));
  }
  else {   // output: MDS(sbox(round 29's wires)) against wires 12..23
    sbox_wires(V, POS_SBF + 36, sb);
    full_rows(V, A, sb, -1, 12);
  }
}

// the part is a compile-time constant in each branch, so every part gets its own registers
template <int R>
__device__ __forceinline__ void gate_poseidon(const Vars& V, Acc<R>& A, int part) {
  switch (part) {
    case 0: gate_poseidon_part<0>(V, A); break;
    case 1: gate_poseidon_part<1>(V, A); break;
    case 2: gate_poseidon_part<2>(V, A); break;
    case 3: gate_poseidon_part<3>(V, A); break;
    case 4: gate_poseidon_part<4>(V, A); break;
    case 5: gate_poseidon_part<5>(V, A); break;
    case 6: gate_poseidon_part<6>(V, A); break;
    default: gate_poseidon_part<7>(V, A); break;
  }
}

}  // namespace

#ifndef P2V_NO_VANISH_KERNELS   // (register experiments include this file for its device code only)
// one-wave work-groups at <= 112 VGPRs (the space one retiring k_merkle wave leaves).  (One launch
// for all three item classes was tried: the fused program stops being inlined, 186 VGPRs and
// 1.5 KB of scratch per lane; the classes stay separate kernels.)
extern "C" __global__ void __launch_bounds__(64) k_vanish_poseidon_r2(DevCircuit c) {
  vanish_body<VK_POSEIDON, P2V_R_STD>(c);
}
extern "C" __global__ void __launch_bounds__(64) k_vanish_poseidon_rn(DevCircuit c) {
  vanish_body<VK_POSEIDON, P2V_MAX_R>(c);
}
#endif
