// valu_rates.hip — measured VALU issue costs on gfx950 for the instructions the Goldilocks /
// Poseidon code is built from, and the production permutation's cost in SIMD cycles.
//
// Part A: for each instruction, every lane runs 8 independent dependency chains of exactly that
// instruction (one inline-asm statement = one instruction), 32x unrolled; launched with w waves
// per SIMD (w = 1, 2, 4, 8) on all 256 CUs.  Output: SIMD cycles per wave64 instruction at
// saturation, i.e. (elapsed x shader clock) / (instructions issued per SIMD).  The shader clock
// is measured in the same kernel (s_memtime against s_memrealtime), not assumed.
// Part B: p2::permute_dev (the hashing permutation of k_phase1 / k_merkle, generic and
// compression forms), one permutation per lane per iteration, w = 2..8: SIMD cycles per
// permutation per wave, and permutations per second.
// Used by tools/valu_roofline.py (bench.py's `valu` block); output committed under profiles/.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../../plonky2-verifier_amd/csrc/poseidon.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int CHAINS = 8, UNROLL = 8, PER_STMT = 32;   // 8 statements x 32 instructions per iteration

// OP applied 4x to each of the 8 chains (32 instructions) in ONE asm statement: hipcc pads every inline-asm
// statement with an s_nop (it cannot see hazards inside), so one statement per instruction
// would measure the s_nop too.  Carry-outs go to a clobbered SGPR pair.
#define X8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define X32(I) X8(I) X8(I) X8(I) X8(I)
template <int OP>
__device__ __forceinline__ void step8(uint32_t* x, uint64_t* xx, uint32_t k, uint64_t kk) {
#define R32 "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])
#define R64 "+v"(xx[0]), "+v"(xx[1]), "+v"(xx[2]), "+v"(xx[3]), "+v"(xx[4]), "+v"(xx[5]), "+v"(xx[6]), "+v"(xx[7])
#define S(i) #i
  const uint32_t k2 = k ^ 5u;   // operands: %8 k (v32), %9 kk (s64), %10 kk (v64), %11 k2 (v32)
#define A(str) asm volatile(str : R32 : "v"(k), "s"(kk), "v"(kk), "v"(k2) : "s96", "s97")
#define A64(str) asm volatile(str : R64 : "v"(k), "s"(kk), "v"(kk), "v"(k2) : "s96", "s97")
#define MAD(i) "v_mad_u64_u32 %" S(i) ", s[96:97], %8, %11, %" S(i) "\n"
#define MULHI(i) "v_mul_hi_u32 %" S(i) ", %" S(i) ", %8\n"
#define MULLO(i) "v_mul_lo_u32 %" S(i) ", %" S(i) ", %8\n"
#define ADDCO(i) "v_add_co_u32_e64 %" S(i) ", s[96:97], %" S(i) ", %8\n"
#define SUBCO(i) "v_sub_co_u32_e64 %" S(i) ", s[96:97], %" S(i) ", %8\n"
#define ADDC(i) "v_addc_co_u32_e64 %" S(i) ", s[96:97], %" S(i) ", %8, %9\n"
#define CND(i) "v_cndmask_b32_e64 %" S(i) ", %" S(i) ", %8, %9\n"
#define LSHLADD(i) "v_lshl_add_u64 %" S(i) ", %" S(i) ", 0, %10\n"
#define ADD(i) "v_add_u32_e32 %" S(i) ", %" S(i) ", %8\n"
#define XOR(i) "v_xor_b32_e32 %" S(i) ", %" S(i) ", %8\n"
#define ADD3(i) "v_add3_u32 %" S(i) ", %" S(i) ", %8, %8\n"
#define MAD24(i) "v_mad_u32_u24 %" S(i) ", %" S(i) ", %8, %8\n"
#define MOV(i) "v_mov_b32_e32 %" S(i) ", %8\n"
#define LSHL64(i) "v_lshlrev_b64 %" S(i) ", 1, %" S(i) "\n"
#define CMP64(i) "v_cmp_gt_u64_e64 s[96:97], %" S(i) ", %10\n"
#define MADK(i) "v_mad_u64_u32 %" S(i) ", s[96:97], %11, 7, %" S(i) "\n"
#define NOP(i) "s_nop 0\n"
// VOP2 encodings of the carry-chain ops (carry in / out through VCC) and a VOP3 / VOP2 mix
#define ADDCO32(i) "v_add_co_u32_e32 %" S(i) ", vcc, %8, %" S(i) "\n"
#define ADDC32(i) "v_addc_co_u32_e32 %" S(i) ", vcc, %8, %" S(i) ", vcc\n"
#define SUBB32(i) "v_subb_co_u32_e32 %" S(i) ", vcc, %8, %" S(i) ", vcc\n"
#define CND32(i) "v_cndmask_b32_e32 %" S(i) ", %8, %" S(i) ", vcc\n"
#define MIX(i) ADDCO(i) ADDC32(i)
#define X16(I) X8(I) X8(I)
#define AV(str) asm volatile(str : R32 : "v"(k), "s"(kk), "v"(kk), "v"(k2) : "s96", "s97", "vcc")
  if constexpr (OP == 0) A64(X32(MAD));
  if constexpr (OP == 1) A(X32(MULHI));
  if constexpr (OP == 2) A(X32(MULLO));
  if constexpr (OP == 3) A(X32(ADDCO));
  if constexpr (OP == 4) A(X32(SUBCO));
  if constexpr (OP == 5) A(X32(ADDC));
  if constexpr (OP == 6) A(X32(CND));
  if constexpr (OP == 7) A64(X32(LSHLADD));
  if constexpr (OP == 8) A(X32(ADD));
  if constexpr (OP == 9) A(X32(XOR));
  if constexpr (OP == 10) A(X32(ADD3));
  if constexpr (OP == 11) A(X32(MAD24));
  if constexpr (OP == 12) A(X32(MOV));
  if constexpr (OP == 13) A64(X32(LSHL64));
  if constexpr (OP == 14) A64(X32(CMP64));
  if constexpr (OP == 15) A64(X32(MADK));
  if constexpr (OP == 16) A(X32(NOP));
  if constexpr (OP == 17) AV(X32(ADDCO32));
  if constexpr (OP == 18) AV(X32(ADDC32));
  if constexpr (OP == 19) AV(X32(SUBB32));
  if constexpr (OP == 20) AV(X32(CND32));
  if constexpr (OP == 21) AV(X16(MIX));
}
static const char* kOpNames[] = {
  "v_mad_u64_u32", "v_mul_hi_u32", "v_mul_lo_u32", "v_add_co_u32", "v_sub_co_u32", "v_addc_co_u32",
  "v_cndmask_b32", "v_lshl_add_u64", "v_add_u32", "v_xor_b32", "v_add3_u32", "v_mad_u32_u24", "v_mov_b32",
  "v_lshlrev_b64", "v_cmp_gt_u64", "v_mad_u64_u32 (const)", "s_nop 0",
  "v_add_co_u32_e32 (VOP2, vcc)", "v_addc_co_u32_e32 (VOP2, vcc)", "v_subb_co_u32_e32 (VOP2, vcc)", "v_cndmask_b32_e32 (VOP2, vcc)",
  "mix: v_add_co_u32_e64 + v_addc_co_u32_e32"};
constexpr int NOPS = 22;

struct Clk { unsigned long long t0, t1, r0, r1; };

template <int OP>
__global__ void __launch_bounds__(256) k_op(uint32_t* out, Clk* clk, int iters, uint32_t seed) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x[CHAINS]; uint64_t xx[CHAINS];
#pragma unroll
  for (int i = 0; i < CHAINS; i++) { x[i] = seed * (t + i) + i; xx[i] = ((uint64_t)x[i] << 32) | (x[i] ^ 0x9e37u); }
  const uint32_t k = seed | 1; const uint64_t kk = ((uint64_t)seed << 32) | 3u;
  unsigned long long t0 = 0, r0 = 0;
  if (t == 0) { t0 = clock64(); r0 = wall_clock64(); }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
      step8<OP>(x, xx, k, kk);
  }
  if (t == 0) { clk->t0 = t0; clk->r0 = r0; clk->t1 = clock64(); clk->r1 = wall_clock64(); }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < CHAINS; i++) s += x[i] + xx[i];
  out[t] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

// Part B: the production permutation, `reps` permutations per lane (state carried over)
template <int COMPRESS>
__global__ void __launch_bounds__(256) k_perm(uint64_t* out, Clk* clk, int reps, uint32_t seed) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t s[12];
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = (uint64_t)(seed + 977u * t + 131u * i) * 0x9E3779B97F4A7C15ULL % gl::P;
  unsigned long long t0 = 0, r0 = 0;
  if (t == 0) { t0 = clock64(); r0 = wall_clock64(); }
  for (int r = 0; r < reps; r++) {
    if (COMPRESS) {
#pragma unroll
      for (int i = 8; i < 12; i++) s[i] = 0;
      p2::permute_dev(s, true, 1);
    } else {
      p2::permute_dev(s, false, 7);
    }
  }
  if (t == 0) { clk->t0 = t0; clk->r0 = r0; clk->t1 = clock64(); clk->r1 = wall_clock64(); }
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) acc ^= s[i];
  out[t] = acc;
}

static int g_cus = 256;
static double g_wall_hz = 100e6;

template <class L>
static void timed(L launch, Clk* dclk, float& ms, double& f_ghz) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  launch();   // warm-up
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a)); launch(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  CK(hipEventElapsedTime(&ms, a, b));
  Clk h; CK(hipMemcpy(&h, dclk, sizeof h, hipMemcpyDeviceToHost));
  f_ghz = (double)(h.t1 - h.t0) / ((double)(h.r1 - h.r0) / g_wall_hz) / 1e9;
  CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
}

template <int OP>
static void run_op(uint32_t* d, Clk* dclk, int iters) {
  for (int w : {1, 2, 4, 8}) {
    const int blocks = g_cus * w;   // 256 threads = one wave on each of the CU's 4 SIMDs
    float ms; double f;
    timed([&] { k_op<OP><<<blocks, 256>>>(d, dclk, iters, 12345u); }, dclk, ms, f);
    const double insts_per_simd = (double)w * iters * UNROLL * PER_STMT;   // wave-instructions issued by each SIMD
    const double cyc = ms * 1e-3 * f * 1e9 / insts_per_simd;
    printf("op %-24s waves/SIMD %d  %8.3f ms  clock %.3f GHz  %6.3f SIMD-cycles/wave-instr  %8.1f G wave-instr/s\n",
           kOpNames[OP], w, ms, f, cyc, (double)g_cus * 4 * insts_per_simd / (ms * 1e-3) / 1e9);
  }
}
template <int OP> static void run_ops(uint32_t* d, Clk* c, int it) { if constexpr (OP < NOPS) { run_op<OP>(d, c, it); run_ops<OP + 1>(d, c, it); } }

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 400;
  const int reps = argc > 2 ? atoi(argv[2]) : 40;
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  g_cus = prop.multiProcessorCount;
  int wall_khz = 0; CK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
  if (wall_khz > 0) g_wall_hz = wall_khz * 1e3;
  printf("device %s  CUs %d  wall clock %.1f MHz  (clock column: s_memtime / s_memrealtime in the kernel)\n", prop.gcnArchName, g_cus, g_wall_hz / 1e6);
  uint32_t* d; CK(hipMalloc(&d, (size_t)g_cus * 8 * 256 * 4));
  uint64_t* d64; CK(hipMalloc(&d64, (size_t)g_cus * 8 * 256 * 8));
  Clk* dclk; CK(hipMalloc(&dclk, sizeof(Clk)));
  run_ops<0>(d, dclk, iters);
  for (int cmp = 0; cmp < 2; cmp++)
    for (int w : {2, 4, 6, 8}) {
      const int blocks = g_cus * w;
      float ms; double f;
      if (cmp) timed([&] { k_perm<1><<<blocks, 256>>>(d64, dclk, reps, 7u); }, dclk, ms, f);
      else timed([&] { k_perm<0><<<blocks, 256>>>(d64, dclk, reps, 7u); }, dclk, ms, f);
      const double perms = (double)blocks * 256 * reps;
      const double cyc_per_wave_perm = ms * 1e-3 * f * 1e9 / ((double)w * reps);   // SIMD cycles per wave-permutation
      printf("perm %-11s waves/SIMD %d  %8.3f ms  clock %.3f GHz  %8.0f SIMD-cycles per wave-permutation  %.3f G perm/s\n",
             cmp ? "compression" : "generic", w, ms, f, cyc_per_wave_perm, perms / (ms * 1e-3) / 1e9);
    }
  return 0;
}
