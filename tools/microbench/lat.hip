// lat.hip — dependent-issue latency on gfx950 for the transcript's building blocks: ONE wave
// per SIMD (4 per CU) running a single dependency chain, cycles per chain link from the
// in-kernel clock (s_memtime, scaled by s_memrealtime to the shader clock).
//   chains: v_mad_u64_u32, v_add_co_u32 (carry chain), v_add_u32, DPP row_ror mov, and the
//   field multiply p2::mul_nc (x = x * x), the S-box, and 1..4 interleaved mul chains.
// The transcript (~115 dependent permutations per proof) runs at these latencies, not at the
// issue rates of valu_rates.hip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../../plonky2-verifier_amd/csrc/poseidon.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// the multiply with every carry handled on the VALU (no SALU op reads a VALU-written carry mask):
// the same value as gl::mul_nc_dev_v<1>, ~3 more VALU
__device__ __forceinline__ uint64_t mul_v3(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  using namespace gl::ax;
  const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  uint64_t cm, c1, c2, ct, c4, bw1, bw2;
  const uint64_t p00 = mad0(a0, b0);
  const uint64_t p01 = mad0(a0, b1);
  const uint64_t m = mad_co(a1, b0, p01, cm);
  const uint64_t p11 = mad0(a1, b1);
  const uint32_t lo1 = add_co((uint32_t)(p00 >> 32), (uint32_t)m, c1);
  const uint32_t h0 = addc_co((uint32_t)p11, (uint32_t)(m >> 32), c1, c2);
  const uint32_t h1 = addc0((uint32_t)(p11 >> 32), c2);
  const uint64_t lo = ((uint64_t)lo1 << 32) | (uint32_t)p00;
  const uint64_t t = madm1_co(h0, lo, ct);
  const uint32_t ul = subb_co((uint32_t)t, h1, cm, bw1);
  const uint32_t uh = subb0_co((uint32_t)(t >> 32), bw1, bw2);
  const uint64_t r1 = madm1_co(mask_1(ct), ((uint64_t)uh << 32) | ul, c4);
  return add64(r1, ((uint64_t)mask_m1(bw2) << 32) | mask_1(bw2));
#else
  return a * b;
#endif
}
__device__ __forceinline__ uint64_t mul_v1(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return gl::mul_nc_dev_v<1>(a, b);
#else
  return a * b;
#endif
}
// the multiply in plain C, no inline asm (so no s_nop padding) and no carry flags: the
// 128-bit product from four 64-bit MADs whose sums cannot overflow, then reduce128_nc
__device__ __forceinline__ uint64_t mul_c(uint64_t a, uint64_t b) {
  const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  const uint64_t p00 = (uint64_t)a0 * b0;
  const uint64_t q = (uint64_t)a0 * b1 + (p00 >> 32);
  const uint64_t r = (uint64_t)a1 * b0 + (uint32_t)q;
  const uint64_t s = (uint64_t)a1 * b1 + (q >> 32);
  const uint64_t lo = (r << 32) | (uint32_t)p00;
  const uint64_t hi = s + (r >> 32);
  return gl::reduce128_nc(hi, lo);
}
__device__ __forceinline__ uint64_t sbox_c(uint64_t x) {
  const uint64_t x2 = mul_c(x, x), x3 = mul_c(x, x2), x4 = mul_c(x2, x2);
  return mul_c(x3, x4);
}
#define X8(I) I I I I I I I I
#define X32(I) X8(I) X8(I) X8(I) X8(I)
constexpr int ITERS = 256;

template <int OP>
__global__ void __launch_bounds__(256) k_lat(uint64_t* out, uint64_t seed) {
  uint64_t x = seed + threadIdx.x, y = seed * 3 + threadIdx.x, z = seed * 5 + 1, w = seed * 7 + 2;
  uint32_t a = (uint32_t)x, k = (uint32_t)(seed | 1);
  uint64_t t0 = 0, t1 = 0, r0 = 0, r1 = 0;
  asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0));
  for (int it = 0; it < ITERS; it++) {
    if constexpr (OP == 0) asm volatile(X32("v_mad_u64_u32 %0, s[96:97], %1, %2, %0\n") : "+v"(x) : "v"(k), "v"(a) : "s96", "s97");
    if constexpr (OP == 1) asm volatile(X32("v_add_co_u32_e64 %0, s[96:97], %0, %1\n") : "+v"(a) : "v"(k) : "s96", "s97");
    if constexpr (OP == 2) asm volatile(X32("v_add_u32_e32 %0, %0, %1\n") : "+v"(a) : "v"(k));
    if constexpr (OP == 3) asm volatile(X32("v_mov_b32_dpp %0, %0 row_ror:1 row_mask:0xf bank_mask:0xf\n") : "+v"(a));
    if constexpr (OP == 4) { X8(x = p2::mul_nc(x, x);) }
    if constexpr (OP == 5) { X8(x = p2::mul_nc(x, x); y = p2::mul_nc(y, y);) }
    if constexpr (OP == 6) { X8(x = p2::mul_nc(x, x); y = p2::mul_nc(y, y); z = p2::mul_nc(z, z); w = p2::mul_nc(w, w);) }
    if constexpr (OP == 7) { X8(x = p2::sbox_lat(x);) }
    if constexpr (OP == 8) { X8(x = gl::mul(x, x);) }
    if constexpr (OP == 10) { X8(x = mul_v1(x, x);) }
    if constexpr (OP == 11) { X8(x = mul_v3(x, x);) }
    if constexpr (OP == 12) { X8(x = mul_v3(x, x); y = mul_v3(y, y);) }
    if constexpr (OP == 15) { X8(x = mul_c(x, x);) }
    if constexpr (OP == 16) { X8(x = mul_c(x, x); y = mul_c(y, y);) }
    if constexpr (OP == 17) { X8(x = sbox_c(x);) }
    if constexpr (OP == 9) asm volatile(X32("v_lshl_add_u64 %0, %0, 0, %1\n") : "+v"(x) : "v"(y));
  }
  asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1));
  if (threadIdx.x == 0 && blockIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }
  if (x == 0x1234567 && y == 3 && z == 4 && w == 5 && a == 9) out[2] = x;   // keep the chains alive
}

template <int OP>
void run(const char* name, double links_per_iter, uint64_t* d) {
  hipLaunchKernelGGL(k_lat<OP>, dim3(256), dim3(256), 0, 0, d, 12345);   // warm-up
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(k_lat<OP>, dim3(256), dim3(256), 0, 0, d, 777);
  CK(hipDeviceSynchronize());
  uint64_t h[2];
  CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
  // s_memtime counts the shader clock's ticks, s_memrealtime a 100 MHz clock
  const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
  printf("%-28s %7.2f cycles per link  (clock %.3f GHz, %.0f links)\n", name, (double)h[0] / (ITERS * links_per_iter), ghz,
         ITERS * links_per_iter);
  fflush(stdout);
}

int main() {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  uint64_t* d;
  CK(hipMalloc(&d, 64));
  run<0>("v_mad_u64_u32 chain", 32, d);
  run<1>("v_add_co_u32 chain", 32, d);
  run<2>("v_add_u32 chain", 32, d);
  run<3>("dpp row_ror mov chain", 32, d);
  run<9>("v_lshl_add_u64 chain", 32, d);
  run<4>("mul_nc chain (x*x)", 8, d);
  run<5>("2 interleaved mul chains", 8, d);
  run<6>("4 interleaved mul chains", 8, d);
  run<7>("sbox_lat chain", 8, d);
  run<8>("gl::mul chain (canonical)", 8, d);
  run<10>("mul_nc_dev (V=1) chain", 8, d);
  run<11>("mul_v3 chain (VALU carries)", 8, d);
  run<12>("2 interleaved mul_v3 chains", 8, d);
  run<15>("mul_c chain (plain C)", 8, d);
  run<16>("2 interleaved mul_c chains", 8, d);
  run<17>("sbox_c chain", 8, d);
  return 0;
}
