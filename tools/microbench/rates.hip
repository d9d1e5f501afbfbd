// Microbenchmark: integer VALU throughput on gfx950 for the ops a Goldilocks / Poseidon
// implementation can be built from.  8 independent chains per lane, full chip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ void __launch_bounds__(256) k_rate(unsigned* out, int iters, unsigned seed) {
  unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned a[8]; unsigned long long acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) { a[i] = seed * (t + i) + i; acc[i] = a[i] ^ 0x12345; }
  const unsigned b = seed | 1;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if (OP == 0) acc[i] = (unsigned long long)(a[i] ^ (unsigned)acc[i]) * b + acc[i];      // v_mad_u64_u32 (+ xor)
        if (OP == 1) acc[i] = (unsigned)acc[i] + __umul24(a[i] ^ (unsigned)acc[i], b);           // v_mad_u32_u24 (+xor)
        if (OP == 2) acc[i] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a[i] ^ (unsigned)acc[i]), __builtin_bit_cast(u16x2, b), (unsigned)acc[i], false);
        if (OP == 3) acc[i] = (unsigned)acc[i] + (a[i] ^ (unsigned)acc[i]);                      // v_add (+xor)
        if (OP == 4) acc[i] = (unsigned)acc[i] * (a[i] ^ (unsigned)acc[i]);                      // v_mul_lo_u32 (+xor)
        if (OP == 5) acc[i] = __umulhi(a[i] ^ (unsigned)acc[i], b) + (unsigned)acc[i];           // v_mul_hi_u32 + add
        if (OP == 6) acc[i] = acc[i] + ((unsigned long long)(a[i] ^ (unsigned)acc[i]) << 7);     // v_lshl_add_u64 (+xor)
      }
    }
  }
  unsigned long long s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += acc[i];
  out[t] = (unsigned)s ^ (unsigned)(s >> 32);
}

int main(int argc, char** argv) {
  int blocks = argc > 1 ? atoi(argv[1]) : 256 * 8;
  int iters = argc > 2 ? atoi(argv[2]) : 200;
  unsigned* d; CK(hipMalloc(&d, (size_t)blocks * 256 * 4));
  const char* names[] = {"mad_u64_u32+xor", "mad_u32_u24+xor", "dot2_u32_u16+xor", "add+xor", "mul_lo_u32+xor", "mul_hi_u32+add+xor", "lshl_add_u64+xor"};
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int op = 0; op < 7; op++) {
    for (int rep = 0; rep < 2; rep++) {
      CK(hipEventRecord(a));
      switch (op) {
        case 0: k_rate<0><<<blocks, 256>>>(d, iters, 3); break;
        case 1: k_rate<1><<<blocks, 256>>>(d, iters, 3); break;
        case 2: k_rate<2><<<blocks, 256>>>(d, iters, 3); break;
        case 3: k_rate<3><<<blocks, 256>>>(d, iters, 3); break;
        case 4: k_rate<4><<<blocks, 256>>>(d, iters, 3); break;
        case 5: k_rate<5><<<blocks, 256>>>(d, iters, 3); break;
        case 6: k_rate<6><<<blocks, 256>>>(d, iters, 3); break;
      }
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      double ops = (double)blocks * 256 * iters * 16 * 8;   // "op pairs" per lane
      if (rep) printf("%-22s %8.3f ms  %7.2f T op-pairs/s  (per CU per cycle @2.4GHz: %.1f lane-op-pairs)\n", names[op], ms, ops / ms / 1e9, ops / (ms * 1e-3) / 256 / 2.4e9);
    }
  }
  return 0;
}
