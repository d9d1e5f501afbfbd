// Microbenchmark: lane-local Poseidon-12 permutation throughput on gfx950 + KAT check.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <chrono>
#include "../../plonky2-verifier_amd/csrc/poseidon.h"
#include "../../plonky2-verifier_amd/csrc/qposeidon.h"
#include "../../plonky2-verifier_amd/csrc/rposeidon.h"
#include "../../plonky2-verifier_amd/csrc/lposeidon.h"

// ---- variant 1: lazy canonicalisation (values kept in [0, 2^64), canonical at the end)
namespace v1 {
__device__ __forceinline__ uint64_t add_nc(uint64_t a, uint64_t b) {   // a < 2^64, b < p
  uint64_t s = a + b;
  return s + ((s < a) ? gl::EPS : 0);
}
__device__ __forceinline__ uint64_t mul_nc(uint64_t a, uint64_t b) { uint64_t hi, lo; gl::mul128(a, b, hi, lo); return gl::reduce128_nc(hi, lo); }
__device__ __forceinline__ uint64_t sbox(uint64_t x) {
  uint64_t x2 = mul_nc(x, x), x3 = mul_nc(x, x2), x4 = mul_nc(x2, x2);
  return mul_nc(x3, x4);
}
__device__ __forceinline__ void mds(uint64_t s[12]) {
  uint64_t out[12];
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t al = 0, ah = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
      const uint64_t c = p2::mds_coeff(i, j);
      al += (uint64_t)(uint32_t)s[j] * c;
      ah += (s[j] >> 32) * c;
    }
    uint64_t l = al + (ah << 32);
    uint64_t h = (ah >> 32) + (l < al ? 1 : 0);
    out[i] = gl::reduce96_nc(h, l);
  }
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = out[i];
}
__device__ __forceinline__ void permute(uint64_t s[12]) {
#pragma unroll 1
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 12; i++) s[i] = sbox(add_nc(s[i], p2::c_round_constants[12 * r + i]));
    mds(s);
  }
#pragma unroll 1
  for (int r = 4; r < 26; r++) {
    s[0] = sbox(add_nc(s[0], p2::c_round_constants[12 * r]));
#pragma unroll
    for (int i = 1; i < 12; i++) s[i] = add_nc(s[i], p2::c_round_constants[12 * r + i]);
    mds(s);
  }
#pragma unroll 1
  for (int r = 26; r < 30; r++) {
#pragma unroll
    for (int i = 0; i < 12; i++) s[i] = sbox(add_nc(s[i], p2::c_round_constants[12 * r + i]));
    mds(s);
  }
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = gl::canon(s[i]);
}
}  // namespace v1


// ---- variant 2: instruction-diet mulmod / MDS reduction (see poseidon.h notes)
namespace v2 {
__device__ __forceinline__ uint64_t add_nc(uint64_t a, uint64_t b) { uint64_t s = a + b; return s + ((s < a) ? gl::EPS : 0); }
__device__ __forceinline__ uint64_t mul_nc(uint64_t a, uint64_t b) {
  const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
  const uint64_t p00 = (uint64_t)a0 * b0;
  const uint64_t p01 = (uint64_t)a0 * b1;
  const uint64_t m = (uint64_t)a1 * b0 + p01;           // may wrap: cm
  const uint64_t cm = m < p01 ? (1ULL << 32) : 0;
  const uint64_t lo = p00 + (m << 32);
  const uint64_t c1 = lo < p00 ? 1 : 0;
  const uint64_t hi = (uint64_t)a1 * b1 + (m >> 32) + (c1 | cm);
  // lo + hi_lo * (2^32 - 1) - hi_hi
  uint64_t t = (hi & 0xFFFFFFFFULL) * 0xFFFFFFFFULL + lo;
  t += t < lo ? gl::EPS : 0;
  const uint64_t hh = hi >> 32;
  uint64_t r = t - hh;
  r -= t < hh ? gl::EPS : 0;
  return r;
}
__device__ __forceinline__ uint64_t sbox(uint64_t x) {
  uint64_t x2 = mul_nc(x, x), x3 = mul_nc(x, x2), x4 = mul_nc(x2, x2);
  return mul_nc(x3, x4);
}
__device__ __forceinline__ void mds(uint64_t s[12]) {
  uint64_t out[12];
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint64_t al = 0, ah = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
      const uint64_t c = p2::mds_coeff(i, j);
      al += (uint64_t)(uint32_t)s[j] * c;
      ah += (s[j] >> 32) * c;
    }
    // value = ah*2^32 + al = ah_hi*2^64 + ah_lo*2^32 + al == ah_hi*(2^32-1) + al + ah_lo*2^32
    const uint64_t t = (ah >> 32) * 0xFFFFFFFFULL + al;   // < 2^43
    uint64_t r = t + (ah << 32);
    r += r < t ? gl::EPS : 0;
    out[i] = r;
  }
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = out[i];
}
__device__ __forceinline__ void permute(uint64_t s[12]) {
#pragma unroll 1
  for (int r = 0; r < 4; r++) {
#pragma unroll
    for (int i = 0; i < 12; i++) s[i] = sbox(add_nc(s[i], p2::c_round_constants[12 * r + i]));
    mds(s);
  }
#pragma unroll 1
  for (int r = 4; r < 26; r++) {
    s[0] = sbox(add_nc(s[0], p2::c_round_constants[12 * r]));
#pragma unroll
    for (int i = 1; i < 12; i++) s[i] = add_nc(s[i], p2::c_round_constants[12 * r + i]);
    mds(s);
  }
#pragma unroll 1
  for (int r = 26; r < 30; r++) {
#pragma unroll
    for (int i = 0; i < 12; i++) s[i] = sbox(add_nc(s[i], p2::c_round_constants[12 * r + i]));
    mds(s);
  }
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = gl::canon(s[i]);
}
}  // namespace v2

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int V>
__global__ void __launch_bounds__(256) k_perm(uint64_t* st, int iters, int n) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  uint64_t s[12];
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = st[(size_t)i * n + t];
  for (int it = 0; it < iters; it++) {
    if (V == 0) p2::permute(s);
    else if (V == 1) v1::permute(s);
    else if (V == 2) v2::permute(s);
    else {   // 2-to-1 compression form: words 8..11 zero on entry, words 0..3 out
#pragma unroll
      for (int i = 8; i < 12; i++) s[i] = 0;
#if defined(__HIP_DEVICE_COMPILE__)
      p2::permute_dev(s, true, 1);
#endif
#pragma unroll
      for (int i = 4; i < 8; i++) s[i] ^= s[i - 4];
    }
  }
#pragma unroll
  for (int i = 0; i < 12; i++) st[(size_t)i * n + t] = s[i];
}

// latency: each quad runs `iters` dependent permutations (transcript-like chain)
__global__ void __launch_bounds__(256) k_quad_chain(uint64_t* st, int iters, int nq) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  const int q = g >> 2, t = g & 3;
  __shared__ qp::TLds T;
  qp::tlds_fill(T, threadIdx.x, blockDim.x);
  if (q >= nq) return;
  uint64_t x[3];
  for (int k = 0; k < 3; k++) x[k] = st[(size_t)(3 * t + k) * nq + q];
  for (int it = 0; it < iters; it++) qp::permute(x, t, T);
  for (int k = 0; k < 3; k++) st[(size_t)(3 * t + k) * nq + q] = x[k];
}

// latency: each 16-lane row runs `iters` dependent permutations
__global__ void __launch_bounds__(256) k_row_chain(uint64_t* st, int iters, int nr) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  const int q = g >> 4, L = g & 15;
  __shared__ qp::TLds T;
  qp::tlds_fill(T, threadIdx.x, blockDim.x);
  if (q >= nr) return;   // whole rows only (nr*16 threads)
  rp::Row R;
  rp::init(R, threadIdx.x);
  uint64_t x = L < 12 ? st[(size_t)L * nr + q] : 0;
  for (int it = 0; it < iters; it++) x = rp::permute(x, R, T);
  if (L < 12) st[(size_t)L * nr + q] = x;
}

// the latency row form of lposeidon.h (round 5): same layout, LDS exchange + merged blocks
__global__ void __launch_bounds__(256) k_lrow_chain(uint64_t* st, int iters, int nr) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  const int q = g >> 4, L = g & 15;
  __shared__ lp::TLdsL T;
  lp::tlds_fill(T, threadIdx.x, blockDim.x);
  if (q >= nr) return;   // whole rows only (nr*16 threads)
  lp::Row R;
  lp::init(R, T, threadIdx.x);
  uint64_t x = L < 12 ? st[(size_t)L * nr + q] : 0;
  for (int it = 0; it < iters; it++) x = lp::permute(x, R, T);
  if (L < 12) st[(size_t)L * nr + q] = x;
}

int main(int argc, char** argv) {
  if (argc > 3 && (atoi(argv[3]) == 8 || atoi(argv[3]) == 10)) {   // row chain latency: argv[1] = rows, argv[2] = chain length (10: lposeidon.h)
    const bool lrow = atoi(argv[3]) == 10;
    int nr = atoi(argv[1]), iters = atoi(argv[2]);
    std::vector<uint64_t> h((size_t)12 * nr);
    for (size_t i = 0; i < h.size(); i++) h[i] = (i * 0x9E3779B97F4A7C15ULL) % gl::P;
    for (int i = 0; i < 12; i++) h[(size_t)i * nr] = i;
    uint64_t* d; CK(hipMalloc(&d, h.size() * 8));
    CK(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    if (lrow) k_lrow_chain<<<(16 * nr + 255) / 256, 256>>>(d, 1, nr);
    else k_row_chain<<<(16 * nr + 255) / 256, 256>>>(d, 1, nr);
    std::vector<uint64_t> o(h.size());
    CK(hipMemcpy(o.data(), d, o.size() * 8, hipMemcpyDeviceToHost));
    const uint64_t kat[12] = {0xd64e1e3efc5b8e9e, 0x53666633020aaa47, 0xd40285597c6a8825, 0x613a4f81e81231d2, 0x414754bfebd051f0, 0xcb1f8980294a023f,
                              0x6eb2a9e4d54a9d0f, 0x1902bc3af467e056, 0xf045d5eafdc6021f, 0xe4150f77caaa3be5, 0xc9bfd01d39b50cce, 0x5c0a27fcb0e1459b};
    int ok = 1; for (int i = 0; i < 12; i++) ok &= o[(size_t)i * nr] == kat[i];
    int bad = 0;
    for (int q = 1; q < nr && q < 500; q++) {
      uint64_t s[12]; for (int i = 0; i < 12; i++) s[i] = h[(size_t)i * nr + q];
      p2::permute(s);
      for (int i = 0; i < 12; i++) bad += s[i] != o[(size_t)i * nr + q];
    }
    printf("%s KAT %s, host mismatches %d\n", lrow ? "lrow" : "row", ok ? "ok" : "FAIL", bad);
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    if (lrow) k_lrow_chain<<<(16 * nr + 255) / 256, 256>>>(d, iters, nr);
    else k_row_chain<<<(16 * nr + 255) / 256, 256>>>(d, iters, nr);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    printf("%s chain: %d rows x %d perms: %.3f ms, %.2f us per dependent permutation\n", lrow ? "lrow" : "row", nr, iters, ms, ms * 1e3 / iters);
    return ok && !bad ? 0 : 1;
  }
  if (argc > 3 && atoi(argv[3]) == 9) {   // quad chain latency: argv[1] = quads, argv[2] = chain length
    int nq = atoi(argv[1]), iters = atoi(argv[2]);
    std::vector<uint64_t> h((size_t)12 * nq);
    for (size_t i = 0; i < h.size(); i++) h[i] = (i * 0x9E3779B97F4A7C15ULL) % gl::P;
    for (int i = 0; i < 12; i++) h[(size_t)i * nq] = i;
    uint64_t* d; CK(hipMalloc(&d, h.size() * 8));
    CK(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    k_quad_chain<<<(4 * nq + 255) / 256, 256>>>(d, 1, nq);
    std::vector<uint64_t> o(h.size());
    CK(hipMemcpy(o.data(), d, o.size() * 8, hipMemcpyDeviceToHost));
    const uint64_t kat0 = 0xd64e1e3efc5b8e9e, kat11 = 0x5c0a27fcb0e1459b;
    printf("quad KAT %s\n", (o[0] == kat0 && o[(size_t)11 * nq] == kat11) ? "ok" : "FAIL");
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    k_quad_chain<<<(4 * nq + 255) / 256, 256>>>(d, iters, nq);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    printf("quad chain: %d quads x %d perms: %.3f ms, %.2f us per dependent permutation\n", nq, iters, ms, ms * 1e3 / iters);
    return 0;
  }
  int n = argc > 1 ? atoi(argv[1]) : 256 * 1024;
  int iters = argc > 2 ? atoi(argv[2]) : 32;
  std::vector<uint64_t> h((size_t)12 * n);
  srand(1);
  for (auto& x : h) x = (((uint64_t)rand() << 33) ^ ((uint64_t)rand() << 11) ^ rand()) % gl::P;
  for (int i = 0; i < 12; i++) h[(size_t)i * n] = i;   // lane 0 = KAT input
  uint64_t* d; CK(hipMalloc(&d, h.size() * 8));
  CK(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  int V = argc > 3 ? atoi(argv[3]) : 0;
  auto launch = [&](int it) {
    if (V == 0) k_perm<0><<<(n + 255) / 256, 256>>>(d, it, n);
    else if (V == 1) k_perm<1><<<(n + 255) / 256, 256>>>(d, it, n);
    else if (V == 2) k_perm<2><<<(n + 255) / 256, 256>>>(d, it, n);
    else k_perm<3><<<(n + 255) / 256, 256>>>(d, it, n);
  };
  launch(1);
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> o(h.size());
  CK(hipMemcpy(o.data(), d, o.size() * 8, hipMemcpyDeviceToHost));
  const uint64_t kat[12] = {0xd64e1e3efc5b8e9e, 0x53666633020aaa47, 0xd40285597c6a8825, 0x613a4f81e81231d2, 0x414754bfebd051f0, 0xcb1f8980294a023f,
                            0x6eb2a9e4d54a9d0f, 0x1902bc3af467e056, 0xf045d5eafdc6021f, 0xe4150f77caaa3be5, 0xc9bfd01d39b50cce, 0x5c0a27fcb0e1459b};
  int ok = 1;
  if (V != 3) for (int i = 0; i < 12; i++) ok &= o[(size_t)i * n] == kat[i];
  // host cross-check on a few lanes
  int bad = 0;
  for (int t = 1; t < 2000; t++) {
    uint64_t s[12]; for (int i = 0; i < 12; i++) s[i] = h[(size_t)i * n + t];
    if (V == 3) for (int i = 8; i < 12; i++) s[i] = 0;
    p2::permute(s);
    for (int i = 0; i < (V == 3 ? 4 : 12); i++) bad += s[i] != o[(size_t)i * n + t];
  }
  printf("KAT %s, host-vs-device mismatches %d\n", ok ? "ok" : "FAIL", bad);
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  launch(iters);
  CK(hipEventRecord(a));
  launch(iters);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  double perms = (double)n * iters;
  printf("variant %d n=%d iters=%d: %.3f ms, %.3f Gperm/s\n", V, n, iters, ms, perms / ms / 1e6);
  return ok && !bad ? 0 : 1;
}
