// stream_pm.hip — calibrates what rocprofv3's FETCH_SIZE reports for the verifier's read
// pattern: one lane per proof streaming its own proof's contiguous words ("proof-major", the
// in-place batch read of devcommon.h ld()), 8 words per sponge block with VALU work between
// blocks, against the coalesced [word][proof] read the transposed layout used.
//
//   ./stream_pm <mode> <spin> [n] [words] [R]
//   mode 0: proof-major, 8-B loads (as ld()) ; 1: proof-major, 16-B loads ;
//   mode 2: transposed [word][n] rows, 8-B loads (coalesced 512-B rows per wave)
//   spin  : dependent 64-bit multiply-adds per lane between 8-word blocks (the permutation's
//           place; ~0 = pure streaming)
// Prints the kernel time and the algorithmic bytes read (n * words * 8); run it under
// `rocprofv3 --pmc FETCH_SIZE` to compare the counter with those bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

typedef uint64_t u64x2 __attribute__((ext_vector_type(2), aligned(8)));

// grid: (n/64 proof blocks) x R segments, one wave per (proof block, segment), proof block
// fastest (the leaf-hash units' (position, query)-major order); lane = proof, each lane reads
// its proof's segment [r*seg, (r+1)*seg) in 8-word blocks
template <int MODE>
__global__ void __launch_bounds__(256) k_stream(const uint64_t* __restrict__ src, int n, int64_t words, int R, int spin, uint64_t* out) {
  const int unit = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int NPB = n >> 6;
  if (unit >= NPB * R) return;
  const int pb = unit % NPB, r = unit / NPB;
  const int p = pb * 64 + (threadIdx.x & 63);
  const int64_t seg = words / R, w0 = r * seg;
  uint64_t acc = p, m = 0x9E3779B97F4A7C15ull;
  for (int64_t w = w0; w + 8 <= w0 + seg; w += 8) {
    uint64_t v[8];
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = src[(int64_t)p * words + w + j];
    } else if (MODE == 1) {
      const u64x2* q = (const u64x2*)(src + (int64_t)p * words + w);
#pragma unroll
      for (int j = 0; j < 4; j++) { u64x2 t = q[j]; v[2 * j] = t.x; v[2 * j + 1] = t.y; }
    } else {
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = src[(w + j) * n + p];
    }
#pragma unroll
    for (int j = 0; j < 8; j++) acc ^= v[j];
    for (int s = 0; s < spin; s++) acc = acc * m + (acc >> 29);
  }
  out[(int64_t)r * n + p] = acc;
}

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: %s mode spin [n] [words]\n", argv[0]); return 2; }
  const int mode = atoi(argv[1]), spin = atoi(argv[2]);
  const int n = argc > 3 ? atoi(argv[3]) : 4096;
  const int64_t words = argc > 4 ? atoll(argv[4]) : 15872;
  const int R = argc > 5 ? atoi(argv[5]) : 64;
  if (mode < 0 || mode > 2 || spin < 0 || n <= 0 || n % 64 || R <= 0 || words % (8 * R)) { fprintf(stderr, "bad arguments\n"); return 2; }
  const size_t bytes = (size_t)n * words * 8;
  uint64_t *d, *o;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&o, (size_t)n * R * 8));
  CK(hipMemset(d, 0x5a, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto launch = [&]() {
    const unsigned g = (unsigned)(((n >> 6) * R + 3) / 4);
    if (mode == 0) k_stream<0><<<g, 256>>>(d, n, words, R, spin, o);
    else if (mode == 1) k_stream<1><<<g, 256>>>(d, n, words, R, spin, o);
    else k_stream<2><<<g, 256>>>(d, n, words, R, spin, o);
  };
  launch();
  CK(hipDeviceSynchronize());
  const int reps = 3;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  CK(hipGetLastError());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("{\"mode\": %d, \"spin\": %d, \"n\": %d, \"R\": %d, \"words\": %lld, \"bytes_per_launch\": %zu, \"ms_per_launch\": %.4f, \"GBps\": %.1f}\n",
         mode, spin, n, R, (long long)words, bytes, ms / reps, bytes / (ms / reps * 1e-3) / 1e9);
  CK(hipFree(d)); CK(hipFree(o));
  return 0;
}
