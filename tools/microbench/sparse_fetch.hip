// sparse_fetch.hip — calibrates rocprofv3's FETCH_SIZE for the chain kernel's read pattern
// (k_merkle_cse): the 64 lanes of a wave read one 8-B word each from rows of
// the tiled layout, but only S of the 16 words of every 128-B line are wanted by the wave, and
// the rest of the line is read by other waves long after (or never).  The guide's FETCH_SIZE
// correction (x2, MI355X_MICROARCH.md "HBM") is calibrated for wide coalesced streaming reads
// only; this measures what the counter reports, and what the link moves (time), when a line is
// touched by S lanes and never again.
//
//   ./sparse_fetch <S> [MiB]     S in {1,2,4,8,16}: lanes per 128-B line (16 = dense rows)
//
// Every line of the buffer (MiB, default 2048: past the 256 MiB Infinity Cache) is touched by
// exactly one wave, at S word positions chosen by a per-line hash (as the proofs of a 16-proof
// line fall into the chain buckets), so each launch reads every line once: the line bytes are
// the buffer's bytes, and the words actually used are S/16 of them.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

// one wave covers 64 / S lines; lane l reads word slot (l % S) of line (l / S): S distinct word
// offsets within the line, a random S-subset of its 16 words (a rotation by the line's hash)
__global__ void __launch_bounds__(256) k_sparse(const uint64_t* __restrict__ src, int64_t lines, int S, uint64_t* out) {
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int per = 64 / S;
  const int64_t line = wave * per + lane / S;
  uint64_t v = 0;
  if (line < lines) {
    const int slot = lane % S;
    const uint32_t rot = mix((uint32_t)line) & 15;
    const int word = (int)((rot + (uint32_t)slot * (16 / S)) & 15);
    v = src[line * 16 + word];
  }
  // one store per wave keeps the loads live without adding traffic worth counting
  v = __builtin_amdgcn_readfirstlane((uint32_t)v) ^ v;
  if (v == 0x123456789ull) out[wave & 1023] = v;
}

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: %s S [MiB]\n", argv[0]); return 2; }
  const int S = atoi(argv[1]);
  const int64_t mib = argc > 2 ? atoll(argv[2]) : 2048;
  if (S != 1 && S != 2 && S != 4 && S != 8 && S != 16) { fprintf(stderr, "S must be 1, 2, 4, 8 or 16\n"); return 2; }
  if (mib < 1 || mib > 16384) { fprintf(stderr, "MiB out of range\n"); return 2; }
  const size_t bytes = (size_t)mib << 20;
  const int64_t lines = (int64_t)(bytes / 128);
  const int64_t waves = (lines + (64 / S) - 1) / (64 / S);
  const unsigned grid = (unsigned)((waves + 3) / 4);
  uint64_t *d, *o;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&o, 1024 * 8));
  CK(hipMemset(d, 0x5a, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  k_sparse<<<grid, 256>>>(d, lines, S, o);
  CK(hipDeviceSynchronize());
  const int reps = 5;
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) k_sparse<<<grid, 256>>>(d, lines, S, o);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  CK(hipGetLastError());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double t = ms / reps;
  printf("{\"S\": %d, \"line_bytes_per_launch\": %zu, \"used_bytes_per_launch\": %lld, \"ms_per_launch\": %.4f, "
         "\"line_GBps\": %.1f}\n", S, bytes, (long long)(lines * S * 8), t, bytes / (t * 1e-3) / 1e9);
  CK(hipFree(d)); CK(hipFree(o));
  return 0;
}
