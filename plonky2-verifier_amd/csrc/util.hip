// util.hip — measurement helpers exported through the C-ABI (include/p2v.h): the device-side
// status check a caller folds into every launch it times, and the shader-clock probe.  Neither
// touches a verifier's buffers; both are enqueued on the caller's stream.
#include <hip/hip_runtime.h>
#include <cstdint>

// counters[0] += #{i < n : results[i] != expect[i]}; counters[1] += 1 (this check ran).  One
// workgroup-reduced atomic per 256 statuses; expect may be shorter than results' batch only if
// the caller passes the shorter n.
extern "C" __global__ void __launch_bounds__(256) k_count_mismatches(const int8_t* results, const int8_t* expect, int64_t n,
                                                                     unsigned long long* counters) {
  __shared__ unsigned int part[4];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool bad = i < n && results[i] != expect[i];
  const unsigned long long m = __ballot(bad);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) part[wave] = (unsigned int)__popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int s = part[0] + part[1] + part[2] + part[3];
    if (s) atomicAdd(&counters[0], (unsigned long long)s);
    if (blockIdx.x == 0) atomicAdd(&counters[1], 1ull);
  }
}

// One wave per workgroup: lane 0 writes (XCC id, shader-clock counter, 100 MHz real-time counter)
// to stamps[3 * blockIdx.x ..].  Two probes around a timed pass give, per XCD, the shader clock
// the chip held over it: d(memtime) / d(memrealtime) x 100 MHz (MI355X_MICROARCH.md, DVFS item 6).
extern "C" __global__ void __launch_bounds__(64) k_clock_probe(unsigned long long* stamps) {
  unsigned int xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned long long r = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): both counters are back
  if (threadIdx.x == 0) {
    unsigned long long* o = stamps + 3 * blockIdx.x;
    o[0] = xcc;
    o[1] = t;
    o[2] = r;
  }
}
