// Shared device helpers for libmmb (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mmb.h"

#define MMB_LAUNCH_CHECK()                               \
  do {                                                   \
    hipError_t e_ = hipGetLastError();                   \
    if (e_ != hipSuccess) return static_cast<int>(e_);   \
  } while (0)

#define MMB_REQUIRE(cond) \
  do {                    \
    if (!(cond)) return MMB_EINVAL; \
  } while (0)

namespace mmb {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Sum within each 32-lane half of the wave (lanes l and l^k for k < 32).
__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// LDS ordering inside one wave (no workgroup barrier needed).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// CUs a launch on `stream` can use: the device's, or the subset a stream made
// by hipExtStreamCreateWithCUMask is restricted to (sif_kernels.hip).
int stream_cu_count(hipStream_t stream);

// Grid size for streaming kernels: enough workgroups to fill the stream's CUs
// several times over, capped so per-workgroup setup is amortised by a
// grid-stride loop.  Sized from the stream's CUs: a grid made for 256 CUs on
// a 160-CU stream queues a partial round of late workgroups (a tail).
inline int stream_grid(int64_t units, int per_cu, hipStream_t stream) {
  int64_t cap = static_cast<int64_t>(stream_cu_count(stream)) * per_cu;
  return static_cast<int>(units < cap ? (units > 0 ? units : 1) : cap);
}

}  // namespace mmb
