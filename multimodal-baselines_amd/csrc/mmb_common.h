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

// Sums over the 16 lanes of a DPP row (lanes 16k .. 16k+15), every lane
// receiving the row's total: quad_perm [1,0,3,2], [2,3,0,1], then
// row_half_mirror and row_mirror -- register-to-register moves, where
// __shfl_xor is an LDS-unit ds_bpermute waited on per step.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(u & 0xffffffffu), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(u >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((static_cast<unsigned long long>(static_cast<unsigned>(hi)) << 32) |
                              static_cast<unsigned>(lo));
}
constexpr int kDppQuad1032 = 0xB1, kDppQuad2301 = 0x4E, kDppRowHalfMirror = 0x141,
              kDppRowMirror = 0x140;
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f32<kDppQuad1032>(v);
  v += dpp_f32<kDppQuad2301>(v);
  v += dpp_f32<kDppRowHalfMirror>(v);
  v += dpp_f32<kDppRowMirror>(v);
  return v;
}
// 64-lane sum in f64, fixed order: the four row sums combined from lanes 0,
// 16, 32, 48 (wave-uniform result)
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_f64<kDppQuad1032>(v);
  v += dpp_f64<kDppQuad2301>(v);
  v += dpp_f64<kDppRowHalfMirror>(v);
  v += dpp_f64<kDppRowMirror>(v);
  auto rl = [&](int l) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane(static_cast<int>(u & 0xffffffffu), l);
    const unsigned hi = __builtin_amdgcn_readlane(static_cast<int>(u >> 32), l);
    return __longlong_as_double((static_cast<unsigned long long>(hi) << 32) | lo);
  };
  return (rl(0) + rl(16)) + (rl(32) + rl(48));
}
__device__ __forceinline__ float wave_sum_dpp_f32(float v) {
  v = row16_sum(v);
  auto rl = [&](int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); };
  return (rl(0) + rl(16)) + (rl(32) + rl(48));
}
// 64-lane max (exact in any order) by DPP within rows + readlane: no
// ds_bpermute round trips (wave-uniform result; fmaxf drops NaN)
__device__ __forceinline__ float wave_max_dpp_f32(float v) {
  v = fmaxf(v, dpp_f32<kDppQuad1032>(v));
  v = fmaxf(v, dpp_f32<kDppQuad2301>(v));
  v = fmaxf(v, dpp_f32<kDppRowHalfMirror>(v));
  v = fmaxf(v, dpp_f32<kDppRowMirror>(v));
  auto rl = [&](int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); };
  return fmaxf(fmaxf(rl(0), rl(16)), fmaxf(rl(32), rl(48)));
}
// Broadcast of lane l's double (l wave-uniform): two v_readlane, no LDS.
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane(static_cast<int>(u & 0xffffffffu), l);
  const unsigned hi = __builtin_amdgcn_readlane(static_cast<int>(u >> 32), l);
  return __longlong_as_double((static_cast<unsigned long long>(hi) << 32) | lo);
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

// fp16 x3 projection operands (mm2_kernels.hip, the fused stream kernel)
using half8 = __attribute__((ext_vector_type(8))) _Float16;
using f32x4 = __attribute__((ext_vector_type(4))) float;

// The weighted text sum sum_t w_t E_t of a row from the a2 row x = sum / count
// that mmb_mm2_stream writes (count = count_nonzero(w), aux[0]): x * count,
// within one rounding of the sum; 0 for a row whose weights are all zero
// (x is then 0/0 = NaN, like the reference's a2, but the MMB2 text term is 0).
__device__ __forceinline__ float text_sum(float x, float count) {
  return count != 0.f ? x * count : 0.f;
}

// 16-byte slot swizzle of a 64-byte LDS row (4 slots of 8 halves): row r
// keeps data slot j at position j ^ swz(r).  A 64-byte row puts slot
// position p of row r on bank set 4 (r mod 4) + p, so a ds_read_b128 lane
// group (16 lanes: {0-3,12-15,20-27}, {4-11,16-19,28-31}, and the same +32)
// is conflict-free iff its 16 (row mod 4, position) pairs differ.  For the
// 16x16x32 fragment reads (lane l: row 16 t + (l & 15), data slot l >> 4)
// the groups read rows {0-3, 12-15} at one slot and rows {4-11} at the
// next: swz over the four 4-row groups of a 16-row tile = 0, 2, 3, 1 makes
// every group conflict-free (the former (r >> 2) & 3 left them 2-way:
// SQ_LDS_BANK_CONFLICT = 48 % of the kernel's LDS cycles, r02 counters).
__host__ __device__ constexpr int x3_swz(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Zero n 32-bit words with a kernel (probe_kernels.hip).  Used wherever the
// library must clear a buffer on the caller's stream: a hipMemsetAsync
// captured into a HIP graph wrote address-like garbage into its destination
// on every replay after the first (r05, tools/dbg/replay_cause.py:
// gpurun_out r05a -- the PC solve's control words read [0x14ABxxxx, 0x7BE2]),
// so no entry point enqueues a memset node.  Returns 0 or a hipError_t.
int zero_words_async(void* p, int64_t n, hipStream_t stream);

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
