// Bandwidth probes: the same-process HBM ceilings the bench's rooflines are
// quoted against ("also report a measured stream-copy
// ceiling").  No reference counterpart.
//
// Both kernels stream 16-byte words with four independent loads in flight per
// lane, grid-strided over a grid of a few workgroups per CU, with the default
// or the non-temporal cache policy (nt):
//   probe_copy_kernel: dst = src            (read + write bytes)
//   probe_read_kernel: sink[block] = f(src) (read bytes; a per-block XOR of
//                      the words keeps the loads alive)
#include <algorithm>

#include "mmb_common.h"

namespace mmb {
namespace {

typedef float nf4 __attribute__((ext_vector_type(4)));
constexpr int kProbeThreads = 256;
constexpr int kProbeUnroll = 4;

template <bool NT>
__device__ __forceinline__ nf4 ld4(const nf4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st4(nf4 v, nf4* p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <bool NT>
__global__ __launch_bounds__(kProbeThreads) void probe_copy_kernel(const nf4* __restrict__ src,
                                                                   nf4* __restrict__ dst,
                                                                   int64_t n4) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kProbeThreads;
  int64_t i = static_cast<int64_t>(blockIdx.x) * kProbeThreads + threadIdx.x;
  for (; i + (kProbeUnroll - 1) * stride < n4; i += kProbeUnroll * stride) {
    nf4 v[kProbeUnroll];
#pragma unroll
    for (int u = 0; u < kProbeUnroll; ++u) v[u] = ld4<NT>(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < kProbeUnroll; ++u) st4<NT>(v[u], dst + i + u * stride);
  }
  for (; i < n4; i += stride) st4<NT>(ld4<NT>(src + i), dst + i);
}

template <bool NT>
__global__ __launch_bounds__(kProbeThreads) void probe_read_kernel(const nf4* __restrict__ src,
                                                                   int64_t n4,
                                                                   uint32_t* __restrict__ sink) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kProbeThreads;
  int64_t i = static_cast<int64_t>(blockIdx.x) * kProbeThreads + threadIdx.x;
  uint32_t acc = 0;
  for (; i + (kProbeUnroll - 1) * stride < n4; i += kProbeUnroll * stride) {
    nf4 v[kProbeUnroll];
#pragma unroll
    for (int u = 0; u < kProbeUnroll; ++u) v[u] = ld4<NT>(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < kProbeUnroll; ++u)
      acc ^= __float_as_uint(v[u].x) ^ __float_as_uint(v[u].y) ^ __float_as_uint(v[u].z) ^
             __float_as_uint(v[u].w);
  }
  for (; i < n4; i += stride) {
    const nf4 v = ld4<NT>(src + i);
    acc ^= __float_as_uint(v.x) ^ __float_as_uint(v.y) ^ __float_as_uint(v.z) ^ __float_as_uint(v.w);
  }
  // one word per block (a vector store; every lane's value folded in)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc ^= static_cast<uint32_t>(__shfl_xor(static_cast<int>(acc), o, kWave));
  __shared__ uint32_t s_acc[kProbeThreads / kWave];
  if ((threadIdx.x & (kWave - 1)) == 0) s_acc[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t a = 0;
#pragma unroll
    for (int w = 0; w < kProbeThreads / kWave; ++w) a ^= s_acc[w];
    sink[blockIdx.x] = a;
  }
}

int probe_grid(int64_t n4, int blocks) {
  const int64_t need = (n4 + kProbeThreads - 1) / kProbeThreads;
  return static_cast<int>(need < blocks ? (need > 0 ? need : 1) : blocks);
}

__global__ void zero_words_kernel(uint32_t* p, int64_t n) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    p[i] = 0u;
}

}  // namespace

// (declared in mmb_common.h: the library's graph-safe replacement of
// hipMemsetAsync)
int zero_words_async(void* p, int64_t n, hipStream_t stream) {
  if (n <= 0) return 0;
  const int grid = static_cast<int>(std::min<int64_t>(ceil_div(n, 256), 1024));
  zero_words_kernel<<<grid, 256, 0, stream>>>(static_cast<uint32_t*>(p), n);
  return static_cast<int>(hipGetLastError());
}

}  // namespace mmb

using namespace mmb;

extern "C" int mmb_probe_copy(const void* src, void* dst, int64_t bytes, int blocks, int nt,
                              hipStream_t stream) {
  MMB_REQUIRE(src && dst && bytes > 0 && bytes % 16 == 0 && blocks > 0);
  MMB_REQUIRE(reinterpret_cast<uintptr_t>(src) % 16 == 0 && reinterpret_cast<uintptr_t>(dst) % 16 == 0);
  const int64_t n4 = bytes / 16;
  if (nt)
    probe_copy_kernel<true><<<probe_grid(n4, blocks), kProbeThreads, 0, stream>>>(
        static_cast<const nf4*>(src), static_cast<nf4*>(dst), n4);
  else
    probe_copy_kernel<false><<<probe_grid(n4, blocks), kProbeThreads, 0, stream>>>(
        static_cast<const nf4*>(src), static_cast<nf4*>(dst), n4);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_probe_read(const void* src, int64_t bytes, int blocks, int nt, uint32_t* sink,
                              hipStream_t stream) {
  MMB_REQUIRE(src && sink && bytes > 0 && bytes % 16 == 0 && blocks > 0);
  MMB_REQUIRE(reinterpret_cast<uintptr_t>(src) % 16 == 0);
  const int64_t n4 = bytes / 16;
  if (nt)
    probe_read_kernel<true><<<probe_grid(n4, blocks), kProbeThreads, 0, stream>>>(
        static_cast<const nf4*>(src), n4, sink);
  else
    probe_read_kernel<false><<<probe_grid(n4, blocks), kProbeThreads, 0, stream>>>(
        static_cast<const nf4*>(src), n4, sink);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}
