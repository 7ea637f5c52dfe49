// The PC solve's per-round block update in isolation (r05): B = H M^T tile by
// tile over 8 waves with each wave's tile Grams accumulated, as in
// pc_solve_mc_kernel, timed by s_memtime on wave 0.  Variants:
//   0: Y tile stored to LDS and read back for the Gram (the r05 kernel)
//   1: the Gram from the Y tile's MFMA accumulator registers (no round trip)
//   2: the products only (no Gram); 3: the MFMAs on register operands;
//   4: the LDS reads with adds for the MFMAs; 5: the products, no Y store
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 rmul_bench.hip -o rmul_bench
#include <hip/hip_runtime.h>

#include <cstdio>

using f64x4 = __attribute__((ext_vector_type(4))) double;
constexpr int kW = 16, kT = 19, kNW = 8;

template <int V>
__global__ __launch_bounds__(512) void rmul_kernel(const double* in, double* out, long long* cyc, int reps) {
  __shared__ double sZ[kT * 16 * kW], sY[kT * 16 * kW], sM[256], part[kNW * 256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < kT * 16 * kW; e += 512) sZ[e] = in[e % 4096];
  if (tid < 256) sM[tid] = in[tid] * 0.5;
  __syncthreads();
  long long t0 = 0;
  for (int rep = 0; rep < reps; ++rep) {
    if (rep == 1 && tid == 0) t0 = __builtin_amdgcn_s_memtime();
    f64x4 pa = {0, 0, 0, 0};
    for (int tt = wave; tt < kT; tt += kNW) {
      f64x4 acc = {0, 0, 0, 0};
      if constexpr (V == 3) {  // the MFMAs on register operands
#pragma unroll
        for (int st = 0; st < 4; ++st) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[st] + tt, pa[3 - st], acc, 0, 0, 0);
      } else if constexpr (V == 4) {  // the LDS reads, adds instead of MFMAs
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          const int m = 4 * st + (lane >> 4);
          acc[st] += sZ[(tt * 16 + (lane & 15)) * kW + m] * sM[(lane & 15) * kW + m];
        }
      } else {
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          const int m = 4 * st + (lane >> 4);
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sZ[(tt * 16 + (lane & 15)) * kW + m], sM[(lane & 15) * kW + m],
                                                     acc, 0, 0, 0);
        }
      }
      if constexpr (V == 3 || V == 4) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) pa[reg] += acc[reg];
      }
      if constexpr (V != 5)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) sY[(tt * 16 + (lane >> 4) + 4 * reg) * kW + (lane & 15)] = acc[reg];
      else
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) pa[reg] += acc[reg];
      if constexpr (V == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          const double y = sY[(tt * 16 + 4 * st + (lane >> 4)) * kW + (lane & 15)];
          pa = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, pa, 0, 0, 0);
        }
      } else if constexpr (V == 1) {
#pragma unroll
        for (int st = 0; st < 4; ++st) pa = __builtin_amdgcn_mfma_f64_16x16x4f64(acc[st], acc[st], pa, 0, 0, 0);
      }
    }
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) part[wave * 256 + ((lane >> 4) + 4 * reg) * 16 + (lane & 15)] = pa[reg];
    __syncthreads();
    if (tid < 256) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < kNW; ++w) s += part[w * 256 + tid];
      sM[tid] = s * 1e-30 + sM[tid];
    }
    __syncthreads();
  }
  if (tid == 0) cyc[0] = __builtin_amdgcn_s_memtime() - t0;
  if (tid < 256) out[tid] = sM[tid] + sY[tid];
}

int main() {
  double *in, *out;
  long long* cyc;
  (void)hipMalloc(&in, 4096 * 8);
  (void)hipMalloc(&out, 256 * 8);
  (void)hipMalloc(&cyc, 8);
  (void)hipMemset(in, 0, 4096 * 8);
  const int reps = 101;
  for (int r = 0; r < 3; ++r) {
    long long c[6];
    rmul_kernel<0><<<1, 512>>>(in, out, cyc, reps);
    (void)hipMemcpy(&c[0], cyc, 8, hipMemcpyDeviceToHost);
    rmul_kernel<1><<<1, 512>>>(in, out, cyc, reps);
    (void)hipMemcpy(&c[1], cyc, 8, hipMemcpyDeviceToHost);
    rmul_kernel<2><<<1, 512>>>(in, out, cyc, reps);
    (void)hipMemcpy(&c[2], cyc, 8, hipMemcpyDeviceToHost);
    rmul_kernel<3><<<1, 512>>>(in, out, cyc, reps);
    (void)hipMemcpy(&c[3], cyc, 8, hipMemcpyDeviceToHost);
    rmul_kernel<4><<<1, 512>>>(in, out, cyc, reps);
    (void)hipMemcpy(&c[4], cyc, 8, hipMemcpyDeviceToHost);
    rmul_kernel<5><<<1, 512>>>(in, out, cyc, reps);
    (void)hipMemcpy(&c[5], cyc, 8, hipMemcpyDeviceToHost);
    printf("cycles per update: LDS round trip %.0f | Gram from registers %.0f | products only %.0f | "
           "MFMAs on registers %.0f | LDS reads, no MFMA %.0f | products, no store %.0f\n",
           double(c[0]) / (reps - 1), double(c[1]) / (reps - 1), double(c[2]) / (reps - 1),
           double(c[3]) / (reps - 1), double(c[4]) / (reps - 1), double(c[5]) / (reps - 1));
  }
  return 0;
}
