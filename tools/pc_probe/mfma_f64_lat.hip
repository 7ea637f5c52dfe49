// Latency / issue rate of v_mfma_f64_16x16x4_f64 on one wave (r05): a chain
// of dependent MFMAs (same accumulator) and 4 independent chains
// interleaved, timed with s_memtime inside the wave.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 mfma_f64_lat.hip -o mfma_f64_lat
#include <hip/hip_runtime.h>

#include <cstdio>

using f64x4 = __attribute__((ext_vector_type(4))) double;

template <int CHAINS>
__global__ void lat_kernel(const double* in, double* out, long long* cyc, int n) {
  const int lane = threadIdx.x;
  double a = in[lane], b = in[64 + lane];
  f64x4 acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = {0, 0, 0, 0};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += acc[c][0] + acc[c][3];
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[lane] = s;
  if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
  double *in, *out;
  long long* cyc;
  (void)hipMalloc(&in, 128 * 8);
  (void)hipMalloc(&out, 64 * 8);
  (void)hipMalloc(&cyc, 8);
  (void)hipMemset(in, 0, 128 * 8);
  const int n = 4096;
  for (int rep = 0; rep < 3; ++rep) {
    long long c1 = 0, c4 = 0;
    lat_kernel<1><<<1, 64>>>(in, out, cyc, n);
    (void)hipMemcpy(&c1, cyc, 8, hipMemcpyDeviceToHost);
    lat_kernel<4><<<1, 64>>>(in, out, cyc, n);
    (void)hipMemcpy(&c4, cyc, 8, hipMemcpyDeviceToHost);
    printf("s_memtime cycles per MFMA: dependent chain %.1f, 4 independent chains %.1f\n",
           double(c1) / n, double(c4) / (4.0 * n));
  }
  int rate = 0;
  (void)hipDeviceGetAttribute(&rate, hipDeviceAttributeClockRate, 0);
  printf("clock rate attribute %d kHz (s_memtime counts the shader clock)\n", rate);
  return 0;
}
