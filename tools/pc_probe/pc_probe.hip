// Phase timing of pc_solve_kernel (wall_clock64 marks, MMB_PC_PROBE build).
//   hipcc -O3 --offload-arch=gfx950 -DMMB_PC_PROBE -I../../include \
//     -I../../multimodal-baselines_amd/csrc pc_probe.hip ../../multimodal-baselines_amd/csrc/host_rng.cpp -o pc_probe
#include "../../multimodal-baselines_amd/csrc/pc_kernels.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

int main() {
  const int D = 300, k = 11, n = 4096;
  std::mt19937_64 rng(1);
  std::normal_distribution<double> nd;
  std::vector<double> X(static_cast<size_t>(n) * D), G(D * D, 0.0), z0(D * k);
  std::vector<double> g(D);
  for (auto& v : g) v = nd(rng);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < D; ++j) X[i * D + j] = 0.4 * nd(rng) + 0.3 * g[j];
  for (int i = 0; i < n; ++i)
    for (int a = 0; a < D; ++a)
      for (int b = 0; b < D; ++b) G[a * D + b] += X[i * D + a] * X[i * D + b];
  for (auto& v : z0) v = nd(rng);
  double *dG, *dz, *dpc;
  (void)hipMalloc(&dG, D * D * 8);
  (void)hipMalloc(&dz, D * k * 8);
  (void)hipMalloc(&dpc, D * 8);
  (void)hipMemcpy(dG, G.data(), D * D * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dz, z0.data(), D * k * 8, hipMemcpyHostToDevice);
  int rate = 0;
  (void)hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);  // kHz
  for (int rep = 0; rep < 3; ++rep) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, 0);
    mmb_pc_solve(dG, D, dz, k, 1, 7, 0, dpc, 0);
    (void)hipEventRecord(b, 0);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    unsigned long long t[64];
    (void)hipMemcpyFromSymbol(t, HIP_SYMBOL(mmb::g_pc_probe), sizeof(t));
    auto us = [&](int i, int j) { return (double)(t[j] - t[i]) * 1e3 / rate; };
    printf("rep %d: kernel %.1f us | orth0 %.1f", rep, ms * 1e3, us(0, 1));
    for (int it = 0; it < 7; ++it) printf(" | gz%d %.1f orth %.1f", it, us(it ? 1 + 2 * it : 1, 2 + 2 * it), us(2 + 2 * it, 3 + 2 * it));
    printf(" | gz_final %.1f | rr %.1f | jacobi %.1f | out %.1f\n", us(15, 40), us(40, 41), us(41, 42), us(42, 43));
  }
  std::vector<double> pc(D), pc_old(D);
  (void)hipMemcpy(pc.data(), dpc, D * 8, hipMemcpyDeviceToHost);
  for (int rep = 0; rep < 2; ++rep) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, 0);
    mmb::pc_solve_kernel<<<1, mmb::kSolveNT>>>(dG, D, dz, k, 1, 7, 0, dpc);
    (void)hipEventRecord(b, 0);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("old kernel %.1f us\n", ms * 1e3);
  }
  (void)hipMemcpy(pc_old.data(), dpc, D * 8, hipMemcpyDeviceToHost);
  double md = 0;
  for (int i = 0; i < D; ++i) md = std::max(md, std::fabs(pc[i] - pc_old[i]));
  printf("pc[0..3] %.9f %.9f %.9f | max|new-old| %.3e\n", pc[0], pc[1], pc[2], md);
  return 0;
}
