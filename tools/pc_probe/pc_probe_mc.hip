// Phase timing of pc_solve_mc_kernel (wall_clock64 marks of workgroup 0,
// MMB_PC_PROBE build) and its PC against the one-workgroup solve.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DMMB_PC_PROBE -include ../diag/diag_hooks.h -I../../include \
//     pc_probe_mc.hip ../../multimodal-baselines_amd/csrc/host_rng.cpp \
//     ../../multimodal-baselines_amd/csrc/probe_kernels.hip -o pc_probe_mc
#include "../../multimodal-baselines_amd/csrc/pc_kernels.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

int main(int argc, char** argv) {
  // argv[1] = "cold": a 1 GiB device copy before every solve (caches and
  // the instruction cache hold other data, as inside a step)
  const bool cold = argc > 1 && argv[1][0] == 'c';
  void *cpa = nullptr, *cpb = nullptr;
  if (cold) {
    (void)hipMalloc(&cpa, size_t{1} << 30);
    (void)hipMalloc(&cpb, size_t{1} << 30);
  }
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
  void* ws;
  int32_t* flag;
  (void)hipMalloc(&dG, D * D * 8);
  (void)hipMalloc(&dz, D * k * 8);
  (void)hipMalloc(&dpc, D * 8);
  (void)hipMalloc(&ws, mmb_pc_solve_mc_ws_bytes(D));
  (void)hipMalloc(&flag, 4);
  (void)hipMemset(flag, 0, 4);
  (void)hipMemcpy(dG, G.data(), D * D * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dz, z0.data(), D * k * 8, hipMemcpyHostToDevice);
  int rate = 0;
  (void)hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);  // kHz
  for (int rep = 0; rep < 5; ++rep) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    if (cold) (void)mmb_probe_copy(cpa, cpb, int64_t{1} << 30, 512, 0, 0);  // a kernel, not a DMA copy
    (void)hipEventRecord(a, 0);
    const int rc = mmb_pc_solve_mc(dG, D, dz, k, 1, 7, 0, dpc, ws, flag, 0);
    (void)hipEventRecord(b, 0);
    (void)hipDeviceSynchronize();
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    unsigned long long t[64];
    (void)hipMemcpyFromSymbol(t, HIP_SYMBOL(mmb::g_pc_probe), sizeof(t));
    auto us = [&](int i, int j) { return (double)(t[j] - t[i]) * 1e3 / rate; };
    printf("rep %d rc %d: kernel+memset %.1f us | gram0 %.1f", rep, rc, ms * 1e3, us(0, 1));
    // rounds (r06: 4 at n_iter = 7, the first three by G2): wave 0's partials
    // + publish + wait, its gather, the join (the last wave's factor), then
    // B_{r+1} = H M^T and W_{r+1}
    int prev = 1;
    for (int r = 0; r < 4; ++r) {
      printf(" | r%d pub+wait %.1f gather %.1f join %.1f rmul+W %.1f", r, us(prev, 2 + 3 * r),
             us(2 + 3 * r, 3 + 3 * r), us(3 + 3 * r, 44 + 2 * r), us(44 + 2 * r, 45 + 2 * r));
      prev = 45 + 2 * r;
    }
    printf(" | last: chol || H pub+wait %.1f Z, gather, GZ %.1f", us(prev, 44 + 14), us(44 + 14, 45 + 14));
    printf(" | tail gather+grams %.1f rr %.1f eig %.1f out %.1f", us(45 + 14, 40), us(40, 41), us(41, 42),
           us(42, 43));
    printf(" | last eq-chol %.2f (equilibrate %.2f factor %.2f substitute %.2f store %.2f)", us(30, 34),
           us(30, 37), us(37, 38), us(38, 39), us(39, 34));
    printf(" | tail chol: factor %.2f substitute %.2f", us(31, 32), us(32, 33));
    printf(" | r3 rmul+W: tiles %.2f barrier %.2f sum %.2f\n", us(44 + 6, 35), us(35, 36), us(36, 45 + 6));
  }
  int32_t hflag = 0;
  (void)hipMemcpy(&hflag, flag, 4, hipMemcpyDeviceToHost);
  std::vector<double> pc(D), pc1(D);
  (void)hipMemcpy(pc.data(), dpc, D * 8, hipMemcpyDeviceToHost);
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
    printf("one-workgroup solve %.1f us\n", ms * 1e3);
  }
  (void)hipMemcpy(pc1.data(), dpc, D * 8, hipMemcpyDeviceToHost);
  double md = 0;
  for (int i = 0; i < D; ++i) md = std::max(md, std::fabs(pc[i] - pc1[i]));
  printf("flag %d | pc[0..3] %.12f %.12f %.12f | max|mc - one-wg| %.3e\n", hflag, pc[0], pc[1], pc[2], md);
  return 0;
}
