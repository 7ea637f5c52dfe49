// numpy RandomState(seed).normal(size=n) restated in C++ (host side of libmmb).
//
// scikit-learn's randomized SVD draws its start block Omega from
// `check_random_state(0).normal(size=(rows, k))` (sklearn 1.7.2
// utils/extmath.py:297).  numpy's legacy RandomState is MT19937 seeded with
// init_genrand(seed) (numpy/random/_mt19937.pyx _legacy_seeding ->
// mt19937_seed) and its normal() is the legacy polar Box-Muller
// (numpy/random/src/legacy/legacy-distributions.c legacy_gauss) over
// 53-bit doubles (a>>5, b>>6).  Reproducing it bit for bit lets the device
// PC solver start from the reference's exact Omega without Python.
// Built with -ffp-contract=off so x1*x1 + x2*x2 is not fused (numpy's C is not).
#include <cmath>
#include <cstdint>

#include "mmb.h"

namespace {

struct MT19937 {
  uint32_t mt[624];
  int pos;
  explicit MT19937(uint32_t seed) {
    mt[0] = seed;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253U * (mt[i - 1] ^ (mt[i - 1] >> 30)) + static_cast<uint32_t>(i);
    pos = 624;
  }
  void regen() {
    static const uint32_t mag01[2] = {0x0U, 0x9908b0dfU};
    int kk = 0;
    uint32_t y;
    for (; kk < 624 - 397; ++kk) {
      y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
      mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1U];
    }
    for (; kk < 623; ++kk) {
      y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
      mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1U];
    }
    y = (mt[623] & 0x80000000U) | (mt[0] & 0x7fffffffU);
    mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1U];
    pos = 0;
  }
  uint32_t next32() {
    if (pos == 624) regen();
    uint32_t y = mt[pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
  }
  double next_double() {
    const int32_t a = static_cast<int32_t>(next32() >> 5), b = static_cast<int32_t>(next32() >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }
};

}  // namespace

extern "C" int mmb_host_randn(uint32_t seed, int64_t count, double* host_out) {
  if (count < 0 || (count > 0 && host_out == nullptr)) return MMB_EINVAL;
  MT19937 g(seed);
  bool has_gauss = false;
  double gauss = 0.0;
  for (int64_t i = 0; i < count; ++i) {
    if (has_gauss) {
      host_out[i] = gauss;
      has_gauss = false;
      continue;
    }
    double x1, x2, r2;
    do {
      x1 = 2.0 * g.next_double() - 1.0;
      x2 = 2.0 * g.next_double() - 1.0;
      r2 = x1 * x1 + x2 * x2;
    } while (r2 >= 1.0 || r2 == 0.0);
    const double f = std::sqrt(-2.0 * std::log(r2) / r2);
    gauss = f * x1;
    has_gauss = true;
    host_out[i] = f * x2;
  }
  return MMB_OK;
}
