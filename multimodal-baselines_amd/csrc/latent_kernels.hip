// Latent-optimisation likelihoods for MI355X.
//
// The reference scores a batch of B latent sentence embeddings l_b under
//   * the angular word model (losses.py:68-95, get_word_log_prob_angular2):
//       c_bv = cos(l_b, W_v) over the WHOLE vocabulary V, Z_b = sum_v (1 - acos(c_bv)/pi),
//       alpha_b = 1/(a Z_b + 1),  P_bt = alpha_b w_bt + (1-alpha_b)(1 - acos(cos(l_b, e_bt))/pi)/Z_b,
//       lp_b = sum_t mask_bt log P_bt
//     — torch broadcasting materialises [B, V, 300] for the cosine;
//   * independent Gaussians per modality combination (losses.py:13-33,
//     216-274): sum_t sum_f mask (log(1/sqrt(2 pi s^2)) - (x - mu)^2 / (2 s^2)),
//     materialising [B, T, F] per combination every step.
//
// Here:
//   * Z_b (and, for the backward pass, G_b = sum_v W_v / s_bv and
//     h_b = sum_v c_bv / s_bv with s = sqrt(1 - c^2)) come from ONE fused
//     kernel per batch: the cosine block C^T = Wn U^T and the gradient block
//     G = R Wn (R = 1/s) are both fp32 MFMA 16x16x4 (exact f32 products, like
//     the reference's f32 arithmetic), acos / rsqrt in registers between them —
//     nothing [B, V] ever reaches memory.  The table is normalised once
//     (Wn = W / max(|W|, 1e-8), torch's cosine_similarity).
//   * the Gaussian term is a function of the per-utterance masked frame sums
//     M0 = sum_t m, M1 = sum_t m x, M2 = sum_t m x^2 only:
//       lp = sum_f M0 (-log s - log(2 pi)/2) - (M2 - 2 mu M1 + mu^2 M0) / (2 s^2),
//     exact algebra; the sums are streamed ONCE per data split (f64), so a step
//     costs O(B F) instead of O(B T F).  Gradients are closed-form too.
#include <algorithm>

#include "mmb_common.h"

namespace mmb {

using f32x4 = __attribute__((ext_vector_type(4))) float;
constexpr float kPi = 3.14159265358979323846f;
constexpr float kCosEps = 1e-8f;  // torch cosine_similarity eps

__host__ __device__ inline int pad16(int d) { return (d + 15) / 16 * 16; }

// ------------------------------------------------------------------ table
// Wn[v][0..Dp) = W[v] / max(||W[v]||, eps), zero padded; one wave per row.
__global__ __launch_bounds__(256) void word_normalize_kernel(const float* __restrict__ W, int64_t V,
                                                             int D, int Dp, float* __restrict__ Wn) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t nw = static_cast<int64_t>(gridDim.x) * (blockDim.x / kWave);
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * (blockDim.x / kWave) + threadIdx.x / kWave;
       v < V; v += nw) {
    float ss = 0.f;
    for (int k = lane; k < D; k += kWave) {
      const float x = W[v * D + k];
      ss = fmaf(x, x, ss);
    }
    const float n = fmaxf(sqrtf(wave_sum(ss)), kCosEps);
    for (int k = lane; k < Dp; k += kWave) Wn[v * Dp + k] = k < D ? W[v * D + k] / n : 0.f;
  }
}

// ------------------------------------------------------------------ Z / G / h
// Block (latent tile of 16, word split): 4 waves, each sweeping 16-word tiles.
//   first product  C^T[word][latent] = Wn[w0..w0+16) . U^T    (MFMA 16x16x4, K = Dp;
//                  a lane's dwordx4 of Wn / U covers the 4 k-steps of a 16-wide
//                  column block: the k order inside the block is permuted, the
//                  same way for both operands)
//   second product G[latent][col] += R[latent][word] Wn[word][col]: the C^T
//                  accumulator (word = 4 (l>>4) + r on registers, latent = l&15
//                  on the lane) IS the A operand of k-step r — no transpose.
// Partials per wave: [16 latents][Dp + 2] (G | Z | h), summed in a fixed
// order by word_finish_kernel (deterministic).
template <int NT>  // Dp / 16
__global__ __launch_bounds__(256) void word_zsum_kernel(const float* __restrict__ lat, int64_t B,
                                                        int D, const float* __restrict__ Wn,
                                                        int64_t V, int want_g,
                                                        float* __restrict__ part) {
  constexpr int Dp = 16 * NT;
  __shared__ __attribute__((aligned(16))) float sU[16 * Dp];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * 16;
  const int split = blockIdx.y, S = gridDim.y;
  // normalised latents of the tile (rows past B are zero)
  for (int i = wave; i < 16; i += 4) {
    const int64_t b = b0 + i;
    float ss = 0.f;
    if (b < B)
      for (int k = lane; k < D; k += kWave) ss = fmaf(lat[b * D + k], lat[b * D + k], ss);
    const float n = fmaxf(sqrtf(wave_sum(ss)), kCosEps);
    for (int k = lane; k < Dp; k += kWave) sU[i * Dp + k] = (b < B && k < D) ? lat[b * D + k] / n : 0.f;
  }
  __syncthreads();

  const int64_t ntiles = (V + 15) / 16;
  f32x4 g[NT];
#pragma unroll
  for (int c = 0; c < NT; ++c) g[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float zp = 0.f, hp = 0.f;
  const int lr = lane & 15, lk = lane >> 4;
  const float* urow = sU + lr * Dp + 4 * lk;
  for (int64_t wt = static_cast<int64_t>(split) * 4 + wave; wt < ntiles; wt += 4LL * S) {
    const int64_t w0 = wt * 16;
    const float* arow = Wn + min(w0 + lr, V - 1) * Dp + 4 * lk;
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NT; ++s) {
      const f32x4 a4 = *reinterpret_cast<const f32x4*>(arow + 16 * s);
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(urow + 16 * s);
#pragma unroll
      for (int t = 0; t < 4; ++t) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[t], b4[t], c, 0, 0, 0);
    }
    float rinv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool ok = w0 + 4 * lk + r < V;
      const float cv = c[r];
      zp += ok ? 1.f - acosf(cv) / kPi : 0.f;
      const float inv = 1.f / sqrtf(1.f - cv * cv);
      rinv[r] = ok ? inv : 0.f;
      hp += ok ? cv * inv : 0.f;
    }
    if (want_g) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float* brow = Wn + min(w0 + 4 * lk + t, V - 1) * Dp + lr;
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
          g[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(rinv[t], brow[16 * ct], g[ct], 0, 0, 0);
      }
    }
  }
  // Z, h: lane l has latent l&15's partial over its 4-word rows; sum the 4 groups
  zp += __shfl_xor(zp, 16, kWave);
  zp += __shfl_xor(zp, 32, kWave);
  hp += __shfl_xor(hp, 16, kWave);
  hp += __shfl_xor(hp, 32, kWave);
  const int64_t slot = (static_cast<int64_t>(blockIdx.x) * (4LL * S) + split * 4 + wave);
  float* pw = part + slot * 16 * (Dp + 2);
  if (lane < 16) {
    pw[lane * (Dp + 2) + Dp] = zp;
    pw[lane * (Dp + 2) + Dp + 1] = hp;
  }
  // G: lane l holds G[latent 4 (l>>4) + r][col 16 ct + (l&15)]
#pragma unroll
  for (int ct = 0; ct < NT; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) pw[(4 * lk + r) * (Dp + 2) + 16 * ct + lr] = want_g ? g[ct][r] : 0.f;
}

// Per-utterance token rows: gathered from the table by id (ids != nullptr) or dense.
struct TokSrc {
  const int32_t* ids;  // [B, L] (rows into `table`), or nullptr
  const float* table;  // [V, D]
  const float* dense;  // [B, L, D] when ids == nullptr
  int64_t V;
};
__device__ __forceinline__ const float* tok_row(const TokSrc& s, int64_t b, int L, int t, int D) {
  if (s.ids) {
    int64_t id = s.ids[b * L + t];
    if (id < 0) id += s.V;  // numpy-style wrap, like table[ids]
    id = min(max(id, static_cast<int64_t>(0)), s.V - 1);
    return s.table + id * D;
  }
  return s.dense + (b * L + t) * static_cast<int64_t>(D);
}

// One block per utterance: fixed-order sum of the partials (Z, h, G), the
// token cosines and lp_b.  State per b: [Z, alpha, h, |l|] and G [Dp].
__global__ __launch_bounds__(256) void word_finish_kernel(const float* __restrict__ lat, int64_t B,
                                                          int D, int Dp, const float* __restrict__ part,
                                                          int S, TokSrc tok, int L,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ mask, float a,
                                                          float* __restrict__ lp,
                                                          float* __restrict__ state,
                                                          float* __restrict__ gsum,
                                                          float* __restrict__ cos_out) {
  __shared__ float s_u[512];
  __shared__ double s_red[8];
  __shared__ float s_zahn[4];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const int64_t b = blockIdx.x;
  const int64_t tile = b / 16;
  const int i = static_cast<int>(b % 16);
  const int nslots = 4 * S;
  const float* pb = part + tile * nslots * 16 * (Dp + 2) + i * (Dp + 2);
  // G (per column, slots in order) and Z, h.  The slot loads are issued 32
  // at a time before they are summed (in slot order, the same f64 sum as a
  // plain loop): a load-add chain per slot cost one memory latency each
  // (106 us per call at B = 64, V = 3016: 192 slots).
  constexpr int kQ = 32;
  const int64_t qs = static_cast<int64_t>(16) * (Dp + 2);
  for (int k = tid; k < Dp; k += blockDim.x) {
    double s = 0.0;
    int q = 0;
    for (; q + kQ <= nslots; q += kQ) {
      float v[kQ];
#pragma unroll
      for (int u = 0; u < kQ; ++u) v[u] = pb[(q + u) * qs + k];
#pragma unroll
      for (int u = 0; u < kQ; ++u) s += v[u];
    }
    for (; q < nslots; ++q) s += pb[q * qs + k];
    if (gsum) gsum[b * Dp + k] = static_cast<float>(s);
  }
  if (wave == 0) {
    double z = 0.0, h = 0.0;
    for (int q = lane; q < nslots; q += kWave) {
      z += pb[static_cast<int64_t>(q) * 16 * (Dp + 2) + Dp];
      h += pb[static_cast<int64_t>(q) * 16 * (Dp + 2) + Dp + 1];
    }
    z = wave_sum(z);
    h = wave_sum(h);
    // latent norm
    float ss = 0.f;
    for (int k = lane; k < D; k += kWave) ss = fmaf(lat[b * D + k], lat[b * D + k], ss);
    const float n = sqrtf(wave_sum(ss));
    if (lane == 0) {
      const float zf = static_cast<float>(z);
      s_zahn[0] = zf;
      s_zahn[1] = 1.f / (zf * a + 1.f);
      s_zahn[2] = static_cast<float>(h);
      s_zahn[3] = n;
    }
  }
  __syncthreads();
  const float n = s_zahn[3], nc = fmaxf(n, kCosEps);
  for (int k = tid; k < D; k += blockDim.x) s_u[k] = lat[b * D + k] / nc;
  __syncthreads();
  const float Z = s_zahn[0], alpha = s_zahn[1];
  // tokens: one wave per token
  double acc = 0.0;
  for (int t = wave; t < L; t += 4) {
    const float* e = tok_row(tok, b, L, t, D);
    float ee = 0.f, eu = 0.f;
    for (int k = lane; k < D; k += kWave) {
      const float x = e[k];
      ee = fmaf(x, x, ee);
      eu = fmaf(x, s_u[k], eu);
    }
    ee = wave_sum(ee);
    eu = wave_sum(eu);
    const float c = eu / fmaxf(sqrtf(ee), kCosEps);
    const float score = 1.f - acosf(c) / kPi;
    const float P = alpha * w[b * L + t] + (1.f - alpha) * score / Z;
    if (lane == 0) {
      if (cos_out) cos_out[b * L + t] = c;
      acc += static_cast<double>(logf(P) * mask[b * L + t]);
    }
  }
  if (lane == 0) s_red[wave] = acc;
  __syncthreads();
  if (tid == 0) {
    lp[b] = static_cast<float>(s_red[0] + s_red[1] + s_red[2] + s_red[3]);
    if (state) {
      state[b * 4 + 0] = Z;
      state[b * 4 + 1] = alpha;
      state[b * 4 + 2] = s_zahn[2];
      state[b * 4 + 3] = n;
    }
  }
}

// d lp_b / d l_b * dlp_b (see the header comment for the algebra):
//   (1/(pi n)) [ A G + sum_t (beta_t/s_t) e_t - (A h + sum_t beta_t c_t/s_t) u ]
//   A = sum_t (m_t/P_t) dP_t/dZ,  beta_t = (m_t/P_t)(1-alpha)/Z
__global__ __launch_bounds__(256) void word_backward_kernel(
    const float* __restrict__ lat, int64_t B, int D, int Dp, const float* __restrict__ state,
    const float* __restrict__ gsum, const float* __restrict__ cosv, TokSrc tok, int L,
    const float* __restrict__ w, const float* __restrict__ mask, float a,
    const float* __restrict__ dlp, float* __restrict__ dlat) {
  __shared__ float s_v[4][512];  // per-wave sum_t (beta_t/s_t) e_t
  __shared__ float s_sc[4][2];   // per-wave A, sum beta c / s
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const int64_t b = blockIdx.x;
  const float Z = state[b * 4 + 0], alpha = state[b * 4 + 1], h = state[b * 4 + 2];
  const float nc = fmaxf(state[b * 4 + 3], kCosEps);
  const float dadz = -a * alpha * alpha;
  for (int k = lane; k < D; k += kWave) s_v[wave][k] = 0.f;
  float A = 0.f, sbc = 0.f;
  for (int t = wave; t < L; t += 4) {
    const float c = cosv[b * L + t];
    const float score = 1.f - acosf(c) / kPi;
    const float wt = w[b * L + t];
    const float P = alpha * wt + (1.f - alpha) * score / Z;
    const float mp = mask[b * L + t] * (1.f / P);
    const float dPdZ = wt * dadz - score * (dadz / Z + (1.f - alpha) / (Z * Z));
    A += mp * dPdZ;
    const float beta = mp * (1.f - alpha) / Z;
    const float st = sqrtf(1.f - c * c);
    sbc += beta * c / st;
    const float coef = beta / st;
    const float* e = tok_row(tok, b, L, t, D);
    float ee = 0.f;
    for (int k = lane; k < D; k += kWave) ee = fmaf(e[k], e[k], ee);
    const float en = fmaxf(sqrtf(wave_sum(ee)), kCosEps);
    if (coef != 0.f)  // NaN / inf pass (as torch's 0-mask x inf)
      for (int k = lane; k < D; k += kWave) s_v[wave][k] += coef * (e[k] / en);
  }
  if (lane == 0) {
    s_sc[wave][0] = A;
    s_sc[wave][1] = sbc;
  }
  __syncthreads();
  const float At = s_sc[0][0] + s_sc[1][0] + s_sc[2][0] + s_sc[3][0];
  const float St = s_sc[0][1] + s_sc[1][1] + s_sc[2][1] + s_sc[3][1];
  const float scale = dlp[b] / (kPi * nc);
  const float cu = At * h + St;
  for (int k = tid; k < D; k += blockDim.x) {
    const float u = lat[b * D + k] / nc;
    const float v = s_v[0][k] + s_v[1][k] + s_v[2][k] + s_v[3][k];
    dlat[b * D + k] = scale * (At * gsum[b * Dp + k] + v - cu * u);
  }
}

// ------------------------------------------------------------------ Gaussians
// stats[n][3][F] (f64): M0 | M1 | M2 of the masked frames of utterance n.
__global__ void gauss_stats_kernel(const float* __restrict__ x, const float* __restrict__ m,
                                   int64_t N, int T, int F, double* __restrict__ stats) {
  const int64_t total = N * F;
  for (int64_t e = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t n = e / F;
    const int f = static_cast<int>(e % F);
    double m0 = 0.0, m1 = 0.0, m2 = 0.0;
    for (int t = 0; t < T; ++t) {
      const int64_t o = (n * T + t) * F + f;
      const double v = x[o];
      const double mm = m ? static_cast<double>(m[o]) : 1.0;
      m0 += mm;
      m1 += mm * v;
      m2 += mm * v * v;
    }
    double* s = stats + n * 3 * F;
    s[f] = m0;
    s[F + f] = m1;
    s[2 * F + f] = m2;
  }
}

constexpr int kMaxKeys = 8;
struct GaussArgs {
  const double* stats[3];  // text, audio, visual: [N][3][F_m]
  int Fm[3];
  const int64_t* idx;      // [B] rows into stats (nullable: b)
  int64_t B;
  int nkeys;
  int mods[kMaxKeys];      // bit 0 text, 1 audio, 2 visual (cat order text, audio, visual)
  const float* mu[kMaxKeys];     // [B][F_k], rows ldm[k] apart
  const float* sigma[kMaxKeys];  // [B][F_k], rows lds[k] apart
  const float* dlp;              // [nkeys][B] (backward)
  float* dmu[kMaxKeys];          // rows ldm[k] apart
  float* dsigma[kMaxKeys];       // rows lds[k] apart
  int64_t ldm[kMaxKeys];
  int64_t lds[kMaxKeys];
};

__device__ __forceinline__ int key_width(const GaussArgs& g, int k) {
  int w = 0;
  for (int m = 0; m < 3; ++m)
    if (g.mods[k] >> m & 1) w += g.Fm[m];
  return w;
}

__device__ __forceinline__ void key_feature(const GaussArgs& g, int k, int f, int& mod, int& ff) {
  mod = 0;
  ff = f;
  for (int m = 0; m < 3; ++m) {
    if (!(g.mods[k] >> m & 1)) continue;
    if (ff < g.Fm[m]) {
      mod = m;
      return;
    }
    ff -= g.Fm[m];
  }
}

// lp[k][b] = sum_f M0 (-log s - log(2 pi)/2) - (M2 - 2 mu M1 + mu^2 M0)/(2 s^2)
// (losses.py:25-33); one block per (b, key), f64 accumulation, fixed order.
__global__ __launch_bounds__(256) void gauss_loglik_kernel(GaussArgs g, float* __restrict__ lp) {
  __shared__ double s_red[4];
  const int64_t b = blockIdx.x;
  const int k = blockIdx.y;
  const int Fk = key_width(g, k);
  const int64_t row = g.idx ? g.idx[b] : b;
  const double hl2pi = 0.5 * log(2.0 * 3.14159265358979323846);
  double acc = 0.0;
  for (int f = threadIdx.x; f < Fk; f += blockDim.x) {
    int mod, ff;
    key_feature(g, k, f, mod, ff);
    const double* st = g.stats[mod] + row * 3 * g.Fm[mod];
    const double m0 = st[ff], m1 = st[g.Fm[mod] + ff], m2 = st[2 * g.Fm[mod] + ff];
    const double mu = g.mu[k][b * g.ldm[k] + f], s = g.sigma[k][b * g.lds[k] + f];
    const double q = m2 - 2.0 * mu * m1 + mu * mu * m0;
    acc += m0 * (-log(s) - hl2pi) - q / (2.0 * s * s);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & (kWave - 1)) == 0) s_red[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) lp[static_cast<int64_t>(k) * g.B + b] = static_cast<float>(s_red[0] + s_red[1] + s_red[2] + s_red[3]);
}

// dmu = dlp (M1 - mu M0)/s^2,  dsigma = dlp (-M0/s + Q/s^3)
__global__ __launch_bounds__(256) void gauss_backward_kernel(GaussArgs g) {
  const int64_t b = blockIdx.x;
  const int k = blockIdx.y;
  const int Fk = key_width(g, k);
  const int64_t row = g.idx ? g.idx[b] : b;
  const double d = g.dlp[static_cast<int64_t>(k) * g.B + b];
  for (int f = threadIdx.x; f < Fk; f += blockDim.x) {
    int mod, ff;
    key_feature(g, k, f, mod, ff);
    const double* st = g.stats[mod] + row * 3 * g.Fm[mod];
    const double m0 = st[ff], m1 = st[g.Fm[mod] + ff], m2 = st[2 * g.Fm[mod] + ff];
    const double mu = g.mu[k][b * g.ldm[k] + f], s = g.sigma[k][b * g.lds[k] + f];
    const double q = m2 - 2.0 * mu * m1 + mu * mu * m0;
    if (g.dmu[k]) g.dmu[k][b * g.ldm[k] + f] = static_cast<float>(d * (m1 - mu * m0) / (s * s));
    if (g.dsigma[k]) g.dsigma[k][b * g.lds[k] + f] = static_cast<float>(d * (-m0 / s + q / (s * s * s)));
  }
}

}  // namespace mmb

using namespace mmb;

extern "C" int mmb_word_pad(int d) { return pad16(d); }

extern "C" int mmb_word_normalize(const float* table, int64_t v, int d, float* wn, hipStream_t stream) {
  MMB_REQUIRE(table && wn && v > 0 && d > 0);
  const int grid = static_cast<int>(std::min<int64_t>(ceil_div(v, 4), 256 * 8));
  word_normalize_kernel<<<grid, 256, 0, stream>>>(table, v, d, pad16(d), wn);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

static int word_splits(int64_t b, int64_t v) {
  const int64_t tiles = ceil_div(b, 16);
  const int64_t wt = ceil_div(v, 16);
  int64_t s = (2048 + tiles - 1) / tiles / 4;  // ~2048 waves over the grid
  s = std::min<int64_t>(s, ceil_div(wt, 4));
  return static_cast<int>(std::max<int64_t>(1, s));
}

extern "C" size_t mmb_word_workspace_bytes(int64_t b, int d, int64_t v) {
  const int64_t tiles = ceil_div(b, 16);
  return static_cast<size_t>(tiles) * 4 * word_splits(b, v) * 16 * (pad16(d) + 2) * sizeof(float);
}

extern "C" int mmb_word_logprob_forward(const float* latents, int64_t b, int d, const float* wn,
                                        int64_t v, const int32_t* ids, const float* table,
                                        const float* sent_dense, int l, const float* w,
                                        const float* mask, float a, int want_grad, void* ws,
                                        float* lp, float* state, float* gsum, float* cos_out,
                                        hipStream_t stream) {
  MMB_REQUIRE(latents && wn && w && mask && lp && ws && b >= 0 && d > 0 && d <= 512 && v > 0 && l >= 0);
  MMB_REQUIRE(ids ? (table != nullptr) : (sent_dense != nullptr || l == 0));
  MMB_REQUIRE(!want_grad || (state && gsum && cos_out));
  if (b == 0) return MMB_OK;
  const int Dp = pad16(d);
  const int S = word_splits(b, v);
  float* part = static_cast<float*>(ws);
  const dim3 grid(static_cast<unsigned>(ceil_div(b, 16)), static_cast<unsigned>(S));
  switch (Dp / 16) {
#define MMB_ZCASE(nt) \
  case nt: word_zsum_kernel<nt><<<grid, 256, 0, stream>>>(latents, b, d, wn, v, want_grad, part); break;
    MMB_ZCASE(1) MMB_ZCASE(2) MMB_ZCASE(3) MMB_ZCASE(4) MMB_ZCASE(5) MMB_ZCASE(6) MMB_ZCASE(7)
    MMB_ZCASE(8) MMB_ZCASE(9) MMB_ZCASE(10) MMB_ZCASE(11) MMB_ZCASE(12) MMB_ZCASE(13)
    MMB_ZCASE(14) MMB_ZCASE(15) MMB_ZCASE(16) MMB_ZCASE(17) MMB_ZCASE(18) MMB_ZCASE(19)
    MMB_ZCASE(20)
#undef MMB_ZCASE
    default: return MMB_EINVAL;  // d > 320
  }
  MMB_LAUNCH_CHECK();
  TokSrc tok{ids, table, sent_dense, v};
  word_finish_kernel<<<static_cast<unsigned>(b), 256, 0, stream>>>(
      latents, b, d, Dp, part, S, tok, l, w, mask, a, lp, state, gsum, cos_out);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_word_logprob_backward(const float* latents, int64_t b, int d, int64_t v,
                                         const int32_t* ids, const float* table,
                                         const float* sent_dense, int l, const float* w,
                                         const float* mask, float a, const float* state,
                                         const float* gsum, const float* cosv, const float* dlp,
                                         float* dlat, hipStream_t stream) {
  MMB_REQUIRE(latents && w && mask && state && gsum && cosv && dlp && dlat && d > 0 && d <= 512);
  MMB_REQUIRE(ids ? (table != nullptr) : (sent_dense != nullptr || l == 0));
  if (b == 0) return MMB_OK;
  TokSrc tok{ids, table, sent_dense, v};
  word_backward_kernel<<<static_cast<unsigned>(b), 256, 0, stream>>>(
      latents, b, d, pad16(d), state, gsum, cosv, tok, l, w, mask, a, dlp, dlat);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_gauss_stats(const float* x, const float* mask, int64_t n, int t, int f,
                               double* stats, hipStream_t stream) {
  MMB_REQUIRE(x && stats && n >= 0 && t >= 0 && f > 0);
  if (n == 0) return MMB_OK;
  const int grid = static_cast<int>(std::min<int64_t>(ceil_div(n * f, 256), 256 * 16));
  gauss_stats_kernel<<<grid, 256, 0, stream>>>(x, mask, n, t, f, stats);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

static int gauss_args(GaussArgs& g, const double* const* stats, const int* fm, const int64_t* idx,
                      int64_t b, int nkeys, const int* mods) {
  MMB_REQUIRE(stats && fm && mods && nkeys >= 1 && nkeys <= kMaxKeys && b >= 0);
  for (int m = 0; m < 3; ++m) {
    g.stats[m] = stats[m];
    g.Fm[m] = fm[m];
  }
  g.idx = idx;
  g.B = b;
  g.nkeys = nkeys;
  for (int k = 0; k < nkeys; ++k) {
    MMB_REQUIRE(mods[k] > 0 && mods[k] < 8);
    for (int m = 0; m < 3; ++m)
      if (mods[k] >> m & 1) MMB_REQUIRE(stats[m] && fm[m] > 0);
    g.mods[k] = mods[k];
  }
  return MMB_OK;
}

// row strides per key: given (the strided entry points), or the key widths
static int gauss_strides(GaussArgs& g, const int64_t* ld_mu, const int64_t* ld_sigma) {
  for (int k = 0; k < g.nkeys; ++k) {
    int w = 0;
    for (int m = 0; m < 3; ++m)
      if (g.mods[k] >> m & 1) w += g.Fm[m];
    g.ldm[k] = ld_mu ? ld_mu[k] : w;
    g.lds[k] = ld_sigma ? ld_sigma[k] : w;
    MMB_REQUIRE(g.ldm[k] >= w && g.lds[k] >= w);
  }
  return MMB_OK;
}

extern "C" int mmb_gauss_loglik_strided(const double* const* stats, const int* fm,
                                        const int64_t* idx, int64_t b, int nkeys, const int* mods,
                                        const float* const* mu, const int64_t* ld_mu,
                                        const float* const* sigma, const int64_t* ld_sigma,
                                        float* lp, hipStream_t stream) {
  GaussArgs g{};
  int rc = gauss_args(g, stats, fm, idx, b, nkeys, mods);
  if (rc != MMB_OK) return rc;
  if ((rc = gauss_strides(g, ld_mu, ld_sigma)) != MMB_OK) return rc;
  MMB_REQUIRE(mu && sigma && lp);
  for (int k = 0; k < nkeys; ++k) {
    MMB_REQUIRE(mu[k] && sigma[k]);
    g.mu[k] = mu[k];
    g.sigma[k] = sigma[k];
  }
  if (b == 0) return MMB_OK;
  gauss_loglik_kernel<<<dim3(static_cast<unsigned>(b), nkeys), 256, 0, stream>>>(g, lp);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_gauss_loglik(const double* const* stats, const int* fm, const int64_t* idx,
                                int64_t b, int nkeys, const int* mods, const float* const* mu,
                                const float* const* sigma, float* lp, hipStream_t stream) {
  return mmb_gauss_loglik_strided(stats, fm, idx, b, nkeys, mods, mu, nullptr, sigma, nullptr, lp,
                                  stream);
}

extern "C" int mmb_gauss_backward_strided(const double* const* stats, const int* fm,
                                          const int64_t* idx, int64_t b, int nkeys,
                                          const int* mods, const float* const* mu,
                                          const int64_t* ld_mu, const float* const* sigma,
                                          const int64_t* ld_sigma, const float* dlp,
                                          float* const* dmu, float* const* dsigma,
                                          hipStream_t stream) {
  GaussArgs g{};
  int rc = gauss_args(g, stats, fm, idx, b, nkeys, mods);
  if (rc != MMB_OK) return rc;
  if ((rc = gauss_strides(g, ld_mu, ld_sigma)) != MMB_OK) return rc;
  MMB_REQUIRE(mu && sigma && dlp && dmu && dsigma);
  for (int k = 0; k < nkeys; ++k) {
    MMB_REQUIRE(mu[k] && sigma[k]);
    g.mu[k] = mu[k];
    g.sigma[k] = sigma[k];
    g.dmu[k] = dmu[k];
    g.dsigma[k] = dsigma[k];
  }
  g.dlp = dlp;
  if (b == 0) return MMB_OK;
  gauss_backward_kernel<<<dim3(static_cast<unsigned>(b), nkeys), 256, 0, stream>>>(g);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_gauss_backward(const double* const* stats, const int* fm, const int64_t* idx,
                                  int64_t b, int nkeys, const int* mods, const float* const* mu,
                                  const float* const* sigma, const float* dlp, float* const* dmu,
                                  float* const* dsigma, hipStream_t stream) {
  return mmb_gauss_backward_strided(stats, fm, idx, b, nkeys, mods, mu, nullptr, sigma, nullptr,
                                    dlp, dmu, dsigma, stream);
}

// ------------------------------------------------------------ LayerNorm backward
// The generator's optional LayerNorm (reference models.py:163-164:
// nn.LayerNorm(embedding_dim) ahead of the mu / log-sigma heads) trains with the
// latents (e2e).  torch's backward is two launches, one of them a column
// reduction that runs ~21 us for a 64 x 300 batch; here ONE launch: blocks
// [0, rb) take 4 rows each (one wave per row: dx), blocks [rb, rb + cb) take
// 64 columns each (4 row groups, fixed-order LDS combine: dgamma, dbeta —
// deterministic).  xhat = (x - mean) rstd from the forward's saved statistics;
//   dx = rstd (g - (sum g + xhat sum g xhat) / D),  g = dy gamma.
__global__ __launch_bounds__(256) void ln_backward_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ gamma, float* __restrict__ dx,
    float* __restrict__ dgamma, float* __restrict__ dbeta, int64_t n, int d, int rb) {
  const int tid = threadIdx.x;
  if (static_cast<int>(blockIdx.x) < rb) {
    const int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (tid >> 6);
    if (r >= n) return;
    const int lane = tid & 63;
    const float mu = mean[r], rs = rstd[r];
    const float* dyr = dy + r * d;
    const float* xr = x + r * d;
    float a = 0.f, b = 0.f;
    for (int c = lane; c < d; c += 64) {
      const float g = dyr[c] * gamma[c];
      a += g;
      b += g * ((xr[c] - mu) * rs);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_xor(a, o);
      b += __shfl_xor(b, o);
    }
    const float inv_d = 1.f / static_cast<float>(d);
    float* dxr = dx + r * d;
    for (int c = lane; c < d; c += 64) {
      const float xh = (xr[c] - mu) * rs;
      dxr[c] = rs * (dyr[c] * gamma[c] - (a + xh * b) * inv_d);
    }
    return;
  }
  __shared__ float part[2][4][64];
  const int cl = tid & 63, rg = tid >> 6;
  const int c = (static_cast<int>(blockIdx.x) - rb) * 64 + cl;
  float sg = 0.f, sb = 0.f;
  if (c < d) {
#pragma unroll 4
    for (int64_t r = rg; r < n; r += 4) {
      const float g = dy[r * d + c];
      sg += g * ((x[r * d + c] - mean[r]) * rstd[r]);
      sb += g;
    }
  }
  part[0][rg][cl] = sg;
  part[1][rg][cl] = sb;
  __syncthreads();
  if (rg == 0 && c < d) {
    if (dgamma) dgamma[c] = (part[0][0][cl] + part[0][1][cl]) + (part[0][2][cl] + part[0][3][cl]);
    if (dbeta) dbeta[c] = (part[1][0][cl] + part[1][1][cl]) + (part[1][2][cl] + part[1][3][cl]);
  }
}

extern "C" int mmb_layer_norm_backward(const float* dy, const float* x, const float* mean,
                                       const float* rstd, const float* gamma, int64_t n, int d,
                                       float* dx, float* dgamma, float* dbeta,
                                       hipStream_t stream) {
  MMB_REQUIRE(gamma && n >= 0 && d > 0);
  if (n == 0) {  // (empty tensors may hand over null row pointers)
    for (float* p : {dgamma, dbeta}) {
      if (!p) continue;
      const hipError_t e = static_cast<hipError_t>(zero_words_async(p, static_cast<int64_t>(sizeof(float) * d) / 4, stream));
      if (e != hipSuccess) return static_cast<int>(e);
    }
    return MMB_OK;
  }
  MMB_REQUIRE(dy && x && mean && rstd && dx && n <= (int64_t{1} << 33));
  const int64_t rb = ceil_div(n, int64_t{4});
  const int cb = (dgamma || dbeta) ? static_cast<int>(ceil_div(int64_t{d}, int64_t{64})) : 0;
  MMB_REQUIRE(rb + cb < (int64_t{1} << 31));
  ln_backward_kernel<<<static_cast<unsigned>(rb + cb), 256, 0, stream>>>(
      dy, x, mean, rstd, gamma, dx, dgamma, dbeta, n, d, static_cast<int>(rb));
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}
