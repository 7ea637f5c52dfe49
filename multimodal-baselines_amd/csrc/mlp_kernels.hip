// Sentiment regressor (a10/a11): SentimentModel(d -> h -> o) forward, L1
// backward and SGD, for MI355X.
//
// The reference trains with one PyTorch step per 32-row mini-batch
// (sentiment_model.py:98-110): ~16 k tiny launches-worth of work per run.
// Here a whole run of mini-batches is ONE launch of ONE workgroup (16 waves):
// the parameters never leave the CU's L1/L2 and no host round trip sits
// between steps.  W1 is kept as fp32-MFMA accumulator tiles of W1^T
// (lane&31 = hidden unit, the 16 accumulator registers = 16 input features)
// in an L2-resident tiled copy.  That layout is at once
//   * the B operand of the forward  pre = X W1^T   (32x32x2, K = features, taken
//     in the accumulator's register order — any K order is a valid sum), and
//   * the C layout of the gradient  dW1^T = X^T dH (32x32x2, K = batch rows),
// so the SGD update W1 -= lr dW1 is a lane-local FMA on the fragment with no
// shuffles.  Each tile is owned by one wave for the whole run (its own
// stores are re-read only by itself).  Bias, output layer and loss are VALU on LDS.
#include <algorithm>
#include <cstdlib>

#include "mmb_common.h"

namespace mmb {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int kMlpNT = 1024;
constexpr int kMaxWaves = kMlpNT / kWave;
constexpr int kBatchMax = 32;  // one MFMA M-tile of batch rows

struct MlpArgs {
  const float* lat;
  const float* lab;
  const int64_t* perm;
  int64_t n_per_epoch;
  int n_epochs, B, D, H, O;
  float lr;
  float* w1;
  float* b1;
  float* w2;
  float* b2;
  float* step_loss;
  float* w1t;  // workspace: [nTh*nTd][64 lanes][16] tiled W1^T
  // tiling
  int nTh, nTd, G, DP, HP;
};

__device__ __forceinline__ int c_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

__device__ __forceinline__ f32x16 load_frag(const float* p) {
  f32x16 v;
  const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 x = q[i];
    v[4 * i] = x.x; v[4 * i + 1] = x.y; v[4 * i + 2] = x.z; v[4 * i + 3] = x.w;
  }
  return v;
}

__device__ __forceinline__ void store_frag(float* p, const f32x16& v) {
  float4* q = reinterpret_cast<float4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
}

// NT threads; REGT > 0: each wave's W1^T tiles (<= REGT) held in registers for
// the whole run (8 waves x 256 VGPRs), so neither the forward nor the SGD
// update touches L2 for W1; REGT = 0: tiles re-read from the L2-resident
// tiled copy every step (16 waves x 128 VGPRs, where the tiles spilled).
template <int NT, int REGT>
__global__ __launch_bounds__(NT) void mlp_train_kernel(MlpArgs a) {
  constexpr int kNW = NT / kWave;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int DP = a.DP, HP = a.HP, O = a.O;
  int64_t* s_perm = reinterpret_cast<int64_t*>(smem);  // [2][32] row indices (prefetch)
  float* sx = smem + 4 * kBatchMax;                   // [32][DP+1]
  float* spart = sx + kBatchMax * (DP + 1);           // [G][32][HP]  (aliased by sdh)
  float* shid = spart + a.G * kBatchMax * HP;         // [32][HP]
  float* sW2 = shid + kBatchMax * HP;                 // [O][HP]
  float* sb1 = sW2 + O * HP;                          // [HP]
  float* sb2 = sb1 + HP;                              // [O]
  float* sg = sb2 + O;                                // [32][O]
  float* sy = sg + kBatchMax * O;                     // [32][O]
  float* s_red = sy + kBatchMax * O;                  // [kNW]
  float* sdh = spart;                                 // [32][HP]
  const int SX = DP + 1;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool mw = wave < a.nTh * a.G;
  const int Th = mw ? wave % a.nTh : 0, grp = mw ? wave / a.nTh : 0;
  const int tpg = (a.nTd + a.G - 1) / a.G;
  const int td0 = grp * tpg;
  const int ntiles = mw ? max(0, min(tpg, a.nTd - td0)) : 0;
  const int hcol = 32 * Th + (lane & 31);
  float* wt = a.w1t + (static_cast<int64_t>(Th) * a.nTd * kWave + lane) * 16;  // + td*64*16

  // W1 -> tiled W1^T workspace (zero outside [H) x [D))
  for (int64_t e = tid; e < static_cast<int64_t>(a.nTh) * a.nTd * kWave * 16; e += NT) {
    const int r = static_cast<int>(e & 15), l = static_cast<int>((e >> 4) & 63);
    const int64_t tile = e >> 10;
    const int th = static_cast<int>(tile / a.nTd), td = static_cast<int>(tile % a.nTd);
    const int h = 32 * th + (l & 31), d = 32 * td + c_row(r, l);
    a.w1t[e] = (h < a.H && d < a.D) ? a.w1[static_cast<int64_t>(h) * a.D + d] : 0.f;
  }
  for (int e = tid; e < O * HP; e += NT) {
    const int o = e / HP, h = e % HP;
    sW2[e] = h < a.H ? a.w2[o * a.H + h] : 0.f;
  }
  for (int h = tid; h < HP; h += NT) sb1[h] = h < a.H ? a.b1[h] : 0.f;
  for (int o = tid; o < O; o += NT) sb2[o] = a.b2[o];
  __threadfence_block();
  __syncthreads();
  f32x16 wreg[REGT > 0 ? REGT : 1];
  if constexpr (REGT > 0) {
#pragma unroll
    for (int t = 0; t < REGT; ++t)
      if (t < ntiles) wreg[t] = load_frag(wt + static_cast<int64_t>(td0 + t) * kWave * 16);
  }

  const int64_t spe = (a.n_per_epoch + a.B - 1) / a.B;
  const int64_t nsteps = spe * a.n_epochs;
  auto batch_of = [&](int64_t st, int64_t& base, int& bc) {
    const int64_t ep = st / spe, bi = st % spe;
    base = ep * a.n_per_epoch + bi * a.B;
    bc = static_cast<int>(min<int64_t>(a.B, a.n_per_epoch - bi * a.B));
  };
  // The batch gather was two dependent round trips (permutation index, then
  // the row) per step.  Now wave 0 reads step s+1's indices into LDS during
  // step s, so a step issues its row loads at once (16-byte loads when
  // D % 4 == 0).
  auto fetch_perm = [&](int64_t st) {
    if (wave == 0 && lane < kBatchMax && st < nsteps) {
      int64_t base;
      int bc;
      batch_of(st, base, bc);
      s_perm[(st & 1) * kBatchMax + lane] = lane < bc ? a.perm[base + lane] : 0;
    }
  };
  const bool v4 = (a.D & 3) == 0 && (reinterpret_cast<uintptr_t>(a.lat) & 15) == 0;
  fetch_perm(0);
  __syncthreads();
  for (int64_t step = 0; step < nsteps; ++step) {
    int64_t base;
    int Bc;
    batch_of(step, base, Bc);
    const int64_t* pp = s_perm + (step & 1) * kBatchMax;
    // 1. gather the batch rows (DataLoader order) into LDS
    if (v4) {
      const int U = DP >> 2;  // float4 units of a padded row
      for (int e = tid; e < kBatchMax * U; e += NT) {
        const int b = e / U, u = e - b * U;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (b < Bc && 4 * u < a.D) v = *reinterpret_cast<const float4*>(a.lat + pp[b] * a.D + 4 * u);
        float* dst = sx + b * SX + 4 * u;
        dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
      }
    } else {
      for (int e = tid; e < kBatchMax * DP; e += NT) {
        const int b = e / DP, d = e % DP;
        float v = 0.f;
        if (b < Bc && d < a.D) v = a.lat[pp[b] * a.D + d];
        sx[b * SX + d] = v;
      }
    }
    for (int e = tid; e < kBatchMax * O; e += NT) {
      const int b = e / O, o = e % O;
      sy[e] = (b < Bc) ? a.lab[pp[b] * O + o] : 0.f;
    }
    fetch_perm(step + 1);  // lands during this step
    __syncthreads();
    // 2. forward partials: pre[b][h] over this wave's feature tiles (MFMA)
    if (mw) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const float* xb = sx + (lane & 31) * SX + 4 * (lane >> 5);
      auto fwd_tile = [&](int t, const f32x16& w) {
        const int td = td0 + t;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float xa = xb[32 * td + (r & 3) + 8 * (r >> 2)];
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa, w[r], acc, 0, 0, 0);
        }
      };
      if constexpr (REGT > 0) {
#pragma unroll
        for (int t = 0; t < REGT; ++t)
          if (t < ntiles) fwd_tile(t, wreg[t]);
      } else {
        for (int t = 0; t < ntiles; ++t)
          fwd_tile(t, load_frag(wt + static_cast<int64_t>(td0 + t) * kWave * 16));
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) spart[(grp * kBatchMax + c_row(r, lane)) * HP + hcol] = acc[r];
    }
    __syncthreads();
    // 3. hidden = relu(sum_g partial + b1)  (fixed group order)
    for (int e = tid; e < kBatchMax * HP; e += NT) {
      const int b = e / HP, h = e % HP;
      float p = sb1[h];
      for (int g = 0; g < a.G; ++g) p += spart[(g * kBatchMax + b) * HP + h];
      shid[e] = (h < a.H && p > 0.f) ? p : 0.f;
    }
    __syncthreads();
    // 4. output layer, L1 loss and its gradient (mean over Bc*O elements);
    //    O = 1: a half-wave per batch row (16 waves x 2 = 32 rows), lane
    //    h-stride partial dots and a 32-lane shuffle sum, instead of a
    //    100-long serial chain per row
    float lsum = 0.f;
    if (O == 1) {
#pragma unroll
      for (int k = 0; k < kBatchMax / (2 * kNW); ++k) {
        const int b = 2 * (wave + kNW * k) + (lane >> 5), l32 = lane & 31;
        float part = 0.f;
        for (int h = l32; h < a.H; h += 32) part = fmaf(sW2[h], shid[b * HP + h], part);
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) part += __shfl_xor(part, o, kWave);
        const float diff = (sb2[0] + part) - sy[b];
        const bool valid = b < Bc;
        if (l32 == 0) {
          sg[b] = valid ? ((diff > 0.f) ? 1.f : (diff < 0.f ? -1.f : 0.f)) / static_cast<float>(Bc) : 0.f;
          if (valid) lsum += fabsf(diff);
        }
      }
    } else {
      for (int e = tid; e < kBatchMax * O; e += NT) {
        const int b = e / O, o = e % O;
        float out = sb2[o];
        for (int h = 0; h < a.H; ++h) out = fmaf(sW2[o * HP + h], shid[b * HP + h], out);
        const float diff = out - sy[e];
        const bool valid = b < Bc;
        sg[e] = valid ? ((diff > 0.f) ? 1.f : (diff < 0.f ? -1.f : 0.f)) / static_cast<float>(Bc * O) : 0.f;
        if (valid) lsum += fabsf(diff);
      }
    }
    lsum = wave_sum(lsum);
    if (lane == 0) s_red[wave] = lsum;
    __syncthreads();
    // 5. dH = relu'(.) * g W2 ; then W2/b2 gradients (old W2 already consumed)
    for (int e = tid; e < kBatchMax * HP; e += NT) {
      const int b = e / HP, h = e % HP;
      float s = 0.f;
      if (shid[e] > 0.f)
        for (int o = 0; o < O; ++o) s = fmaf(sg[b * O + o], sW2[o * HP + h], s);
      sdh[e] = s;
    }
    __syncthreads();
    // 6. dW1^T = X^T dH (MFMA, K = batch) and the SGD step on the owned tiles;
    //    VALU updates of b1/W2/b2
    if (mw) {
      auto grad_tile = [&](int t) {
        const int td = td0 + t;
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
        for (int s = 0; s < kBatchMax / 2; ++s) {
          const int b = 2 * s + (lane >> 5);
          const float xa = sx[b * SX + 32 * td + (lane & 31)];
          const float db = sdh[b * HP + hcol];
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa, db, acc, 0, 0, 0);
        }
        return acc;
      };
      if constexpr (REGT > 0) {
#pragma unroll
        for (int t = 0; t < REGT; ++t) {
          if (t < ntiles) {
            const f32x16 g = grad_tile(t);
#pragma unroll
            for (int r = 0; r < 16; ++r) wreg[t][r] = fmaf(-a.lr, g[r], wreg[t][r]);
          }
        }
      } else {
        for (int t = 0; t < ntiles; ++t) {
          const f32x16 g = grad_tile(t);
          float* p = wt + static_cast<int64_t>(td0 + t) * kWave * 16;
          f32x16 w = load_frag(p);
#pragma unroll
          for (int r = 0; r < 16; ++r) w[r] = fmaf(-a.lr, g[r], w[r]);
          store_frag(p, w);
        }
      }
    }
    for (int e = tid; e < O * HP; e += NT) {
      const int o = e / HP, h = e % HP;
      if (h < a.H) {
        float gsum = 0.f;
        for (int b = 0; b < kBatchMax; ++b) gsum = fmaf(sg[b * O + o], shid[b * HP + h], gsum);
        sW2[e] = fmaf(-a.lr, gsum, sW2[e]);
      }
    }
    for (int h = tid; h < a.H; h += NT) {
      float gsum = 0.f;
      for (int b = 0; b < kBatchMax; ++b) gsum += sdh[b * HP + h];
      sb1[h] = fmaf(-a.lr, gsum, sb1[h]);
    }
    for (int o = tid; o < O; o += NT) {
      float gsum = 0.f;
      for (int b = 0; b < kBatchMax; ++b) gsum += sg[b * O + o];
      sb2[o] = fmaf(-a.lr, gsum, sb2[o]);
    }
    if (tid == 0) {
      float l = 0.f;
      for (int w = 0; w < kNW; ++w) l += s_red[w];
      a.step_loss[step] = l / static_cast<float>(Bc * O);
    }
    __syncthreads();
  }

  // write the parameters back
  if constexpr (REGT > 0) {
#pragma unroll
    for (int t = 0; t < REGT; ++t)
      if (t < ntiles) store_frag(wt + static_cast<int64_t>(td0 + t) * kWave * 16, wreg[t]);
  }
  __threadfence_block();
  __syncthreads();
  for (int64_t e = tid; e < static_cast<int64_t>(a.H) * a.D; e += NT) {
    const int h = static_cast<int>(e / a.D), d = static_cast<int>(e % a.D);
    const int th = h >> 5, td = d >> 5, dr = d & 31;
    // invert c_row: dr = (r&3) + 8*(r>>2) + 4*(lane>>5)
    const int hl = (dr >> 2) & 1, r = (dr & 3) + 4 * (dr >> 3);
    const int l = (h & 31) + 32 * hl;
    a.w1[e] = a.w1t[((static_cast<int64_t>(th) * a.nTd + td) * kWave + l) * 16 + r];
  }
  for (int e = tid; e < O * a.H; e += NT) a.w2[e] = sW2[(e / a.H) * HP + e % a.H];
  for (int h = tid; h < a.H; h += NT) a.b1[h] = sb1[h];
  for (int o = tid; o < O; o += NT) a.b2[o] = sb2[o];
}

// Forward (+ optional L1 per batch) — one workgroup per batch of rows.
__global__ __launch_bounds__(256) void mlp_eval_kernel(const float* __restrict__ lat,
                                                       const float* __restrict__ lab,
                                                       const int64_t* __restrict__ perm, int64_t n,
                                                       int B, int D, int H, int O,
                                                       const float* __restrict__ w1,
                                                       const float* __restrict__ b1,
                                                       const float* __restrict__ w2,
                                                       const float* __restrict__ b2,
                                                       float* __restrict__ batch_loss,
                                                       float* __restrict__ pred) {
  extern __shared__ float sm[];
  float* sx = sm;          // [D]
  float* shid = sx + D;    // [H]
  __shared__ float s_red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * B;
  const int Bc = static_cast<int>(min<int64_t>(B, n - b0));
  float lsum = 0.f;
  for (int bb = 0; bb < Bc; ++bb) {
    const int64_t row = perm ? perm[b0 + bb] : (b0 + bb);
    for (int d = tid; d < D; d += 256) sx[d] = lat[row * D + d];
    __syncthreads();
    for (int h = tid; h < H; h += 256) {
      float p = b1[h];
#pragma unroll 10
      for (int d = 0; d < D; ++d) p = fmaf(w1[static_cast<int64_t>(h) * D + d], sx[d], p);
      shid[h] = p > 0.f ? p : 0.f;
    }
    __syncthreads();
    for (int o = tid; o < O; o += 256) {
      float out = b2[o];
#pragma unroll 20
      for (int h = 0; h < H; ++h) out = fmaf(w2[o * H + h], shid[h], out);
      if (pred) pred[(b0 + bb) * O + o] = out;
      if (lab) lsum += fabsf(out - lab[row * O + o]);
    }
    __syncthreads();
  }
  lsum = wave_sum(lsum);
  if (lane == 0) s_red[wave] = lsum;
  __syncthreads();
  if (tid == 0 && batch_loss) batch_loss[blockIdx.x] = (s_red[0] + s_red[1] + s_red[2] + s_red[3]) / static_cast<float>(Bc * O);
}

// ---------------------------------------------------------------- autograd pieces
// The differentiable forward / backward the e2e joint objective needs
// (simplesif.py:776-790: the regressor's L1 term backpropagates into the
// latents and the regressor's parameters).  Rows are independent in the
// forward and in dX; the parameter gradients reduce over the batch in a
// fixed row order (deterministic).
constexpr int kMlpRows = 8;  // rows per block of the row kernels

// hid[b][h] = relu(b1[h] + x[b] . w1[h]),  y[b][o] = b2[o] + hid[b] . w2[o].
// Block = kMlpRows rows staged in LDS; thread = hidden unit h, walking its own
// w1 row (each 64-byte line reused over 16 k-steps from L1) with the block's
// rows' x broadcast from LDS: one w1 load serves kMlpRows FMAs.
// V4 (D % 4 == 0, 16-byte aligned w1): the block first copies W1 into LDS
// (rows kMlpWPad floats apart) with all of its 16-byte loads in flight at
// once, then every thread walks its own row from LDS as float4.  Reading the
// thread-private rows from L2 instead (one cache line per lane per load, ~75
// dependent round trips per thread) took 38 us for a 64-row batch.  Same FMAs
// in the same order either way.
// LDS row stride of the staged W1 (floats): >= D, a multiple of 4 (16-byte
// rows) and 20 mod 32, so the float4 reads of consecutive threads' rows start
// in 8 different 4-bank groups (D + 4 = 304 = 16 mod 32 put every other
// thread in the same banks)
__host__ __device__ constexpr int mlp_wld(int d) {
  const int r = (d + 3) / 4 * 4;
  return r + ((20 - r % 32) % 32 + 32) % 32;
}

template <bool V4>
__global__ __launch_bounds__(256) void mlp_fwd_rows_kernel(const float* __restrict__ x, int64_t B,
                                                           int D, int H, int O,
                                                           const float* __restrict__ w1,
                                                           const float* __restrict__ b1,
                                                           const float* __restrict__ w2,
                                                           const float* __restrict__ b2,
                                                           float* __restrict__ y,
                                                           float* __restrict__ hid) {
  extern __shared__ float sm[];
  float* sx = sm;                      // [kMlpRows][D]
  float* sh = sx + kMlpRows * D;       // [kMlpRows][H]
  float* sw = sh + kMlpRows * H;       // V4: [H][wld]
  const int wld = mlp_wld(D);
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kMlpRows;
  const int nr = static_cast<int>(min<int64_t>(kMlpRows, B - r0));
  {  // the block's x rows: every thread's loads issued before its LDS stores
    constexpr int kBatch = 12;
    for (int e0 = threadIdx.x; e0 < kMlpRows * D; e0 += kBatch * blockDim.x) {
      // (unconditional loads of clamped addresses: a load under a per-lane
      // condition was waited for inside its branch, one round trip each)
      float v[kBatch];
#pragma unroll
      for (int q = 0; q < kBatch; ++q) {
        const int e = min(e0 + q * static_cast<int>(blockDim.x), kMlpRows * D - 1);
        const int r = min(e / D, nr - 1);
        v[q] = x[(r0 + r) * D + e % D];
      }
#pragma unroll
      for (int q = 0; q < kBatch; ++q) {
        const int e = e0 + q * static_cast<int>(blockDim.x);
        if (e < kMlpRows * D) sx[e] = e / D < nr ? v[q] : 0.f;
      }
    }
  }
  if constexpr (V4) {
    const int U = D / 4, n4 = H * U;
    constexpr int kBatch = 16;  // 16-byte loads per thread in flight
    for (int e0 = threadIdx.x; e0 < n4; e0 += kBatch * blockDim.x) {
      float4 v[kBatch];
#pragma unroll
      for (int q = 0; q < kBatch; ++q) {
        const int e = min(e0 + q * static_cast<int>(blockDim.x), n4 - 1);
        v[q] = reinterpret_cast<const float4*>(w1)[e];
      }
#pragma unroll
      for (int q = 0; q < kBatch; ++q) {
        const int e = e0 + q * static_cast<int>(blockDim.x);
        if (e < n4)
          *reinterpret_cast<float4*>(sw + (e / U) * wld + 4 * (e % U)) = v[q];
      }
    }
  }
  __syncthreads();
  if constexpr (V4) {
    // two thread groups of 128, each a half of the block's rows (4 each):
    // half the FMA chain per thread of one group per row block
    constexpr int RH = kMlpRows / 2;
    const int half = threadIdx.x >> 7;
    for (int h = threadIdx.x & 127; h < H; h += 128) {
      const float* wr = sw + h * wld;
      const float* xs = sx + half * RH * D;
      float p[RH];
#pragma unroll
      for (int r = 0; r < RH; ++r) p[r] = b1[h];
#pragma unroll 5
      for (int d = 0; d < D; d += 4) {
        const float4 w4 = *reinterpret_cast<const float4*>(wr + d);
        float4 x4[RH];  // the rows' 4 values as one broadcast 16-byte read each
#pragma unroll
        for (int r = 0; r < RH; ++r) x4[r] = *reinterpret_cast<const float4*>(xs + r * D + d);
#pragma unroll
        for (int r = 0; r < RH; ++r) p[r] = fmaf(w4.x, x4[r].x, p[r]);
#pragma unroll
        for (int r = 0; r < RH; ++r) p[r] = fmaf(w4.y, x4[r].y, p[r]);
#pragma unroll
        for (int r = 0; r < RH; ++r) p[r] = fmaf(w4.z, x4[r].z, p[r]);
#pragma unroll
        for (int r = 0; r < RH; ++r) p[r] = fmaf(w4.w, x4[r].w, p[r]);
      }
#pragma unroll
      for (int r = 0; r < RH; ++r) {
        const int row = half * RH + r;
        const float v = p[r] > 0.f ? p[r] : 0.f;
        sh[row * H + h] = v;
        if (row < nr) hid[(r0 + row) * H + h] = v;
      }
    }
  } else {
    for (int h = threadIdx.x; h < H; h += blockDim.x) {
      const float* wr = w1 + static_cast<int64_t>(h) * D;
      float p[kMlpRows];
#pragma unroll
      for (int r = 0; r < kMlpRows; ++r) p[r] = b1[h];
#pragma unroll 4
      for (int d = 0; d < D; ++d) {
        const float w = wr[d];
#pragma unroll
        for (int r = 0; r < kMlpRows; ++r) p[r] = fmaf(w, sx[r * D + d], p[r]);
      }
#pragma unroll
      for (int r = 0; r < kMlpRows; ++r) {
        const float v = p[r] > 0.f ? p[r] : 0.f;
        sh[r * H + h] = v;
        if (r < nr) hid[(r0 + r) * H + h] = v;
      }
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < nr * O; e += blockDim.x) {
    const int o = e % O, r = e / O;
    float out = b2[o];
    // (unrolled: the w2 loads are issued ahead of the in-order FMA chain)
#pragma unroll 20
    for (int h = 0; h < H; ++h) out = fmaf(w2[o * H + h], sh[r * H + h], out);
    y[(r0 + r) * O + o] = out;
  }
}

// dh[b][h] = [hid > 0] * sum_o dy[b][o] w2[o][h];  dx[b][d] = sum_h dh[b][h] w1[h][d]
// (thread = column d: w1[h][d] coalesced over the block, dh broadcast from LDS)
// R rows per block (2: 32 blocks for a 64-row batch instead of 8 -- the d
// loop's w1 loads are latency-bound; more blocks keep more of them in flight)
template <int R>
__global__ __launch_bounds__(256) void mlp_bwd_rows_kernel(const float* __restrict__ hid, int64_t B,
                                                           int D, int H, int O,
                                                           const float* __restrict__ w1,
                                                           const float* __restrict__ w2,
                                                           const float* __restrict__ dy,
                                                           float* __restrict__ dh,
                                                           float* __restrict__ dx) {
  extern __shared__ float sm[];
  float* sdh = sm;  // [R][H]
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * R;
  const int nr = static_cast<int>(min<int64_t>(R, B - r0));
  for (int e = threadIdx.x; e < R * H; e += blockDim.x) {
    const int h = e % H, r = e / H;
    float g = 0.f;
    if (r < nr && hid[(r0 + r) * H + h] > 0.f)
      for (int o = 0; o < O; ++o) g = fmaf(dy[(r0 + r) * O + o], w2[o * H + h], g);
    sdh[e] = g;
    if (r < nr) dh[(r0 + r) * H + h] = g;
  }
  __syncthreads();
  if (dx == nullptr) return;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float g[R];
#pragma unroll
    for (int r = 0; r < R; ++r) g[r] = 0.f;
#pragma unroll 10
    for (int h = 0; h < H; ++h) {
      const float w = w1[static_cast<int64_t>(h) * D + d];
#pragma unroll
      for (int r = 0; r < R; ++r) g[r] = fmaf(sdh[r * H + h], w, g[r]);
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (r < nr) dx[(r0 + r) * D + d] = g[r];
  }
}

// block h < H: dw1[h][:] = sum_b dh[b][h] x[b][:], db1[h] = sum_b dh[b][h],
// dw2[:, h] = sum_b dy[b][:] hid[b][h];  block H: db2 = sum_b dy[b][:]
__global__ __launch_bounds__(256) void mlp_bwd_params_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ hid,
                                                             const float* __restrict__ dh,
                                                             const float* __restrict__ dy,
                                                             int64_t B, int D, int H, int O,
                                                             float* __restrict__ dw1,
                                                             float* __restrict__ db1,
                                                             float* __restrict__ dw2,
                                                             float* __restrict__ db2) {
  const int h = blockIdx.x;
  if (h == H) {
    for (int o = threadIdx.x; o < O; o += blockDim.x) {
      float g = 0.f;
#pragma unroll 16
      for (int64_t b = 0; b < B; ++b) g += dy[b * O + o];
      if (db2) db2[o] = g;
    }
    return;
  }
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float g = 0.f;
#pragma unroll 16
    for (int64_t b = 0; b < B; ++b) g = fmaf(dh[b * H + h], x[b * D + d], g);
    if (dw1) dw1[static_cast<int64_t>(h) * D + d] = g;
  }
  if (threadIdx.x == 0 && db1) {
    float g = 0.f;
#pragma unroll 16
    for (int64_t b = 0; b < B; ++b) g += dh[b * H + h];
    db1[h] = g;
  }
  for (int o = threadIdx.x; o < O; o += blockDim.x) {
    float g = 0.f;
#pragma unroll 16
    for (int64_t b = 0; b < B; ++b) g = fmaf(dy[b * O + o], hid[b * H + h], g);
    if (dw2) dw2[o * H + h] = g;
  }
}

template <int NT, int REGT>
static int launch_train(const MlpArgs& a, size_t lds, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_train_kernel<NT, REGT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  mlp_train_kernel<NT, REGT><<<1, NT, lds, stream>>>(a);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

// W1 tiles in registers (8 waves, <= 5 tiles each) where they fit, else the
// L2-tile kernel (the tools build's MMB_MLP_REG=0 forces the latter)
constexpr int kRegWaves = 8, kRegTiles = 5;
static int mlp_reg() {
#ifdef MMB_DIAG
  const char* e = getenv("MMB_MLP_REG");
  return e ? atoi(e) : 1;
#else
  return 1;
#endif
}

}  // namespace mmb

using namespace mmb;

extern "C" int mmb_mlp_forward(const float* latents, const int64_t* idx, int64_t b, int d, int h,
                               int o, const float* w1, const float* b1, const float* w2,
                               const float* b2, float* y_out, hipStream_t stream) {
  MMB_REQUIRE(latents && w1 && b1 && w2 && b2 && y_out && b >= 0 && d > 0 && h > 0 && o > 0);
  if (b == 0) return MMB_OK;
  const int B = 32;
  mlp_eval_kernel<<<static_cast<int>(ceil_div(b, B)), 256, sizeof(float) * (d + h), stream>>>(
      latents, nullptr, idx, b, B, d, h, o, w1, b1, w2, b2, nullptr, y_out);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_mlp_eval(const float* latents, const float* labels, const int64_t* perm,
                            int64_t n, int batch, int d, int h, int o, const float* w1,
                            const float* b1, const float* w2, const float* b2, float* batch_loss,
                            float* pred_out, hipStream_t stream) {
  MMB_REQUIRE(latents && labels && w1 && b1 && w2 && b2 && n >= 0 && batch > 0 && d > 0 && h > 0 && o > 0);
  if (n == 0) return MMB_OK;
  mlp_eval_kernel<<<static_cast<int>(ceil_div(n, batch)), 256, sizeof(float) * (d + h), stream>>>(
      latents, labels, perm, n, batch, d, h, o, w1, b1, w2, b2, batch_loss, pred_out);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" size_t mmb_mlp_workspace_bytes(int d, int h) {
  return static_cast<size_t>(ceil_div(h, 32)) * ceil_div(d, 32) * kWave * 16 * sizeof(float);
}

extern "C" int mmb_mlp_train(const float* latents, const float* labels, const int64_t* perm,
                             int64_t n_per_epoch, int n_epochs, int batch, int d, int h, int o,
                             float lr, float* w1, float* b1, float* w2, float* b2,
                             float* step_loss, void* ws, hipStream_t stream) {
  MMB_REQUIRE(latents && labels && perm && w1 && b1 && w2 && b2 && step_loss && ws);
  MMB_REQUIRE(n_per_epoch > 0 && n_epochs >= 0 && batch >= 1 && batch <= kBatchMax);
  MMB_REQUIRE(d > 0 && h > 0 && o >= 1 && o <= 32);
  MMB_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 15) == 0);
  if (n_epochs == 0) return MMB_OK;
  MlpArgs a{};
  a.lat = latents; a.lab = labels; a.perm = perm; a.n_per_epoch = n_per_epoch;
  a.n_epochs = n_epochs; a.B = batch; a.D = d; a.H = h; a.O = o; a.lr = lr;
  a.w1 = w1; a.b1 = b1; a.w2 = w2; a.b2 = b2; a.step_loss = step_loss;
  a.w1t = static_cast<float*>(ws);
  a.nTh = static_cast<int>(ceil_div(h, 32));
  a.nTd = static_cast<int>(ceil_div(d, 32));
  MMB_REQUIRE(a.nTh <= kMaxWaves);
  bool reg = false;
  if (mlp_reg() && a.nTh <= kRegWaves) {
    const int g = std::min(kRegWaves / a.nTh, a.nTd);
    reg = ceil_div(a.nTd, g) <= kRegTiles;
  }
  a.G = (reg ? kRegWaves : kMaxWaves) / a.nTh;
  if (a.G > a.nTd) a.G = a.nTd;
  a.DP = a.nTd * 32;
  a.HP = a.nTh * 32;
  const size_t lds = sizeof(float) * (4 * kBatchMax + static_cast<size_t>(kBatchMax) * (a.DP + 1) +
                                      static_cast<size_t>(a.G) * kBatchMax * a.HP +
                                      static_cast<size_t>(kBatchMax) * a.HP + o * a.HP + a.HP +
                                      o + 2 * kBatchMax * o + kMaxWaves);
  MMB_REQUIRE(lds <= 160 * 1024);
  return reg ? launch_train<kRegWaves * kWave, kRegTiles>(a, lds, stream)
             : launch_train<kMlpNT, 0>(a, lds, stream);
}

extern "C" int mmb_mlp_forward_train(const float* x, int64_t b, int d, int h, int o,
                                     const float* w1, const float* b1, const float* w2,
                                     const float* b2, float* y_out, float* hid_out,
                                     hipStream_t stream) {
  MMB_REQUIRE(x && w1 && b1 && w2 && b2 && y_out && hid_out && b >= 0 && d > 0 && h > 0 && o > 0);
  if (b == 0) return MMB_OK;
  const size_t lds = sizeof(float) * kMlpRows * (d + h);
  MMB_REQUIRE(lds <= 64 * 1024);
  const int grid = static_cast<int>(ceil_div(b, kMlpRows));
  const size_t lds_w = lds + sizeof(float) * static_cast<size_t>(h) * mlp_wld(d);
  if (d % 4 == 0 && (reinterpret_cast<uintptr_t>(w1) & 15) == 0 && lds_w <= 160 * 1024) {
    static bool attr_set = false;  // > 64 KB of dynamic LDS (the regressor: 134 KB)
    if (!attr_set) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_fwd_rows_kernel<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr_set = true;
    }
    mlp_fwd_rows_kernel<true><<<grid, 256, lds_w, stream>>>(x, b, d, h, o, w1, b1, w2, b2, y_out,
                                                           hid_out);
  } else {
    mlp_fwd_rows_kernel<false><<<grid, 256, lds, stream>>>(x, b, d, h, o, w1, b1, w2, b2, y_out,
                                                          hid_out);
  }
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_mlp_backward(const float* x, const float* hid, int64_t b, int d, int h, int o,
                                const float* w1, const float* w2, const float* dy, float* dh_ws,
                                float* dx, float* dw1, float* db1, float* dw2, float* db2,
                                hipStream_t stream) {
  MMB_REQUIRE(x && hid && w1 && w2 && dy && dh_ws && b >= 0 && d > 0 && h > 0 && o > 0);
  if (b == 0) {  // an empty batch: zero gradients (the sums over no rows)
    const size_t nbytes[4] = {sizeof(float) * h * d, sizeof(float) * h, sizeof(float) * o * h,
                              sizeof(float) * o};
    float* outs[4] = {dw1, db1, dw2, db2};
    for (int q = 0; q < 4; ++q) {
      if (!outs[q]) continue;
      const hipError_t e = hipMemsetAsync(outs[q], 0, nbytes[q], stream);
      if (e != hipSuccess) return static_cast<int>(e);
    }
    return MMB_OK;
  }
  constexpr int kBwdRows = 2;
  const size_t lds = sizeof(float) * kBwdRows * h;
  MMB_REQUIRE(lds <= 64 * 1024);
  mlp_bwd_rows_kernel<kBwdRows><<<static_cast<int>(ceil_div(b, kBwdRows)), 256, lds, stream>>>(
      hid, b, d, h, o, w1, w2, dy, dh_ws, dx);
  MMB_LAUNCH_CHECK();
  if (dw1 || db1 || dw2 || db2) {
    mlp_bwd_params_kernel<<<h + 1, 256, 0, stream>>>(x, hid, dh_ws, dy, b, d, h, o, dw1, db1, dw2,
                                                     db2);
    MMB_LAUNCH_CHECK();
  }
  return MMB_OK;
}
