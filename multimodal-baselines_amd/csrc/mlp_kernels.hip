// Sentiment regressor (a10/a11): SentimentModel(d -> h -> o) forward, L1
// backward and SGD, for MI355X.
//
// The reference trains with one PyTorch step per 32-row mini-batch
// (sentiment_model.py:98-110): ~16 k tiny launches-worth of work per run, and
// a validation pass every 10 epochs (:114-127).  Here a whole run -- every
// SGD step AND the validation passes -- is ONE launch (mmb_mlp_train).
//
// r04: the run is split over P = ceil(h / 32) workgroups, one 32-wide tile of
// hidden units each (one XCD's worth of CUs at most: P <= 16).  A workgroup
// keeps its tile of W1^T in registers for the whole run as fp32-MFMA
// (32x32x2) accumulator tiles -- lane & 31 = hidden unit, the 16 registers =
// 16 input features of a 32-feature tile, tile t on wave t % 8 -- which is at
// once the B operand of the forward pre = X W1^T (K = features, taken in the
// registers' order: any K order is a valid sum) and the C layout of its
// gradient dW1^T = X^T dH (K = batch rows): the SGD update is a lane-local FMA.
// Per mini-batch (all workgroups in lockstep):
//   forward partial products per wave -> fixed-order sum + b1 -> ReLU (LDS);
//   this tile's share of the output, yp[b][o] = sum_{h in tile} W2[o][h] hid[b][h],
//   published with write-through stores, then ONE exchange: an arrival
//   counter (relaxed agent-scope atomics, release / acquire fences around it,
//   bounded poll), and every workgroup sums the P shares in tile order --
//   identical outputs, loss and gradient sign everywhere;
//   g = sign(y - label) / (rows * o); dH = relu' g W2 (own tile); dW1^T for
//   the own tiles (MFMA) and the SGD steps of W1 / b1 / W2 (own tile) and b2
//   (every workgroup, identical).
// The next mini-batch's rows are loaded into registers while this one is
// computed (their indices two batches ahead) and land in the other LDS
// buffer at the end of the step.  The single-workgroup kernel this replaces
// spent ~8.5 us of its 19.3 us step in the MFMAs of all hidden tiles on one
// CU.
#include <algorithm>
#include <cstdlib>

#include "mmb_common.h"

namespace mmb {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int kBatchMax = 32;  // one MFMA M-tile of batch rows

__device__ __forceinline__ int c_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

constexpr int kTrWaves = 8;
constexpr int kTrNT = kTrWaves * kWave;  // 512
constexpr int kTrMaxFT = 2;              // 32-feature tiles per wave (d <= 512)
constexpr int kTrMaxP = 16;              // hidden tiles = workgroups (h <= 512)
constexpr int kTrMaxO = 16;              // outputs (n_out <= 16)

struct TrainArgs {
  const float* lat;
  const float* lab;
  const int64_t* perm;
  int64_t n;
  int n_epochs;
  const float* vlat;  // nullable: no validation
  const float* vlab;
  const int64_t* vperm;
  int64_t nv;
  int valid_every, epoch0;
  float* valid_loss;
  int B, D, H, O, nTd, P, spe, nbv;
  float lr;
  float* w1;
  float* b1;
  float* w2;
  float* b2;
  float* step_loss;
  float* xbuf;    // [2][P][32 * O] output shares
  unsigned* ctl;  // arrival counter, abort word (zero at entry; left zero)
  int32_t* flag;
};

// Position in the run's item sequence: epoch e, item pos (< spe: training
// mini-batch, else validation batch pos - spe), vk = validations before e.
struct TrItem {
  int e, pos, vk;
};

__device__ __forceinline__ bool tr_valid_epoch(const TrainArgs& a, int e) {
  return a.vlat != nullptr && (a.epoch0 + e) % a.valid_every == 0;
}
__device__ __forceinline__ void tr_advance(const TrainArgs& a, TrItem& it) {
  const bool v = tr_valid_epoch(a, it.e);
  if (++it.pos >= a.spe + (v ? a.nbv : 0)) {
    it.pos = 0;
    it.vk += v ? 1 : 0;
    ++it.e;
  }
}
// rows of an item: index base into perm / vperm, row count
__device__ __forceinline__ void tr_rows(const TrainArgs& a, const TrItem& it, bool& train,
                                        int64_t& base, int& bc) {
  train = it.pos < a.spe;
  if (train) {
    base = static_cast<int64_t>(it.e) * a.n + static_cast<int64_t>(it.pos) * a.B;
    bc = static_cast<int>(min<int64_t>(a.B, a.n - static_cast<int64_t>(it.pos) * a.B));
  } else {
    const int j = it.pos - a.spe;
    base = static_cast<int64_t>(it.vk) * a.nv + static_cast<int64_t>(j) * a.B;
    bc = static_cast<int>(min<int64_t>(a.B, a.nv - static_cast<int64_t>(j) * a.B));
  }
}

// NTD: 32-feature tiles (d <= 32 NTD), a compile-time count so the row
// prefetch and the tile loops carry no runtime bounds
template <int NTD>
__global__ __launch_bounds__(kTrNT) void mlp_train_mc_kernel(TrainArgs a) {
  constexpr int DP = 32 * NTD, SX = DP + 1;
  constexpr int U = DP / 4;                                    // float4 units of a padded row
  constexpr int kPf = (kBatchMax * U + kTrNT - 1) / kTrNT;     // prefetched float4 per thread
  constexpr int kFT = (NTD + kTrWaves - 1) / kTrWaves;         // feature tiles per wave
  constexpr int nwu = NTD < kTrWaves ? NTD : kTrWaves;         // waves holding feature tiles
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int O = a.O;
  int64_t* s_perm = reinterpret_cast<int64_t*>(smem);  // [3][32] row indices
  float* sx = smem + 6 * kBatchMax;                     // [2][32][SX]
  float* sy = sx + 2 * kBatchMax * SX;                  // [2][32][O]
  float* spart = sy + 2 * kBatchMax * O;                // [8][32][32] (aliased by sdh)
  float* shid = spart + kTrWaves * kBatchMax * 32;      // [32][32]
  float* sg = shid + kBatchMax * 32;                    // [32][O]
  float* sW2 = sg + kBatchMax * O;                      // [O][32]
  float* sb1 = sW2 + O * 32;                            // [32]
  float* sb2 = sb1 + 32;                                // [O]
  float* s_red = sb2 + O;                               // [8]
  float* sdh = spart;                                   // [32][32]
  __shared__ int s_abort;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = blockIdx.x;       // hidden tile
  const int h0 = 32 * g;
  const int hl = lane & 31;       // this lane's hidden unit in MFMA layouts

  // parameters: this tile's W1^T (registers), W2 columns, b1, b2
  f32x16 wreg[kFT];
#pragma unroll
  for (int j = 0; j < kFT; ++j) {
    const int td = wave + kTrWaves * j;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int h = h0 + hl, d = 32 * td + c_row(r, lane);
      wreg[j][r] = (td < NTD && h < a.H && d < a.D) ? a.w1[static_cast<int64_t>(h) * a.D + d] : 0.f;
    }
  }
  for (int e = tid; e < O * 32; e += kTrNT) {
    const int o = e >> 5, h = h0 + (e & 31);
    sW2[e] = h < a.H ? a.w2[o * a.H + h] : 0.f;
  }
  if (tid < 32) sb1[tid] = h0 + tid < a.H ? a.b1[h0 + tid] : 0.f;
  if (tid < O) sb2[tid] = a.b2[tid];
  if (tid == 0) s_abort = 0;

  // rows of an item -> registers (one float4 unit per (row, unit) item)
  float4 pf[kPf];
  float pfy = 0.f;
  auto fetch_rows = [&](const TrItem& it, const int64_t* pidx) {
    bool train;
    int64_t base;
    int bc;
    tr_rows(a, it, train, base, bc);
    const float* src = train ? a.lat : a.vlat;
    const float* lsrc = train ? a.lab : a.vlab;
#pragma unroll
    for (int k = 0; k < kPf; ++k) {
      const int e = tid + kTrNT * k;
      const int b = e / U, u = e - b * U;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (it.e < a.n_epochs && b < bc && 4 * u < a.D)
        v = *reinterpret_cast<const float4*>(src + pidx[b] * a.D + 4 * u);
      pf[k] = v;
    }
    pfy = 0.f;
    if (it.e < a.n_epochs && tid < kBatchMax * O) {
      const int b = tid / O, o = tid - (tid / O) * O;
      if (b < bc) pfy = lsrc[pidx[b] * O + o];
    }
  };
  auto store_rows = [&](int buf) {
    float* dst = sx + buf * kBatchMax * SX;
#pragma unroll
    for (int k = 0; k < kPf; ++k) {
      const int e = tid + kTrNT * k;
      const int b = e / U, u = e - b * U;
      if (b < kBatchMax) {
        float* q = dst + b * SX + 4 * u;
        q[0] = pf[k].x; q[1] = pf[k].y; q[2] = pf[k].z; q[3] = pf[k].w;
      }
    }
    if (tid < kBatchMax * O) sy[buf * kBatchMax * O + tid] = pfy;
  };
  auto fetch_perm = [&](const TrItem& it, int slot) {
    if (wave == 0 && lane < kBatchMax && it.e < a.n_epochs) {
      bool train;
      int64_t base;
      int bc;
      tr_rows(a, it, train, base, bc);
      s_perm[slot * kBatchMax + lane] = lane < bc ? (train ? a.perm : a.vperm)[base + lane] : 0;
    }
  };

  // pipeline: item k's rows in sx[k & 1]; item k + 1's rows in registers
  // during k; item k + 2's indices land in s_perm during k
  TrItem cur{0, 0, 0}, nx1 = cur, nx2;
  tr_advance(a, nx1);
  nx2 = nx1;
  tr_advance(a, nx2);
  fetch_perm(cur, 0);
  fetch_perm(nx1, 1);
  __syncthreads();
  fetch_rows(cur, s_perm);
  store_rows(0);
  __syncthreads();
  unsigned xc = 0;  // exchanges so far
  for (int k = 0; cur.e < a.n_epochs; ++k) {
    bool train;
    int64_t base;
    int Bc;
    tr_rows(a, cur, train, base, Bc);
    const float* xs = sx + (k & 1) * kBatchMax * SX;
    const float* ys = sy + (k & 1) * kBatchMax * O;
    fetch_rows(nx1, s_perm + ((k + 1) % 3) * kBatchMax);  // in flight through this item
    fetch_perm(nx2, (k + 2) % 3);

    // 1. forward partial products of this wave's feature tiles
    if (wave < nwu) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const float* xb = xs + (lane & 31) * SX + 4 * (lane >> 5);
#pragma unroll
      for (int j = 0; j < kFT; ++j) {
        const int td = wave + kTrWaves * j;
        if (td < NTD) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xb[32 * td + (r & 3) + 8 * (r >> 2)], wreg[j][r],
                                                       acc, 0, 0, 0);
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) spart[(wave * kBatchMax + c_row(r, lane)) * 32 + hl] = acc[r];
    }
    __syncthreads();
    // 2. hid = relu(b1 + sum of the partials in wave order)
    for (int e = tid; e < kBatchMax * 32; e += kTrNT) {
      const int h = e & 31;
      float p = sb1[h];
      for (int w = 0; w < nwu; ++w) p += spart[w * kBatchMax * 32 + e];
      shid[e] = (h0 + h < a.H && p > 0.f) ? p : 0.f;
    }
    __syncthreads();
    // 3. this tile's share of the outputs -> exchange slot (write-through),
    //    drained by every storing wave before the arrival
    float* slot = a.xbuf + static_cast<int64_t>(xc & 1) * a.P * kBatchMax * O;
    if (tid < kBatchMax * O) {
      const int b = tid / O, o = tid - b * O;
      float yp = 0.f;
#pragma unroll 8
      for (int h = 0; h < 32; ++h) yp = fmaf(sW2[o * 32 + h], shid[b * 32 + h], yp);
      __hip_atomic_store(reinterpret_cast<unsigned*>(slot + g * kBatchMax * O + tid),
                         __float_as_uint(yp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    }
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(a.ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = static_cast<unsigned>(a.P) * (xc + 1);
      // exchange xc's arrivals find the counter in [P xc, P (xc + 1)); any
      // other count is a workspace handed over dirty: abort (as pm_arrive)
      bool ok = false;
      const bool counted = old >= target - static_cast<unsigned>(a.P) && old < target;
      for (int it = 0; counted && it < (1 << 21); ++it) {
        if (__hip_atomic_load(a.ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
        if (__hip_atomic_load(a.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) {
          ok = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (!ok) {  // ~1 s without the other workgroups, one of them gave up, or a dirty count
        __hip_atomic_store(a.ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.flag) atomicOr(a.flag, MMB_FLAG_SYNC_TIMEOUT);
        s_abort = 1;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (s_abort) return;
    ++xc;
    // 4. outputs = b2 + the P shares in tile order (identical everywhere),
    //    the L1 loss and its gradient sign(y - label) / (rows * o)
    float lsum = 0.f;
    if (tid < kBatchMax * O) {
      const int b = tid / O, o = tid - b * O;
      float sh[kTrMaxP];
#pragma unroll
      for (int q = 0; q < kTrMaxP; ++q)
        sh[q] = q < a.P ? __uint_as_float(__hip_atomic_load(
                              reinterpret_cast<const unsigned*>(slot + q * kBatchMax * O + tid),
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                        : 0.f;
      float y = sb2[o];
#pragma unroll
      for (int q = 0; q < kTrMaxP; ++q)
        if (q < a.P) y += sh[q];
      const float diff = y - ys[tid];
      const bool valid = b < Bc;
      sg[tid] = valid ? ((diff > 0.f) ? 1.f : (diff < 0.f ? -1.f : 0.f)) / static_cast<float>(Bc * O) : 0.f;
      if (valid) lsum = fabsf(diff);
    }
    lsum = wave_sum(lsum);
    if (lane == 0) s_red[wave] = lsum;
    __syncthreads();
    if (g == 0 && tid == 0) {
      float l = 0.f;
      for (int w = 0; w < kTrWaves; ++w) l += s_red[w];
      l /= static_cast<float>(Bc * O);
      if (train) a.step_loss[static_cast<int64_t>(cur.e) * a.spe + cur.pos] = l;
      else a.valid_loss[static_cast<int64_t>(cur.vk) * a.nbv + (cur.pos - a.spe)] = l;
    }
    if (train) {
      // 5. dH = relu'(.) g W2 (old W2)
      for (int e = tid; e < kBatchMax * 32; e += kTrNT) {
        const int b = e >> 5, h = e & 31;
        float s = 0.f;
        if (shid[e] > 0.f)
          for (int o = 0; o < O; ++o) s = fmaf(sg[b * O + o], sW2[o * 32 + h], s);
        sdh[e] = s;
      }
      __syncthreads();
      // 6. dW1^T = X^T dH on the own feature tiles (K = batch rows) and their
      //    SGD step; W2 / b1 (own tile) and b2 (everywhere) on VALU
      if (wave < nwu) {
#pragma unroll
        for (int j = 0; j < kFT; ++j) {
          const int td = wave + kTrWaves * j;
          if (td < NTD) {
            f32x16 acc;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
            for (int s2 = 0; s2 < kBatchMax / 2; ++s2) {
              const int b = 2 * s2 + (lane >> 5);
              acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xs[b * SX + 32 * td + (lane & 31)],
                                                         sdh[b * 32 + hl], acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) wreg[j][r] = fmaf(-a.lr, acc[r], wreg[j][r]);
          }
        }
      }
      for (int e = tid; e < O * 32; e += kTrNT) {
        const int o = e >> 5, h = e & 31;
        float gsum = 0.f;
        for (int b = 0; b < kBatchMax; ++b) gsum = fmaf(sg[b * O + o], shid[b * 32 + h], gsum);
        if (h0 + h < a.H) sW2[e] = fmaf(-a.lr, gsum, sW2[e]);
      }
      if (tid < 32) {
        float gsum = 0.f;
        for (int b = 0; b < kBatchMax; ++b) gsum += sdh[b * 32 + tid];
        if (h0 + tid < a.H) sb1[tid] = fmaf(-a.lr, gsum, sb1[tid]);
      }
      if (tid >= 64 && tid < 64 + O) {
        const int o = tid - 64;
        float gsum = 0.f;
        for (int b = 0; b < kBatchMax; ++b) gsum += sg[b * O + o];
        sb2[o] = fmaf(-a.lr, gsum, sb2[o]);
      }
    }
    // the next item's rows (loaded during this one) into the other buffer
    store_rows((k + 1) & 1);
    __syncthreads();
    cur = nx1;
    nx1 = nx2;
    tr_advance(a, nx2);
  }

  // the last workgroup past its final exchange returns the counter to 0 (the
  // next launch then needs no memset to find it there)
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(a.ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == static_cast<unsigned>(a.P) * (xc + 1) - 1)
      __hip_atomic_store(a.ctl, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // write this tile's parameters back (b2 by workgroup 0)
#pragma unroll
  for (int j = 0; j < kFT; ++j) {
    const int td = wave + kTrWaves * j;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int h = h0 + hl, d = 32 * td + c_row(r, lane);
      if (td < NTD && h < a.H && d < a.D) a.w1[static_cast<int64_t>(h) * a.D + d] = wreg[j][r];
    }
  }
  for (int e = tid; e < O * 32; e += kTrNT) {
    const int o = e >> 5, h = h0 + (e & 31);
    if (h < a.H) a.w2[o * a.H + h] = sW2[e];
  }
  if (tid < 32 && h0 + tid < a.H) a.b1[h0 + tid] = sb1[tid];
  if (g == 0 && tid < O) a.b2[tid] = sb2[tid];
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

template <int NTD>
static int launch_train_mc(const TrainArgs& a, size_t lds, hipStream_t stream) {
  // the dynamic LDS this launch needs (the kernel also has a static word, so
  // the full 160 KB cannot be requested)
  static size_t attr_set = 0;
  if (lds > attr_set) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_train_mc_kernel<NTD>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             static_cast<int>(lds));
    if (e != hipSuccess) return static_cast<int>(e);
    attr_set = lds;
  }
  // the P workgroups wait on each other every mini-batch, so they must be
  // resident together: check the occupancy the device gives this kernel, and
  // launch cooperatively where the device supports it (the runtime then
  // refuses a grid that cannot be co-resident instead of dispatching part of
  // it behind other work; the bounded waits stay as the last line)
  // (the CUs of the stream: a CU-masked stream co-schedules fewer)
  int dev = 0, per_cu = 0, coop = 0;
  const int n_cu = stream_cu_count(stream);
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
  if (e == hipSuccess)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, reinterpret_cast<const void*>(&mlp_train_mc_kernel<NTD>), kTrNT, lds);
  if (e != hipSuccess) return static_cast<int>(e);
  if (static_cast<int64_t>(per_cu) * n_cu < a.P) return MMB_EINVAL;
  if (coop) {
    TrainArgs arg = a;
    void* args[] = {&arg};
    e = hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&mlp_train_mc_kernel<NTD>),
                                   dim3(a.P), dim3(kTrNT), args, static_cast<unsigned>(lds), stream);
    return e == hipSuccess ? MMB_OK : static_cast<int>(e);
  }
  mlp_train_mc_kernel<NTD><<<a.P, kTrNT, lds, stream>>>(a);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
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
  (void)d;
  // arrival counter + abort word, then the double-buffered output shares
  return 16 + sizeof(float) * 2 * static_cast<size_t>(ceil_div(h, 32)) * kBatchMax * kTrMaxO;
}

extern "C" int mmb_mlp_train(const float* latents, const float* labels, const int64_t* perm,
                             int64_t n_per_epoch, int n_epochs, int batch, int d, int h, int o,
                             float lr, float* w1, float* b1, float* w2, float* b2,
                             float* step_loss, const float* v_latents, const float* v_labels,
                             const int64_t* v_perm, int64_t n_valid, int valid_every, int epoch0,
                             float* valid_loss, void* ws, int32_t* flag, hipStream_t stream) {
  MMB_REQUIRE(latents && labels && perm && w1 && b1 && w2 && b2 && step_loss && ws);
  MMB_REQUIRE(n_per_epoch > 0 && n_epochs >= 0 && batch >= 1 && batch <= kBatchMax);
  MMB_REQUIRE(d > 0 && d <= 32 * kTrWaves * kTrMaxFT && h > 0 && h <= 32 * kTrMaxP);
  MMB_REQUIRE(o >= 1 && o <= kTrMaxO && epoch0 >= 0);
  MMB_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 15) == 0 && (reinterpret_cast<uintptr_t>(latents) & 15) == 0);
  MMB_REQUIRE(d % 4 == 0);
  if (v_latents) {
    MMB_REQUIRE(v_labels && v_perm && valid_loss && n_valid > 0 && valid_every > 0);
    MMB_REQUIRE((reinterpret_cast<uintptr_t>(v_latents) & 15) == 0);
  }
  if (n_epochs == 0) return MMB_OK;
  TrainArgs a{};
  a.lat = latents; a.lab = labels; a.perm = perm; a.n = n_per_epoch; a.n_epochs = n_epochs;
  a.vlat = v_latents; a.vlab = v_labels; a.vperm = v_perm; a.nv = v_latents ? n_valid : 0;
  a.valid_every = v_latents ? valid_every : 1; a.epoch0 = epoch0; a.valid_loss = valid_loss;
  a.B = batch; a.D = d; a.H = h; a.O = o; a.lr = lr;
  a.w1 = w1; a.b1 = b1; a.w2 = w2; a.b2 = b2; a.step_loss = step_loss; a.flag = flag;
  a.nTd = static_cast<int>(ceil_div(d, 32));
  a.P = static_cast<int>(ceil_div(h, 32));
  a.spe = static_cast<int>(ceil_div(n_per_epoch, batch));
  a.nbv = v_latents ? static_cast<int>(ceil_div(n_valid, batch)) : 0;
  a.ctl = static_cast<unsigned*>(ws);
  a.xbuf = reinterpret_cast<float*>(static_cast<char*>(ws) + 16);
  const size_t lds = sizeof(float) * (6 * kBatchMax + 2 * static_cast<size_t>(kBatchMax) * (32 * a.nTd + 1) +
                                      2 * kBatchMax * o + kTrWaves * kBatchMax * 32 +
                                      kBatchMax * 32 + kBatchMax * o + o * 32 + 32 + o + kTrWaves);
  MMB_REQUIRE(lds <= 156 * 1024);
  // the control words are zero when ws is first handed over and the last
  // workgroup leaves them zero (no memset node: see mmb_pc_solve_mc)
  switch (a.nTd) {
#define MMB_TRAIN_NTD(n) \
    case n: return launch_train_mc<n>(a, lds, stream);
    MMB_TRAIN_NTD(1) MMB_TRAIN_NTD(2) MMB_TRAIN_NTD(3) MMB_TRAIN_NTD(4) MMB_TRAIN_NTD(5)
    MMB_TRAIN_NTD(6) MMB_TRAIN_NTD(7) MMB_TRAIN_NTD(8) MMB_TRAIN_NTD(9) MMB_TRAIN_NTD(10)
    MMB_TRAIN_NTD(11) MMB_TRAIN_NTD(12) MMB_TRAIN_NTD(13) MMB_TRAIN_NTD(14) MMB_TRAIN_NTD(15)
    MMB_TRAIN_NTD(16)
#undef MMB_TRAIN_NTD
    default: return MMB_EINVAL;
  }
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
      const hipError_t e = static_cast<hipError_t>(zero_words_async(outs[q], static_cast<int64_t>(nbytes[q]) / 4, stream));
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
