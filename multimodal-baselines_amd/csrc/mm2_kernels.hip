// Closed-form MMB2 projection (a7/a8 after the frame sums) for MI355X.
//
// The reference (sif2.py:164-208) materialises q_mean/q_sigma [N,T,F_k] for
// six modality combinations and runs twelve [N,T,F_k] x [F_k,300] matmuls
// before summing over T.  Both q's are affine in the frame values, so the sum
// over T commutes with them (exact algebra):
//   sum_t q_mean_k  = a_k (Sx - T b_k)
//   sum_t q_sigma_k = a_k (Sxx - 2 b_k Sx + T b_k^2) - T,   a_k = 1/exp(2 ls_k)
// with Sx, Sxx the per-feature frame sums of each raw modality (streamed by
// mmb_mm2_stream).  All twelve projections then fold into ONE merged matrix
// Wm [2(d+a+vd), d+1] (column d accumulates the total weight, sif2.py:186-188)
// and a constant c0 — a single [N,K] x [K,ldw] fp32-MFMA GEMM with the
// division by the total weight and the row L2 normalisation (:207) fused into
// its epilogue.
#include "mmb_common.h"

namespace mmb {

struct PrepArgs {
  const float* wmu[6];
  const float* bmu[6];
  const float* wls[6];
  const float* bls[6];
  int D, A, Vd, T, ldw, Kp;
  float* wm;
  float* c0;
};

// Offset of modality m (0 text, 1 audio, 2 visual) inside combination k's
// feature vector (torch.cat order text, audio, visual), or -1.
__host__ __device__ inline int combo_offset(int k, int m, int D, int A) {
  // keys: 0 audio, 1 visual, 2 audiovisual, 3 textaudio, 4 textvisual, 5 textaudiovisual
  switch (k) {
    case 0: return m == 1 ? 0 : -1;
    case 1: return m == 2 ? 0 : -1;
    case 2: return m == 1 ? 0 : (m == 2 ? A : -1);
    case 3: return m == 0 ? 0 : (m == 1 ? D : -1);
    case 4: return m == 0 ? 0 : (m == 2 ? D : -1);
    default: return m == 0 ? 0 : (m == 1 ? D : D + A);
  }
}

__host__ __device__ inline int combo_width(int k, int D, int A, int Vd) {
  switch (k) {
    case 0: return A;
    case 1: return Vd;
    case 2: return A + Vd;
    case 3: return D + A;
    case 4: return D + Vd;
    default: return D + A + Vd;
  }
}

__global__ void mm2_prepare_wm_kernel(PrepArgs p) {
  const int K = 2 * (p.D + p.A + p.Vd);
  const int64_t total = static_cast<int64_t>(p.Kp) * p.ldw;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int r = static_cast<int>(e / p.ldw), j = static_cast<int>(e % p.ldw);
    double acc = 0.0;
    if (r < K && j <= p.D) {
      // row r -> (modality m, kind sq, feature f)
      int m, f, sq;
      if (r < 2 * p.D) { m = 0; sq = r >= p.D; f = r - sq * p.D; }
      else if (r < 2 * p.D + 2 * p.A) { m = 1; const int rr = r - 2 * p.D; sq = rr >= p.A; f = rr - sq * p.A; }
      else { m = 2; const int rr = r - 2 * p.D - 2 * p.A; sq = rr >= p.Vd; f = rr - sq * p.Vd; }
      for (int k = 0; k < 6; ++k) {
        const int o = combo_offset(k, m, p.D, p.A);
        if (o < 0) continue;
        const int ff = o + f;
        const double b = p.bmu[k][ff];
        const double al = 1.0 / exp(2.0 * static_cast<double>(p.bls[k][ff]));
        if (j < p.D) {
          const double wmu = p.wmu[k][static_cast<int64_t>(ff) * p.D + j];
          const double wls = p.wls[k][static_cast<int64_t>(ff) * p.D + j];
          acc += sq ? al * wls : al * (wmu - 2.0 * b * wls);
        } else {
          acc += sq ? al : al * (1.0 - 2.0 * b);
        }
      }
    }
    p.wm[e] = static_cast<float>(acc);
  }
}

// c0[j] = T * sum_k sum_f (-a b Wmu + a b^2 Wls - Wls)[f][j];  c0[d] = T * sum (-a b + a b^2 - 1)
// Block: 64 columns x 16 feature groups; fixed-order combine (deterministic).
__global__ __launch_bounds__(1024) void mm2_prepare_c0_kernel(PrepArgs p) {
  __shared__ double s_part[16][64];
  const int jl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + jl;
  double acc = 0.0;
  if (j <= p.D) {
    for (int k = 0; k < 6; ++k) {
      const int F = combo_width(k, p.D, p.A, p.Vd);
      for (int f = g; f < F; f += 16) {
        const double b = p.bmu[k][f];
        const double al = 1.0 / exp(2.0 * static_cast<double>(p.bls[k][f]));
        if (j < p.D) {
          const double wmu = p.wmu[k][static_cast<int64_t>(f) * p.D + j];
          const double wls = p.wls[k][static_cast<int64_t>(f) * p.D + j];
          acc += -al * b * wmu + al * b * b * wls - wls;
        } else {
          acc += -al * b + al * b * b - 1.0;
        }
      }
    }
  }
  s_part[g][jl] = acc;
  __syncthreads();
  if (g == 0 && j < p.ldw) {
    double s = 0.0;
    for (int q = 0; q < 16; ++q) s += s_part[q][jl];
    p.c0[j] = (j <= p.D) ? static_cast<float>(s * p.T) : 0.f;
  }
}

// The same c0 with the features of all six combinations cut into S splits:
// block (column group, split) reduces its split into part[split][ldw] (f64),
// mm2_c0_reduce_kernel sums the splits in a fixed order (deterministic).
constexpr int kC0Splits = 64;
__global__ __launch_bounds__(1024) void mm2_prepare_c0_part_kernel(PrepArgs p, double* part) {
  __shared__ double s_part[16][64];
  const int jl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + jl, split = blockIdx.y;
  int Ftot = 0;
  for (int k = 0; k < 6; ++k) Ftot += combo_width(k, p.D, p.A, p.Vd);
  const int per = (Ftot + kC0Splits - 1) / kC0Splits;
  const int e0 = split * per, e1 = min(Ftot, e0 + per);
  double acc = 0.0;
  if (j <= p.D) {
    for (int e = e0 + g; e < e1; e += 16) {
      int k = 0, f = e;
      while (f >= combo_width(k, p.D, p.A, p.Vd)) {
        f -= combo_width(k, p.D, p.A, p.Vd);
        ++k;
      }
      const double b = p.bmu[k][f];
      const double al = 1.0 / exp(2.0 * static_cast<double>(p.bls[k][f]));
      if (j < p.D) {
        const double wmu = p.wmu[k][static_cast<int64_t>(f) * p.D + j];
        const double wls = p.wls[k][static_cast<int64_t>(f) * p.D + j];
        acc += -al * b * wmu + al * b * b * wls - wls;
      } else {
        acc += -al * b + al * b * b - 1.0;
      }
    }
  }
  s_part[g][jl] = acc;
  __syncthreads();
  if (g == 0 && j < p.ldw) {
    double s = 0.0;
    for (int q = 0; q < 16; ++q) s += s_part[q][jl];
    part[static_cast<int64_t>(split) * p.ldw + j] = s;
  }
}

__global__ void mm2_c0_reduce_kernel(const double* __restrict__ part, int D, int ldw, int T,
                                     float* __restrict__ c0) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ldw) return;
  double s = 0.0;
  for (int q = 0; q < kC0Splits; ++q) s += part[static_cast<int64_t>(q) * ldw + j];
  c0[j] = (j <= D) ? static_cast<float>(s * T) : 0.f;
}

// ------------------------------------------------------------------ projection
// fp32 MFMA 32x32x2: lane l holds A[l&31][l>>5] and B[l>>5][l&31];
// C/D: col = l&31, row = (reg&3) + 8*(reg>>2) + 4*(l>>5).
using f32x16 = __attribute__((ext_vector_type(16))) float;


constexpr int kPM = 64;   // rows per workgroup
constexpr int kPK = 32;   // K chunk staged in LDS

template <int CT>  // 32-wide column tiles per wave; ldw = 64*CT
__global__ __launch_bounds__(256) void mm2_project_kernel(const float* __restrict__ S,
                                                          const float* __restrict__ num,
                                                          const float* __restrict__ aux,
                                                          const float* __restrict__ Wm,
                                                          const float* __restrict__ c0, int64_t N,
                                                          int Kp, int D, float* __restrict__ out) {
  constexpr int LDW = 64 * CT;
  __shared__ float sA[kPM][kPK + 1];
  __shared__ float sB[kPK][LDW];
  __shared__ float s_tot[kPM];
  __shared__ float s_ss[2][kPM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int64_t n0 = static_cast<int64_t>(blockIdx.x) * kPM;

  f32x16 acc[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  for (int k0 = 0; k0 < Kp; k0 += kPK) {
    // A tile 64 x 32 (float4 loads, 2 per thread)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + 256 * q;
      const int row = idx >> 3, c4 = idx & 7;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (n0 + row < N) v = *reinterpret_cast<const float4*>(S + (n0 + row) * Kp + k0 + c4 * 4);
      sA[row][c4 * 4 + 0] = v.x;
      sA[row][c4 * 4 + 1] = v.y;
      sA[row][c4 * 4 + 2] = v.z;
      sA[row][c4 * 4 + 3] = v.w;
    }
    // B tile 32 x LDW
    for (int idx = tid; idx < kPK * LDW / 4; idx += 256) {
      const int row = idx / (LDW / 4), c4 = idx % (LDW / 4);
      *reinterpret_cast<float4*>(&sB[row][c4 * 4]) =
          *reinterpret_cast<const float4*>(Wm + static_cast<int64_t>(k0 + row) * LDW + c4 * 4);
    }
    __syncthreads();
#pragma unroll 4
    for (int kk = 0; kk < kPK; kk += 2) {
      const float a = sA[wr * 32 + (lane & 31)][kk + (lane >> 5)];
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        const float b = sB[kk + (lane >> 5)][(wc * CT + t) * 32 + (lane & 31)];
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // epilogue: y = acc + (num | sum w) + c0; cs = y / total; out = cs / ||cs||
  const int hl = lane >> 5, cl = lane & 31;
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    const int col = (wc * CT + t) * 32 + cl;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
      const int64_t row = n0 + rl;
      float add = 0.f;
      if (row < N) {
        if (col < D) add = text_sum(num[row * D + col], aux[row]) + c0[col];
        else if (col == D) add = aux[N + row] + c0[D];
      }
      acc[t][r] += add;
      if (col == D) s_tot[rl] = acc[t][r];
    }
  }
  __syncthreads();
  float ss[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) ss[r] = 0.f;
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    const int col = (wc * CT + t) * 32 + cl;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
      const float cs = acc[t][r] / s_tot[rl];
      acc[t][r] = cs;
      if (col < D) ss[r] = fmaf(cs, cs, ss[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float s = half_sum(ss[r]);
    if (cl == 0) s_ss[wc][wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl] = s;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int rl = wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
    const int64_t row = n0 + rl;
    const float nrm = sqrtf(s_ss[0][rl] + s_ss[1][rl]);
    if (row < N) {
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        const int col = (wc * CT + t) * 32 + cl;
        if (col < D) out[row * D + col] = acc[t][r] / nrm;
      }
    }
  }
}

// ------------------------------------------------------------------ fp16x3 projection
// The same GEMM on the f16 MFMA pipe (32x32x16, 16x the fp32 MFMA rate): each
// operand is split into an fp16 hi part and an fp16 lo part (the residual),
// after a power-of-2 scale per S row (from the stream kernel) and per Wm
// column (from the split kernel) that puts each row/column max in
// [2^14, 2^15).  a*b ~= ah*bh + ah*bl + al*bh: three f16 MFMAs per product,
// ~22 significant bits per operand, products exact, fp32 accumulation —
// 5.3x fewer MFMA cycles than fp32 MFMA at fp32-class accuracy.
// f16 32x32x16: lane l holds A[l&31][8(l>>5)+j] and B[8(l>>5)+j][l&31], j<8.
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
using half4 = __attribute__((ext_vector_type(4))) _Float16;

constexpr int kXM = 128;  // rows per workgroup (8 waves: 4 row tiles x 2 column halves)
constexpr int kXK = 32;   // K chunk (2 MFMA k-steps)
constexpr int kXT = 512;  // threads
constexpr int kXAbuf = 4; // A chunk ring (3 chunks in flight from HBM)
constexpr int kXBbuf = 2; // B chunk ring (1 chunk in flight from L2)


// Weight split, written in the projection kernel's B chunk image order so the
// kernel stages B with straight 16-byte global->LDS copies:
//   img[c][plane][col][slot position q] = plane(Wm[32c + 8 (q ^ swz(col)) + e][col] * scale_col)
// plane 0 = fp16 hi, 1 = fp16 lo (residual); col_inv[col] = 1 / scale_col.
__global__ void mm2_split_wm_kernel(const float* __restrict__ wm, int Kp, int ldw,
                                    _Float16* __restrict__ img, float* __restrict__ col_inv) {
  __shared__ float s_m[4];
  const int j = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float m = 0.f;
  for (int k = tid; k < Kp; k += blockDim.x) m = fmaxf(m, fabsf(wm[static_cast<int64_t>(k) * ldw + j]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, kWave));
  if (lane == 0) s_m[wave] = m;
  __syncthreads();
  m = fmaxf(fmaxf(s_m[0], s_m[1]), fmaxf(s_m[2], s_m[3]));
  float sc = 1.f;
  if (m > 0.f && isfinite(m)) {
    int ex;
    frexpf(m, &ex);
    sc = ldexpf(1.f, 15 - ex);
  }
  for (int k = tid; k < Kp; k += blockDim.x) {
    const float v = wm[static_cast<int64_t>(k) * ldw + j] * sc;
    const _Float16 h = static_cast<_Float16>(v);
    const int c = k / kXK, kk = k % kXK;
    const int64_t at = static_cast<int64_t>(c) * 2 * ldw * kXK + static_cast<int64_t>(j) * kXK +
                       ((kk >> 3) ^ x3_swz(j)) * 8 + (kk & 7);
    img[at] = h;
    img[at + static_cast<int64_t>(ldw) * kXK] = static_cast<_Float16>(v - static_cast<float>(h));
  }
  if (tid == 0) col_inv[j] = 1.f / sc;
}

// The same split in PIECE order for the fused stream + projection kernel
// (mmb_mm2_stream_project): the K rows of each raw modality's sums
// [Sx_m | Sxx_m] (2 w_m rows) padded to a multiple of 32, so every 32-deep
// chunk belongs to one modality piece.  Chunk layout and column scales as
// mm2_split_wm_kernel (the same col_inv).
__global__ void mm2_split_wm_pieces_kernel(const float* __restrict__ wm, int ldw, int D, int A,
                                           int Vd, _Float16* __restrict__ img,
                                           float* __restrict__ col_inv) {
  __shared__ float s_m[4];
  const int j = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int w[3] = {D, A, Vd};
  int src0[3], dst0[3], kq[3];
  int sb = 0, db = 0;
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    src0[m] = sb;
    dst0[m] = db;
    kq[m] = (2 * w[m] + 31) / 32 * 32;
    sb += 2 * w[m];
    db += kq[m];
  }
  const int K = sb, Kq = db;
  float m = 0.f;
  for (int k = tid; k < K; k += blockDim.x) m = fmaxf(m, fabsf(wm[static_cast<int64_t>(k) * ldw + j]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, kWave));
  if (lane == 0) s_m[wave] = m;
  __syncthreads();
  m = fmaxf(fmaxf(s_m[0], s_m[1]), fmaxf(s_m[2], s_m[3]));
  float sc = 1.f;
  if (m > 0.f && isfinite(m)) {
    int ex;
    frexpf(m, &ex);
    sc = ldexpf(1.f, 15 - ex);
  }
  for (int k = tid; k < Kq; k += blockDim.x) {
    const int pm = k < dst0[1] ? 0 : (k < dst0[2] ? 1 : 2);
    const int r = k - dst0[pm];
    const float v = r < 2 * w[pm] ? wm[static_cast<int64_t>(src0[pm] + r) * ldw + j] * sc : 0.f;
    const _Float16 h = static_cast<_Float16>(v);
    const int c = k / kXK, kk = k % kXK;
    const int64_t at = static_cast<int64_t>(c) * 2 * ldw * kXK + static_cast<int64_t>(j) * kXK +
                       ((kk >> 3) ^ x3_swz(j)) * 8 + (kk & 7);
    img[at] = h;
    img[at + static_cast<int64_t>(ldw) * kXK] = static_cast<_Float16>(v - static_cast<float>(h));
  }
  if (tid == 0) col_inv[j] = 1.f / sc;
}

template <int CT>
constexpr int x3_bbuf_halves() { return 2 * 64 * CT * kXK; }  // hi + lo planes of a chunk
constexpr int kXAbufHalves = 2 * kXM * kXK;
template <int CT>
constexpr size_t x3_lds_bytes() {
  return (kXBbuf * x3_bbuf_halves<CT>() + kXAbuf * kXAbufHalves) * sizeof(_Float16) +
         4 * kXM * sizeof(float);
}

using gptr_t = const __attribute__((address_space(1))) void*;
using lptr_t = __attribute__((address_space(3))) void*;

// 16 bytes per lane global -> LDS; the LDS destination is the wave-uniform
// `lds` plus 16 * lane (M0 = readfirstlane(lds))
__device__ __forceinline__ void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds((gptr_t)g, (lptr_t)lds, 16, 0, 0);
}




// Row-wise epilogue (D % 4 == 0, 16-byte aligned rows, 256 <= D < 320) of
// the fp16x3 projection kernels: the raw accumulators of 64 rows at a time
// go through the idle LDS rings (row stride 324 floats: the 4 row groups of
// an MFMA store land on disjoint banks), then each wave finishes 8 whole rows
// with 16-byte loads / stores: lane l owns columns 4l.. and 256 + 4l.. .  One
// read of x serves the weighted text sum and the fused PC removal.  M rows
// per workgroup; each wave row block (wr) holds NI 16-row tiles; a wave
// finishes Q rows at a time (all their loads first).
// LAYOUT 0: waves (wr, wc) = 2 x 4, a wave holds rows wr*64 + 16 i, columns
// (wc*CT + t)*16 (acc[NI][CT]); LAYOUT 1: waves 4 x 2, rows wr*32 + 16 i,
// columns (wc*NT + t)*16 (acc[2][NT], NT = 10); LAYOUT 2: waves 4 x 2 of a
// 256-row tile, rows wr*64 + 16 i (acc[4][NT]).
template <int CT, int NI, int Q = 4, int LAYOUT = 0, int NT = CT>
__device__ __forceinline__ void x3_row_epilogue(f32x4 (&acc)[NI][NT], float* sacc, const float* s_rs,
                                                int M, int wr, int wc, int lq, int lc, int wave,
                                                int lane, int64_t n0, int64_t N, int D,
                                                const float* __restrict__ num,
                                                const float* __restrict__ aux,
                                                const float* __restrict__ col_inv,
                                                const float* __restrict__ c0,
                                                const double* __restrict__ pc,
                                                float* __restrict__ out, float* __restrict__ sif) {
  constexpr int LDW = 64 * CT;
  constexpr int kRS = 324;
  const int U = D >> 2;                 // float4 units of a row
  const bool u1 = lane + 64 < U;        // second unit (columns 256 + 4l..)
  const int c0a = 4 * lane, c1a = 256 + 4 * min(lane, 15);  // acc columns (LDW <= 320)
  const int c0x = 4 * min(lane, U - 1), c1x = 4 * min(lane + 64, U - 1);
  float4 ci0, ci1, ca0, ca1;
  {
    const int cA = min(c0a, LDW - 4), cB = c1a;
    ci0 = make_float4(col_inv[cA], col_inv[cA + 1], col_inv[cA + 2], col_inv[cA + 3]);
    ca0 = make_float4(c0[cA], c0[cA + 1], c0[cA + 2], c0[cA + 3]);
    ci1 = make_float4(col_inv[cB], col_inv[cB + 1], col_inv[cB + 2], col_inv[cB + 3]);
    ca1 = make_float4(c0[cB], c0[cB + 1], c0[cB + 2], c0[cB + 3]);
  }
  double pv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) pv[e] = 0.0;
  if (pc) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      pv[e] = lane < U ? pc[c0x + e] : 0.0;
      pv[4 + e] = u1 ? pc[c1x + e] : 0.0;
    }
  }
  const int lane_tot = (D - 256) >> 2, e_tot = (D - 256) & 3;  // column D in unit 1
#pragma unroll 1
  for (int p = 0; p < M / 64; ++p) {
    __syncthreads();  // the rings' last reads / the previous pass's rows
    // the wave row block holding rows [64 p, 64 p + 64): its tiles i with
    // 16 i in that range, i.e. i / 4 == ip
    if constexpr (LAYOUT == 0) {
      const int ip = ((p * 64) % (NI * 16)) / 64;
      if (wr == (p * 64) / (NI * 16)) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
          if (i / 4 == ip)
#pragma unroll
            for (int t = 0; t < CT; ++t)
#pragma unroll
              for (int j = 0; j < 4; ++j)
                sacc[((i % 4) * 16 + lq * 4 + j) * kRS + (wc * CT + t) * 16 + lc] = acc[i][t][j];
      }
    } else if constexpr (LAYOUT == 2) {
      if (wr == p) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              sacc[(i * 16 + lq * 4 + j) * kRS + (wc * NT + t) * 16 + lc] = acc[i][t][j];
      }
    } else {
      if ((wr >> 1) == p) {
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              sacc[((wr & 1) * 32 + i * 16 + lq * 4 + j) * kRS + (wc * NT + t) * 16 + lc] = acc[i][t][j];
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int h = 0; h < 8 / Q; ++h) {
      // Q rows of this wave: all loads first
      float4 xa[Q], xb[Q], aa[Q], ab[Q];
      float cn[Q], tw[Q];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int rl = p * 64 + wave * 8 + h * Q + q;
        const int64_t rowc = min(n0 + rl, N - 1);
        xa[q] = *reinterpret_cast<const float4*>(num + rowc * D + c0x);
        xb[q] = *reinterpret_cast<const float4*>(num + rowc * D + c1x);
        cn[q] = aux[rowc];
        tw[q] = aux[N + rowc];
        const float* sr = sacc + (rl - p * 64) * kRS;
        aa[q] = *reinterpret_cast<const float4*>(sr + c0a);
        ab[q] = *reinterpret_cast<const float4*>(sr + c1a);
      }
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int rl = p * 64 + wave * 8 + h * Q + q;
        const int64_t row = n0 + rl;
        const float irs = s_rs[rl];
        // y = unscaled product + (weighted text sum x * count, or the total
        // weight sum_t w at column D) + c0 -- the tile epilogue's order
        const float av[8] = {aa[q].x, aa[q].y, aa[q].z, aa[q].w, ab[q].x, ab[q].y, ab[q].z, ab[q].w};
        const float civ[8] = {ci0.x, ci0.y, ci0.z, ci0.w, ci1.x, ci1.y, ci1.z, ci1.w};
        const float cav[8] = {ca0.x, ca0.y, ca0.z, ca0.w, ca1.x, ca1.y, ca1.z, ca1.w};
        const float xv[8] = {xa[q].x, xa[q].y, xa[q].z, xa[q].w, xb[q].x, xb[q].y, xb[q].z, xb[q].w};
        float y[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int col = (e < 4 ? c0a : 256 + 4 * lane) + (e & 3);
          const bool in = e < 4 ? lane < U : u1;
          const float add = (in && col < D) ? text_sum(xv[e], cn[q]) : (col == D ? tw[q] : 0.f);
          y[e] = av[e] * (civ[e] * irs) + add + cav[e];
        }
        // the total (column D) from its lane; cs = y / total
        const float ysel = e_tot == 0 ? y[4] : e_tot == 1 ? y[5] : e_tot == 2 ? y[6] : y[7];
        const float tot = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ysel), lane_tot));
        const float rt = 1.f / tot;
        float ss = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool in = e < 4 ? lane < U : u1;
          y[e] *= rt;
          if (in) ss = fmaf(y[e], y[e], ss);
        }
        const float inv = 1.f / sqrtf(wave_sum_dpp_f32(ss));
        double dot = 0.0;
        if (pc) {
#pragma unroll
          for (int e = 0; e < 8; ++e) dot = fma(static_cast<double>(xv[e]), pv[e], dot);
          dot = wave_sum_dpp(dot);
        }
        if (row < N) {
          float* orow = out + row * D;
          if (lane < U)
            *reinterpret_cast<float4*>(orow + c0x) =
                make_float4(y[0] * inv, y[1] * inv, y[2] * inv, y[3] * inv);
          if (u1)
            *reinterpret_cast<float4*>(orow + c1x) =
                make_float4(y[4] * inv, y[5] * inv, y[6] * inv, y[7] * inv);
          if (pc) {
            float* srow = sif + row * D;
            float o[8];
#pragma unroll
            for (int e = 0; e < 8; ++e)
              o[e] = static_cast<float>(static_cast<double>(xv[e]) - dot * pv[e]);
            if (lane < U) *reinterpret_cast<float4*>(srow + c0x) = make_float4(o[0], o[1], o[2], o[3]);
            if (u1) *reinterpret_cast<float4*>(srow + c1x) = make_float4(o[4], o[5], o[6], o[7]);
          }
        }
      }
    }
  }
}

// DIAG (timing-only builds, wrong outputs; MMB_PROJ_DIAG): bit 0 skips the
// epilogue (accumulators kept live), bit 1 stages A chunk 0 every time
// (L2-resident A), bit 2 B chunk 0 every time, bit 3 drops the MFMAs (the
// fragment reads kept live)
// SPLIT (r06, a few rows: POM's 100 / 203-row splits ran the whole K loop on
// one or two workgroups, ~75 us): workgroup (tile, slice) = (blockIdx.x /
// nsl, blockIdx.x % nsl) runs chunks [slice * cps, (slice + 1) * cps) of the
// K loop and writes its raw accumulators to `part` for x3_splitk_finish_kernel.
template <int CT, bool ROWEPI, bool PIPE = false, int DIAG = 0, bool SPLIT = false>
__global__ __launch_bounds__(kXT) void mm2_project_x3b_kernel(
    const _Float16* __restrict__ S, const float* __restrict__ num, const float* __restrict__ aux,
    const _Float16* __restrict__ img, const float* __restrict__ col_inv,
    const float* __restrict__ c0, int64_t N, int Kp, int D, float* __restrict__ out,
    const double* __restrict__ pc, float* __restrict__ sif, int nsl = 1, int cps = 0,
    f32x4* __restrict__ part = nullptr) {
  constexpr int LDW = 64 * CT;
  constexpr int BBUF = x3_bbuf_halves<CT>();
  constexpr int BQ = BBUF * 2 / 16 / kXT;  // 16-byte pieces per thread per B chunk (= CT)
  constexpr int AQ = kXAbufHalves * 2 / 16 / kXT;  // = 2
  static_assert(BQ * kXT * 16 == BBUF * 2 && AQ * kXT * 16 == kXAbufHalves * 2, "staging split");
  // one dynamic LDS array: B ring, A ring, per-row scalars
  extern __shared__ __attribute__((aligned(16))) _Float16 lds[];
  _Float16* bring = lds;
  _Float16* aring = lds + kXBbuf * BBUF;
  float* s_rs = reinterpret_cast<float*>(aring + kXAbuf * kXAbufHalves);
  float* s_tot = s_rs + kXM;
  float(*s_ss)[kXM] = reinterpret_cast<float(*)[kXM]>(s_tot + kXM);  // [4][kXM]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // wave (wr, wc): rows wr*64 + [0,64) as 4 16-row tiles, columns
  // wc*16*CT + [0,16*CT) as CT 16-column tiles (v_mfma_f32_16x16x32_f16:
  // lane l holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15],
  // D[row 4(l>>4)+j][col l&15])
  const int wr = wave >> 2, wc = wave & 3;
  const int lq = lane >> 4, lc = lane & 15;
  const int tile = SPLIT ? static_cast<int>(blockIdx.x) / nsl : static_cast<int>(blockIdx.x);
  const int slice = SPLIT ? static_cast<int>(blockIdx.x) - tile * nsl : 0;
  const int64_t n0 = static_cast<int64_t>(tile) * kXM;
  // this workgroup's chunks [kc0, kc0 + nch) (all of K unless SPLIT)
  const int kc0 = SPLIT ? slice * cps : 0;
  const int nch = SPLIT ? min(cps, Kp / kXK - kc0) : Kp / kXK;

  // A piece g = q * kXT + tid of a chunk: plane g >> 9, row (g >> 2) & 127,
  // LDS slot position g & 3 <- data slot (g & 3) ^ swz(row); rows past N
  // re-read row N-1 (never stored)
  const _Float16* asrc[AQ];
#pragma unroll
  for (int q = 0; q < AQ; ++q) {
    const int g = q * kXT + tid;
    const int plane = g >> 9, row = (g >> 2) & (kXM - 1);
    const int64_t r = min(n0 + row, N - 1);
    asrc[q] = S + r * 2 * Kp + plane * Kp + ((g & 3) ^ x3_swz(row)) * 8;
  }
  auto stage_a = [&](int c) {
    if ((DIAG & 64) && c >= 3) return;
    const int cc = (DIAG & 2) ? 0 : kc0 + min(c, nch - 1);
    _Float16* dst = aring + (c & (kXAbuf - 1)) * kXAbufHalves;
#pragma unroll
    for (int q = 0; q < AQ; ++q)
      glds16(asrc[q] + cc * kXK, dst + (q * kXT + wave * 64) * 8);
  };
  auto stage_b = [&](int c) {
    if ((DIAG & 32) && c >= 2) return;
    const int cc = (DIAG & 4) ? 0 : kc0 + min(c, nch - 1);
    const _Float16* src = img + static_cast<int64_t>(cc) * BBUF;
    _Float16* dst = bring + (c & (kXBbuf - 1)) * BBUF;
#pragma unroll
    for (int q = 0; q < BQ; ++q) glds16(src + (q * kXT + tid) * 8, dst + (q * kXT + wave * 64) * 8);
  };

  // 1 / row scale (a power of two: exact)
  if (tid < kXM) s_rs[tid] = (n0 + tid < N) ? 1.f / aux[2 * N + n0 + tid] : 1.f;

  f32x4 acc[4][CT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < CT; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (PIPE) {
    // Software-pipelined K loop: the fragments an MFMA consumes were read
    // from LDS while the previous MFMAs ran.  B(c+1)'s fragments (a second
    // register set) are read during chunk c's MFMAs; A(c)'s row tiles one
    // tile ahead (A(c+1) tile 0 during chunk c's last tile).  One barrier per
    // chunk, placed where chunk c+1 has landed (own copies by a counted
    // vmcnt that leaves A(c+2) in flight, everyone's by the barrier) and
    // every wave has finished reading B(c) and A(c-1) -- whose ring slots
    // the copies issued right after it (B(c+2), A(c+3)) overwrite.  The
    // MFMA pipe then idles only for the barrier skew, not for LDS latency.
    stage_b(0);
    stage_a(0);
    stage_a(1);
    stage_b(1);
    stage_a(2);
    // B(0), A(0) landed; A(1), B(1), A(2) may be in flight
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * AQ + BQ) : "memory");
    __builtin_amdgcn_s_barrier();
    half8 bh0[CT], bl0[CT], bh1[CT], bl1[CT], ah0, al0, ah1, al1;
    if constexpr ((DIAG & 16) != 0) {
      const half8 z = {};
      ah0 = al0 = ah1 = al1 = z;
#pragma unroll
      for (int t = 0; t < CT; ++t) bh0[t] = bl0[t] = bh1[t] = bl1[t] = z;
    }
    auto rd_b = [&](int c, half8 (&bh)[CT], half8 (&bl)[CT]) {
      if constexpr ((DIAG & 16) != 0) {
#pragma unroll
        for (int t = 0; t < CT; ++t) asm volatile("" : "+v"(bh[t]), "+v"(bl[t]));
        return;
      }
      const _Float16* b = bring + (c & (kXBbuf - 1)) * BBUF;
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        const int col = (wc * CT + t) * 16 + lc;
        const int bo = col * kXK + ((lq ^ x3_swz(col)) * 8);
        bh[t] = *reinterpret_cast<const half8*>(b + bo);
        bl[t] = *reinterpret_cast<const half8*>(b + LDW * kXK + bo);
      }
    };
    auto rd_a = [&](int c, int i, half8& ah, half8& al) {
      if constexpr ((DIAG & 16) != 0) {
        asm volatile("" : "+v"(ah), "+v"(al));
        return;
      }
      const _Float16* a = aring + (c & (kXAbuf - 1)) * kXAbufHalves;
      const int row = wr * 64 + i * 16 + lc;
      const int ao = row * kXK + ((lq ^ x3_swz(row)) * 8);
      ah = *reinterpret_cast<const half8*>(a + ao);
      al = *reinterpret_cast<const half8*>(a + kXM * kXK + ao);
    };
    auto tile = [&](int i, const half8& ah, const half8& al, const half8 (&bh)[CT],
                    const half8 (&bl)[CT]) {
      if constexpr ((DIAG & 8) != 0) {
        asm volatile("" ::"v"(ah), "v"(al));
#pragma unroll
        for (int t = 0; t < CT; ++t) asm volatile("" ::"v"(bh[t]), "v"(bl[t]));
        return;
      }
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[t], acc[i][t], 0, 0, 0);
        acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[t], acc[i][t], 0, 0, 0);
        acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[t], acc[i][t], 0, 0, 0);
      }
    };
    rd_b(0, bh0, bl0);
    rd_a(0, 0, ah0, al0);
    // chunk c with B(c) in (bh, bl), A(c) tile 0 in (ah0, al0); reads B(c+1)
    // into (nbh, nbl) and leaves A(c+1) tile 0 in (ah0, al0)
    auto chunk = [&](int c, half8 (&bh)[CT], half8 (&bl)[CT], half8 (&nbh)[CT],
                     half8 (&nbl)[CT]) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(AQ) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      stage_b(c + 2);
      stage_a(c + 3);
      rd_b(c + 1, nbh, nbl);
      rd_a(c, 1, ah1, al1);
      tile(0, ah0, al0, bh, bl);
      rd_a(c, 2, ah0, al0);
      tile(1, ah1, al1, bh, bl);
      rd_a(c, 3, ah1, al1);
      tile(2, ah0, al0, bh, bl);
      rd_a(c + 1, 0, ah0, al0);
      tile(3, ah1, al1, bh, bl);
    };
#pragma unroll 1
    for (int c = 0; c + 1 < nch; c += 2) {
      chunk(c, bh0, bl0, bh1, bl1);
      chunk(c + 1, bh1, bl1, bh0, bl0);
    }
    if (nch & 1) chunk(nch - 1, bh0, bl0, bh1, bl1);
  } else {
  stage_b(0);
  stage_a(0);
  stage_a(1);
  stage_a(2);
  for (int c = 0; c < nch; ++c) {
    // chunk c landed: this wave's copies of B(c) and A(c) retired (only the
    // newest A chunk, AQ copies, may still be in flight; in the first
    // iteration A(1) and A(2) too), then every wave's, by the barrier; the
    // barrier also retires all reads of the buffers restaged below
    if (c == 0) {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    stage_b(c + 1);
    stage_a(c + 3);
    const _Float16* a = aring + (c & (kXAbuf - 1)) * kXAbufHalves;
    const _Float16* b = bring + (c & (kXBbuf - 1)) * BBUF;
    // the whole 32-deep chunk is one k-step: 8 A + 2 CT B fragment reads,
    // 12 CT MFMAs (ah bh + ah bl + al bh per 16x16 output tile)
    half8 ah[4], al[4], bh[CT], bl[CT];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr * 64 + i * 16 + lc;
      const int ao = row * kXK + ((lq ^ x3_swz(row)) * 8);
      ah[i] = *reinterpret_cast<const half8*>(a + ao);
      al[i] = *reinterpret_cast<const half8*>(a + kXM * kXK + ao);
    }
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int col = (wc * CT + t) * 16 + lc;
      const int bo = col * kXK + ((lq ^ x3_swz(col)) * 8);
      bh[t] = *reinterpret_cast<const half8*>(b + bo);
      bl[t] = *reinterpret_cast<const half8*>(b + LDW * kXK + bo);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[t], acc[i][t], 0, 0, 0);
        acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[t], acc[i][t], 0, 0, 0);
        acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[t], acc[i][t], 0, 0, 0);
      }
  }
  }  // PIPE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr ((DIAG & 1) != 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < CT; ++t) asm volatile("" ::"v"(acc[i][t]));
    return;
  }
  if constexpr (SPLIT) {  // the raw accumulators as rows [kXM][LDW] (16 lanes: 64 contiguous bytes)
    float* pw = reinterpret_cast<float*>(part) + static_cast<int64_t>(blockIdx.x) * kXM * LDW;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < CT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          pw[(wr * 64 + 16 * i + 4 * lq + j) * LDW + (wc * CT + t) * 16 + lc] = acc[i][t][j];
    return;
  }

  if constexpr (ROWEPI) {
    x3_row_epilogue<CT, 4>(acc, reinterpret_cast<float*>(lds), s_rs, kXM, wr, wc, lq, lc, wave, lane,
                           n0, N, D, num, aux, col_inv, c0, pc, out, sif);
    return;
  }
  // epilogue (as mm2_project_kernel): unscale, add weighted text sum + c0,
  // divide by the total weight (column D), L2-normalise the row.  Every load
  // is unconditional (row and column clamped in range, results selected
  // afterwards).  Lane value (i, t, j): row wr*64 + 16 i + 4 lq + j, column
  // (wc*CT + t)*16 + lc.
  {
    float nv[16][CT], tv[16], cv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = wr * 64 + (r >> 2) * 16 + lq * 4 + (r & 3);
      const int64_t rowc = min(n0 + rl, N - 1);
      tv[r] = aux[N + rowc];
      cv[r] = aux[rowc];
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        const int col = (wc * CT + t) * 16 + lc;
        nv[r][t] = num[rowc * D + min(col, D - 1)];
      }
    }
    float cadd[CT], cinv[CT];
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int col = (wc * CT + t) * 16 + lc;
      cinv[t] = col_inv[col];
      cadd[t] = c0[col];
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = wr * 64 + (r >> 2) * 16 + lq * 4 + (r & 3);
      const float inv_rs = s_rs[rl];
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        const int col = (wc * CT + t) * 16 + lc;
        const float add = col < D ? text_sum(nv[r][t], cv[r]) : (col == D ? tv[r] : 0.f);
        const float y = acc[r >> 2][t][r & 3] * (cinv[t] * inv_rs) + add + cadd[t];
        acc[r >> 2][t][r & 3] = y;
        if (col == D) s_tot[rl] = y;
      }
    }
  }
  __syncthreads();
  // one division per row: cs = y * (1 / total) (1 / 0 = inf keeps the
  // reference's NaN rows for a zero total)
  float ss[16], rt[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    ss[r] = 0.f;
    rt[r] = 1.f / s_tot[wr * 64 + (r >> 2) * 16 + lq * 4 + (r & 3)];
  }
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    const int col = (wc * CT + t) * 16 + lc;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float cs = acc[r >> 2][t][r & 3] * rt[r];
      acc[r >> 2][t][r & 3] = cs;
      if (col < D) ss[r] = fmaf(cs, cs, ss[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float v = row16_sum(ss[r]);  // the 16 lanes of a row
    if (lc == 0) s_ss[wc][wr * 64 + (r >> 2) * 16 + lq * 4 + (r & 3)] = v;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int rl = wr * 64 + (r >> 2) * 16 + lq * 4 + (r & 3);
    const int64_t row = n0 + rl;
    const float inv = 1.f / sqrtf((s_ss[0][rl] + s_ss[1][rl]) + (s_ss[2][rl] + s_ss[3][rl]));
    if (row < N) {
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        const int col = (wc * CT + t) * 16 + lc;
        if (col < D) out[row * D + col] = acc[r >> 2][t][r & 3] * inv;
      }
    }
  }

  if (pc) {
    // fused first-PC removal of the a2 rows (sif_functions.py:77-78, npc = 1):
    // sif = x - (x . pc) pc in f64, with the accumulators dead.  Wave w owns
    // rows w, w + 8, ... of the tile (4 at a time, every load issued first);
    // lane l columns l + 64 m.  The x rows come back from L2 / Infinity Cache
    // (this workgroup read them for the text sum above).
    constexpr int PER = (LDW + 63) / 64;
    double pcv[PER];
#pragma unroll
    for (int m = 0; m < PER; ++m) {
      const int col = lane + 64 * m;
      pcv[m] = col < D ? pc[col] : 0.0;
    }
    for (int g = wave; g < kXM; g += 4 * (kXT / 64)) {
      float xv[4][PER];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t rowc = min(n0 + g + q * (kXT / 64), N - 1);
#pragma unroll
        for (int m = 0; m < PER; ++m) xv[q][m] = num[rowc * D + min(lane + 64 * m, D - 1)];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = n0 + g + q * (kXT / 64);
        double dp = 0.0;
#pragma unroll
        for (int m = 0; m < PER; ++m) dp = fma(static_cast<double>(xv[q][m]), pcv[m], dp);
        const double dot = wave_sum_dpp(dp);
        if (row < N) {
#pragma unroll
          for (int m = 0; m < PER; ++m) {
            const int col = lane + 64 * m;
            if (col < D) sif[row * D + col] = static_cast<float>(static_cast<double>(xv[q][m]) - dot * pcv[m]);
          }
        }
      }
    }
  }
}



template <int CT>
constexpr size_t x3b_lds_bytes() { return x3_lds_bytes<CT>() + 2 * kXM * sizeof(float); }

// The split-K slices' rows, one wave per row (blockIdx.x * 4 + wave): the
// slices' raw accumulator rows [kXM][320] summed in slice order (every
// slice's two float4 columns of a lane in flight together), then the row-wise
// epilogue's arithmetic of x3_row_epilogue on the same lane columns (4 l..,
// 256 + 4 l..) in the same order -- so the fused PC removal's rows are the
// one-pass kernel's bit for bit and the MMB2 rows differ only by the K sum's
// f32 order.  (The 64-row pass of x3_row_epilogue itself ran ~23 us per 64
// rows on one workgroup: its staging barriers and dependent loads, which a
// full chip of tiles hides and two workgroups do not.)
constexpr int kXSplitMax = 16;  // slices the finish sums (the launcher's cap)
__global__ __launch_bounds__(256) void x3_splitk_rows_kernel(
    const float* __restrict__ part, int nsl, const float* __restrict__ num,
    const float* __restrict__ aux, const float* __restrict__ col_inv, const float* __restrict__ c0,
    int64_t N, int D, float* __restrict__ out, const double* __restrict__ pc, float* __restrict__ sif) {
  constexpr int LDW = 320;
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const int64_t tile = row / kXM;
  const int rl = static_cast<int>(row - tile * kXM);
  const int U = D >> 2;
  const bool u1 = lane + 64 < U;
  const int c0a = 4 * lane, c1a = 256 + 4 * min(lane, 15);
  const int c0x = 4 * min(lane, U - 1), c1x = 4 * min(lane + 64, U - 1);
  f32x4 v0[kXSplitMax], v1[kXSplitMax];
  const float* pr = part + (tile * nsl * kXM + rl) * LDW;
#pragma unroll
  for (int sl = 0; sl < kXSplitMax; ++sl) {
    const float* q = pr + static_cast<int64_t>(min(sl, nsl - 1)) * kXM * LDW;
    v0[sl] = *reinterpret_cast<const f32x4*>(q + c0a);
    v1[sl] = *reinterpret_cast<const f32x4*>(q + c1a);
  }
  const float4 xa = *reinterpret_cast<const float4*>(num + row * D + c0x);
  const float4 xb = *reinterpret_cast<const float4*>(num + row * D + c1x);
  const float cn = aux[row], tw = aux[N + row];
  const float irs = 1.f / aux[2 * N + row];
  const int cA = min(c0a, LDW - 4), cB = c1a;
  const float civ[8] = {col_inv[cA], col_inv[cA + 1], col_inv[cA + 2], col_inv[cA + 3],
                        col_inv[cB], col_inv[cB + 1], col_inv[cB + 2], col_inv[cB + 3]};
  const float cav[8] = {c0[cA], c0[cA + 1], c0[cA + 2], c0[cA + 3], c0[cB], c0[cB + 1], c0[cB + 2], c0[cB + 3]};
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int sl = 0; sl < kXSplitMax; ++sl) {
    if (sl < nsl) {
      s0 += v0[sl];
      s1 += v1[sl];
    }
  }
  const float av[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  const float xv[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
  float y[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int col = (e < 4 ? c0a : 256 + 4 * lane) + (e & 3);
    const bool in = e < 4 ? lane < U : u1;
    const float add = (in && col < D) ? text_sum(xv[e], cn) : (col == D ? tw : 0.f);
    y[e] = av[e] * (civ[e] * irs) + add + cav[e];
  }
  const int lane_tot = (D - 256) >> 2, e_tot = (D - 256) & 3;  // column D in unit 1
  const float ysel = e_tot == 0 ? y[4] : e_tot == 1 ? y[5] : e_tot == 2 ? y[6] : y[7];
  const float tot = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ysel), lane_tot));
  const float rt = 1.f / tot;
  float ss = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const bool in = e < 4 ? lane < U : u1;
    y[e] *= rt;
    if (in) ss = fmaf(y[e], y[e], ss);
  }
  const float inv = 1.f / sqrtf(wave_sum_dpp_f32(ss));
  float* orow = out + row * D;
  if (lane < U) *reinterpret_cast<float4*>(orow + c0x) = make_float4(y[0] * inv, y[1] * inv, y[2] * inv, y[3] * inv);
  if (u1) *reinterpret_cast<float4*>(orow + c1x) = make_float4(y[4] * inv, y[5] * inv, y[6] * inv, y[7] * inv);
  if (pc) {
    double pv[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      pv[e] = lane < U ? pc[c0x + e] : 0.0;
      pv[4 + e] = u1 ? pc[c1x + e] : 0.0;
    }
    double dot = 0.0;
#pragma unroll
    for (int e = 0; e < 8; ++e) dot = fma(static_cast<double>(xv[e]), pv[e], dot);
    dot = wave_sum_dpp(dot);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = static_cast<float>(static_cast<double>(xv[e]) - dot * pv[e]);
    float* srow = sif + row * D;
    if (lane < U) *reinterpret_cast<float4*>(srow + c0x) = make_float4(o[0], o[1], o[2], o[3]);
    if (u1) *reinterpret_cast<float4*>(srow + c1x) = make_float4(o[4], o[5], o[6], o[7]);
  }
}

// Projection kernel variant: 0 = 32x32x16 MFMA tiles (wave = 32 rows x 32 CT
// columns), 1 = 16x16x32 tiles (wave = 64 rows x 16 CT columns: 18 instead of
// 24 fragment reads per chunk), 2 = the 16x16x32 kernel with the
// software-pipelined K loop.  MMB_PROJ_VARIANT overrides (read once).
// Row-wise projection epilogue (1, default) or the MFMA-tile-layout one (0);
// MMB_PROJ_ROWEPI overrides (tools build, read per launch).

// The product dispatch: the 16x16x32 kernel with the software-pipelined K
// loop (variant 2), row-wise epilogue where the shape allows it.
template <int CT>
static int launch_project_x3(const _Float16* s, const float* num, const float* aux,
                             const _Float16* img, const float* ci, const float* c0, int64_t n,
                             int kp, int d, float* out, const double* pc, float* sif,
                             hipStream_t stream) {
#ifndef MMB_HOOK_PROJECT_X3  // (tools/diag: the MMB_PROJ_* variants and ablations)
#define MMB_HOOK_PROJECT_X3(rc) false
#endif
  {
    int rc_ = MMB_OK;
    if (MMB_HOOK_PROJECT_X3(rc_)) return rc_;
  }
  const int grid = static_cast<int>(ceil_div(n, kXM));
  constexpr size_t ldsb = x3b_lds_bytes<CT>();
  static_assert(ldsb <= 160 * 1024, "x3b chunk rings exceed LDS");
  static bool attr_b = false;
  if (!attr_b) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mm2_project_x3b_kernel<CT, false, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(ldsb));
    if constexpr (CT == 5)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mm2_project_x3b_kernel<CT, true, true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(ldsb));
    attr_b = true;
  }
  auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  // the row-wise epilogue: D in [256, 320) (column D in a lane's second
  // unit), whole float4 units, 16-byte aligned rows
  const bool rowepi = d >= 256 && d % 4 == 0 && a16(num) && a16(out) && (sif == nullptr || a16(sif));
  if constexpr (CT == 5) {
    if (rowepi) {
      mm2_project_x3b_kernel<CT, true, true><<<grid, kXT, ldsb, stream>>>(s, num, aux, img, ci, c0,
                                                                          n, kp, d, out, pc, sif);
      MMB_LAUNCH_CHECK();
      return MMB_OK;
    }
  }
  mm2_project_x3b_kernel<CT, false, true><<<grid, kXT, ldsb, stream>>>(s, num, aux, img, ci, c0,
                                                                       n, kp, d, out, pc, sif);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

template <int CT>
static int launch_project(const float* s, const float* num, const float* aux, const float* wm,
                          const float* c0, int64_t n, int kp, int d, float* out,
                          hipStream_t stream) {
  const int grid = static_cast<int>(ceil_div(n, kPM));
  mm2_project_kernel<CT><<<grid, 256, 0, stream>>>(s, num, aux, wm, c0, n, kp, d, out);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

}  // namespace mmb

using namespace mmb;

extern "C" int mmb_mm2_ldw(int d) { return (d + 1 + 63) / 64 * 64; }

extern "C" size_t mmb_mm2_split_bytes(int d, int a, int vd) {
  const size_t ldw = mmb_mm2_ldw(d), kp = mmb_mm2_k(d, a, vd);
  return 2 * ldw * kp * sizeof(_Float16) + ldw * sizeof(float);
}

extern "C" int mmb_mm2_prepare(const float* const* w_mu, const float* const* b_mu,
                               const float* const* w_ls, const float* const* b_ls, int d, int a,
                               int vd, int t, float* wm, int ldw, float* c0, void* wsplit,
                               hipStream_t stream) {
  MMB_REQUIRE(w_mu && b_mu && w_ls && b_ls && wm && c0 && d > 0 && a > 0 && vd > 0 && t > 0);
  MMB_REQUIRE(ldw == mmb_mm2_ldw(d));
  PrepArgs p{};
  for (int k = 0; k < 6; ++k) {
    MMB_REQUIRE(w_mu[k] && b_mu[k] && w_ls[k] && b_ls[k]);
    p.wmu[k] = w_mu[k];
    p.bmu[k] = b_mu[k];
    p.wls[k] = w_ls[k];
    p.bls[k] = b_ls[k];
  }
  p.D = d; p.A = a; p.Vd = vd; p.T = t; p.ldw = ldw; p.Kp = mmb_mm2_k(d, a, vd);
  p.wm = wm; p.c0 = c0;
  const int64_t total = static_cast<int64_t>(p.Kp) * ldw;
  mm2_prepare_wm_kernel<<<static_cast<int>(std::min<int64_t>(ceil_div(total, 256), 4096)), 256, 0, stream>>>(p);
  MMB_LAUNCH_CHECK();
  if (wsplit && p.Kp >= 128) {
    // the split image is written last: its memory is the c0 partials' scratch
    // (kC0Splits x ldw doubles <= 2 x ldw x Kp halves for every Kp >= 128)
    double* part = static_cast<double*>(wsplit);
    mm2_prepare_c0_part_kernel<<<dim3(ldw / 64, kC0Splits), 1024, 0, stream>>>(p, part);
    MMB_LAUNCH_CHECK();
    mm2_c0_reduce_kernel<<<static_cast<int>(ceil_div(ldw, 256)), 256, 0, stream>>>(part, d, ldw, t, c0);
    MMB_LAUNCH_CHECK();
  } else {
    mm2_prepare_c0_kernel<<<ldw / 64, 1024, 0, stream>>>(p);
    MMB_LAUNCH_CHECK();
  }
  if (wsplit) {
    _Float16* img = static_cast<_Float16*>(wsplit);
    float* ci = reinterpret_cast<float*>(img + 2 * static_cast<size_t>(ldw) * p.Kp);
    mm2_split_wm_kernel<<<ldw, 256, 0, stream>>>(wm, p.Kp, ldw, img, ci);
    MMB_LAUNCH_CHECK();
  }
  return MMB_OK;
}

extern "C" int mmb_mm2_project_x3_rmpc(const void* s_split, const float* num, const float* aux,
                                       const void* wsplit, int ldw, const float* c0, int64_t n,
                                       int k, int d, float* out, const double* pc, float* sif_out,
                                       hipStream_t stream) {
  MMB_REQUIRE(s_split && num && aux && wsplit && c0 && out && n >= 0 && d > 0);
  MMB_REQUIRE(ldw == mmb_mm2_ldw(d) && k % 32 == 0 && k >= 32);
  MMB_REQUIRE((pc == nullptr) == (sif_out == nullptr));
  MMB_REQUIRE((reinterpret_cast<uintptr_t>(s_split) & 15) == 0 &&
              (reinterpret_cast<uintptr_t>(wsplit) & 15) == 0);
  if (n == 0) return MMB_OK;
  const _Float16* s = static_cast<const _Float16*>(s_split);
  const _Float16* img = static_cast<const _Float16*>(wsplit);
  const float* ci = reinterpret_cast<const float*>(img + 2 * static_cast<size_t>(ldw) * k);
  switch (ldw / 64) {
    case 1: return launch_project_x3<1>(s, num, aux, img, ci, c0, n, k, d, out, pc, sif_out, stream);
    case 2: return launch_project_x3<2>(s, num, aux, img, ci, c0, n, k, d, out, pc, sif_out, stream);
    case 3: return launch_project_x3<3>(s, num, aux, img, ci, c0, n, k, d, out, pc, sif_out, stream);
    case 4: return launch_project_x3<4>(s, num, aux, img, ci, c0, n, k, d, out, pc, sif_out, stream);
    case 5: return launch_project_x3<5>(s, num, aux, img, ci, c0, n, k, d, out, pc, sif_out, stream);
    default: return MMB_EINVAL;  // d >= 320: the chunk rings exceed the 160 KB LDS
  }
}

// split-K plan of the x3 projection for a few rows (r06): about one
// workgroup per 4 CUs in all, at least 4 chunks per slice; 1 = no split
// (the row tiles alone fill the chip, or K is short).  Only the row-wise
// epilogue's shapes (ldw = 320, 256 <= d < 320) split.
static int x3_split_slices(int64_t n, int k, int cus) {
  const int64_t tiles = ceil_div(n, kXM);
  const int nch = k / kXK;
  const int64_t want = cus / (4 * std::max<int64_t>(1, tiles));
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>({want, nch / 4, kXSplitMax})));
}

extern "C" int mmb_mm2_project_x3_split_slices(int64_t n, int k) {
  return x3_split_slices(n, k, stream_cu_count(nullptr));
}

extern "C" size_t mmb_mm2_project_x3_split_ws_bytes(int64_t n, int k, int slices) {
  if (n <= 0 || k < kXK) return 0;
  const int nsl = slices > 0 ? slices : mmb_mm2_project_x3_split_slices(n, k);
  return static_cast<size_t>(ceil_div(n, kXM)) * nsl * kXM * 320 * sizeof(float);
}

extern "C" int mmb_mm2_project_x3_split(const void* s_split, const float* num, const float* aux,
                                        const void* wsplit, int ldw, const float* c0, int64_t n,
                                        int k, int d, float* out, const double* pc, float* sif_out,
                                        int slices, void* ws, size_t ws_bytes, hipStream_t stream) {
  MMB_REQUIRE(slices >= 0);
  const int nsl = slices > 0 ? std::min({slices, std::max(1, k / kXK), kXSplitMax})
                             : mmb_mm2_project_x3_split_slices(n, k);
  auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const bool rowepi = ldw == 320 && ldw == mmb_mm2_ldw(d) && d >= 256 && d % 4 == 0 && a16(num) &&
                      a16(out) && (sif_out == nullptr || a16(sif_out));
  if (nsl < 2 || !rowepi || n <= 0)  // nothing to split: the one-pass kernel
    return mmb_mm2_project_x3_rmpc(s_split, num, aux, wsplit, ldw, c0, n, k, d, out, pc, sif_out, stream);
  MMB_REQUIRE(s_split && num && aux && wsplit && c0 && out && k % 32 == 0 && k >= 32);
  MMB_REQUIRE((pc == nullptr) == (sif_out == nullptr));
  MMB_REQUIRE(a16(s_split) && a16(wsplit) && a16(ws));
  const int64_t tiles = ceil_div(n, kXM);
  MMB_REQUIRE(ws && ws_bytes >= static_cast<size_t>(tiles) * nsl * kXM * 320 * sizeof(float));
  MMB_REQUIRE(tiles * nsl <= (int64_t{1} << 31) - 1);
  const _Float16* s = static_cast<const _Float16*>(s_split);
  const _Float16* img = static_cast<const _Float16*>(wsplit);
  const float* ci = reinterpret_cast<const float*>(img + 2 * static_cast<size_t>(ldw) * k);
  constexpr size_t ldsb = x3b_lds_bytes<5>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mm2_project_x3b_kernel<5, true, true, 0, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(ldsb));
    attr = true;
  }
  const int cps = static_cast<int>(ceil_div(k / kXK, nsl));  // chunks per slice
  const int nse = static_cast<int>(ceil_div(k / kXK, cps));   // slices holding >= 1 chunk (<= nsl)
  f32x4* part = static_cast<f32x4*>(ws);
  mm2_project_x3b_kernel<5, true, true, 0, true><<<static_cast<unsigned>(tiles * nse), kXT, ldsb, stream>>>(
      s, num, aux, img, ci, c0, n, k, d, out, pc, sif_out, nse, cps, part);
  MMB_LAUNCH_CHECK();
  x3_splitk_rows_kernel<<<static_cast<unsigned>(ceil_div(n, 4)), 256, 0, stream>>>(
      reinterpret_cast<const float*>(part), nse, num, aux, ci, c0, n, d, out, pc, sif_out);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_mm2_project_x3(const void* s_split, const float* num, const float* aux,
                                  const void* wsplit, int ldw, const float* c0, int64_t n, int k,
                                  int d, float* out, hipStream_t stream) {
  return mmb_mm2_project_x3_rmpc(s_split, num, aux, wsplit, ldw, c0, n, k, d, out, nullptr,
                                 nullptr, stream);
}

extern "C" int mmb_mm2_project(const float* s, const float* num, const float* aux,
                               const float* wm, int ldw, const float* c0, int64_t n, int k,
                               int d, float* out, hipStream_t stream) {
  MMB_REQUIRE(s && num && aux && wm && c0 && out && n >= 0 && d > 0);
  MMB_REQUIRE(ldw == mmb_mm2_ldw(d) && k % 32 == 0);
  if (n == 0) return MMB_OK;
  switch (ldw / 64) {
    case 1: return launch_project<1>(s, num, aux, wm, c0, n, k, d, out, stream);
    case 2: return launch_project<2>(s, num, aux, wm, c0, n, k, d, out, stream);
    case 3: return launch_project<3>(s, num, aux, wm, c0, n, k, d, out, stream);
    case 4: return launch_project<4>(s, num, aux, wm, c0, n, k, d, out, stream);
    case 5: return launch_project<5>(s, num, aux, wm, c0, n, k, d, out, stream);
    case 6: return launch_project<6>(s, num, aux, wm, c0, n, k, d, out, stream);
    default: return MMB_EINVAL;
  }
}

static int mm2_pieces_k(int d, int a, int vd) {
  auto q = [](int w) { return (2 * w + 31) / 32 * 32; };
  return q(d) + q(a) + q(vd);
}

extern "C" size_t mmb_mm2_split_pieces_bytes(int d, int a, int vd) {
  const size_t ldw = mmb_mm2_ldw(d), kq = mm2_pieces_k(d, a, vd);
  return 2 * ldw * kq * sizeof(_Float16) + ldw * sizeof(float);
}

extern "C" int mmb_mm2_split_pieces(const float* wm, int d, int a, int vd, int ldw, void* img,
                                    hipStream_t stream) {
  MMB_REQUIRE(wm && img && d > 0 && a > 0 && vd > 0 && ldw == mmb_mm2_ldw(d));
  _Float16* im = static_cast<_Float16*>(img);
  float* ci = reinterpret_cast<float*>(im + 2 * static_cast<size_t>(ldw) * mm2_pieces_k(d, a, vd));
  mm2_split_wm_pieces_kernel<<<ldw, 256, 0, stream>>>(wm, ldw, d, a, vd, im, ci);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

namespace mmb {

// ------------------------------------------------------------------ text cache (r04)
// The MOSI-width fused step (mmb_mm2_stream_project_narrow) projects the text
// sums per vocabulary row instead of per utterance: the text rows of Wm enter
// the MMB2 numerator only through sum_t E_t Wm_text1 + sum_t E_t^2 Wm_text2 =
// sum_t P[id_t] with
//   P[v][j] = sum_f E[v][f] Wm[f][j] + E[v][f]^2 Wm[D + f][j]     (j <= D)
// (exact algebra; column D carries the total weight), so an utterance gathers
// one P row per token beside its table row, and the per-utterance GEMM shrinks
// to the audio / visual sums (K = 2 (A + Vd) instead of 2 (D + A + Vd)).  P is
// computed in f64 and rounded once.  The cache also ranks the words by weight:
// the kTextHot smallest SIF weights a / (a + p(w)) are the most frequent words
// (the pad id 0 too where its weight is 0), whose E and P rows the fused
// kernel keeps in LDS.
//   cache layout: rows [v][kTextLdq] f32 = E[v][0, d) | P[v][0, d] | 0 pad
//   (the word's table row and its projection side by side: one token, one
//   contiguous 2d + 4 floats) | hot_slot1 [v] int32 (slot + 1, 0 = not hot) |
//   hot_ids [kTextHot] int32 | w [v] f32 (a copy of the weights: the fused
//   kernel reads all of it through one buffer descriptor)
constexpr int kTextLdp = 304;   // P columns kept (d + 1 <= 304)
constexpr int kTextLdq = 608;   // cache row stride (floats): 2 d + 4 <= 608, 16-byte rows
constexpr int kTextHot = 32;    // words whose rows live in LDS
constexpr int64_t kTextMaxV = 16384;

__global__ __launch_bounds__(320) void mm2_text_table_kernel(const float* __restrict__ E, int D,
                                                             const float* __restrict__ wm, int ldw,
                                                             float* __restrict__ rows) {
  __shared__ double se[kTextLdp], se2[kTextLdp];
  const int64_t v = blockIdx.x;
  for (int f = threadIdx.x; f < D; f += blockDim.x) {
    const double e = E[v * D + f];
    se[f] = e;
    se2[f] = e * e;
  }
  __syncthreads();
  float* row = rows + v * kTextLdq;
  for (int f = threadIdx.x; f < D; f += blockDim.x) row[f] = E[v * D + f];
  for (int j = threadIdx.x; j + D < kTextLdq; j += blockDim.x) {
    double acc = 0.0;
    if (j <= D) {
      for (int f = 0; f < D; ++f) {
        acc = fma(se[f], static_cast<double>(wm[static_cast<int64_t>(f) * ldw + j]), acc);
        acc = fma(se2[f], static_cast<double>(wm[static_cast<int64_t>(D + f) * ldw + j]), acc);
      }
    }
    row[D + j] = static_cast<float>(acc);
  }
}

// rank of each word among the weights (ascending; ties: lower id first):
// hot_slot1[v] = rank + 1 for the k smallest, else 0; hot_ids[rank] = v
__global__ __launch_bounds__(1024) void text_hot_kernel(const float* __restrict__ wtab, int V, int k,
                                                        int32_t* __restrict__ hot_slot1,
                                                        int32_t* __restrict__ hot_ids,
                                                        float* __restrict__ wcopy) {
  __shared__ float sw[1024];
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  const float wv = v < V ? wtab[v] : 0.f;
  int rank = 0;
  for (int u0 = 0; u0 < V; u0 += 1024) {
    __syncthreads();
    if (u0 + static_cast<int>(threadIdx.x) < V) sw[threadIdx.x] = wtab[u0 + threadIdx.x];
    __syncthreads();
    const int n = min(1024, V - u0);
    for (int j = 0; j < n; ++j) {
      const float wu = sw[j];
      rank += (wu < wv || (wu == wv && u0 + j < v)) ? 1 : 0;
    }
  }
  if (v < V) {
    hot_slot1[v] = rank < k ? rank + 1 : 0;
    if (rank < k) hot_ids[rank] = v;
    wcopy[v] = wv;
  }
}

}  // namespace mmb

extern "C" size_t mmb_mm2_text_cache_bytes(int64_t v, int d) {
  (void)d;
  return sizeof(float) * static_cast<size_t>(v) * (kTextLdq + 1) + sizeof(int32_t) * (v + kTextHot);
}

extern "C" int mmb_mm2_text_cache(const float* table, int64_t v, int d, const float* wtab32,
                                  const float* wm, int ldw, void* cache, hipStream_t stream) {
  MMB_REQUIRE(table && wtab32 && wm && cache && v > 0 && v <= kTextMaxV);
  MMB_REQUIRE(d > 0 && d % 4 == 0 && d + 1 <= kTextLdp && ldw > d &&
              (reinterpret_cast<uintptr_t>(cache) & 15) == 0);
  float* ptab = static_cast<float*>(cache);
  int32_t* hot_slot1 = reinterpret_cast<int32_t*>(ptab + static_cast<size_t>(v) * kTextLdq);
  int32_t* hot_ids = hot_slot1 + v;
  float* wcopy = reinterpret_cast<float*>(hot_ids + kTextHot);
  mm2_text_table_kernel<<<static_cast<unsigned>(v), 320, 0, stream>>>(table, d, wm, ldw, ptab);
  MMB_LAUNCH_CHECK();
  text_hot_kernel<<<static_cast<unsigned>(ceil_div(v, 1024)), 1024, 0, stream>>>(
      wtab32, static_cast<int>(v), static_cast<int>(std::min<int64_t>(v, kTextHot)), hot_slot1, hot_ids,
      wcopy);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

// the tools build's projection variants, launches and knobs (tools/diag/);
// the product library includes an empty header here
#ifndef MMB_TOOLS_TAIL_MM2
#define MMB_TOOLS_TAIL_MM2 "mmb_no_tools.h"
#endif
#include MMB_TOOLS_TAIL_MM2
