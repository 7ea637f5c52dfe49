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
        if (col < D) add = num[row * D + col] + c0[col];
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
using half8 = __attribute__((ext_vector_type(8))) _Float16;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using half4 = __attribute__((ext_vector_type(4))) _Float16;

constexpr int kXM = 128;  // rows per workgroup (8 waves: 4 row tiles x 2 column halves)
constexpr int kXK = 32;   // K chunk (2 MFMA k-steps)
constexpr int kXS = kXK + 8;  // padded LDS row (halves)

__global__ void mm2_split_wm_kernel(const float* __restrict__ wm, int Kp, int ldw,
                                    _Float16* __restrict__ wth, _Float16* __restrict__ wtl,
                                    float* __restrict__ col_inv) {
  // one workgroup per column j: max |Wm[:, j]| -> scale, then the transposed
  // hi/lo planes Wt[j][k] (K contiguous, the B-fragment order)
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
    wth[static_cast<int64_t>(j) * Kp + k] = h;
    wtl[static_cast<int64_t>(j) * Kp + k] = static_cast<_Float16>(v - static_cast<float>(h));
  }
  if (tid == 0) col_inv[j] = 1.f / sc;
}

// LDS image of one K chunk: A hi, A lo [kXM][kXS], B hi, B lo [LDW][kXS]
// halves; each lo plane sits 32 halves past its hi plane's end so the hi and
// lo 16-byte stores of one 8-lane group land on disjoint banks
constexpr int kXPad = 32;
template <int CT>
constexpr int x3_buf_halves() { return 2 * (kXM * kXS + kXPad) + 2 * (64 * CT * kXS + kXPad); }
template <int CT>
constexpr size_t x3_lds_bytes() {
  return 2 * x3_buf_halves<CT>() * sizeof(_Float16) + 4 * kXM * sizeof(float);
}
// MR = 32-row MFMA tiles per wave: the 128 x LDW block is split over
// (4 / MR) x 2 waves, each owning MR x CT tiles of 32 x 32
template <int MR>
constexpr int x3_threads() { return 64 * 2 * (4 / MR); }

template <int CT, int MR>
__global__ __launch_bounds__(x3_threads<MR>()) void mm2_project_x3_kernel(
    const float* __restrict__ S, const float* __restrict__ num, const float* __restrict__ aux,
    const _Float16* __restrict__ wth, const _Float16* __restrict__ wtl,
    const float* __restrict__ col_inv, const float* __restrict__ c0, int64_t N, int Kp, int D,
    float* __restrict__ out) {
  constexpr int LDW = 64 * CT;
  constexpr int BUF = x3_buf_halves<CT>();
  constexpr int kXT = x3_threads<MR>();
  constexpr int AQ = kXM * 8 / kXT;   // float4 A pieces per thread per chunk
  constexpr int BQ = LDW * 8 / kXT;   // 16-byte B pieces per thread per chunk
  constexpr int OA = 0, OAL = kXM * kXS + kXPad;
  constexpr int OB = 2 * OAL, OBL = OB + LDW * kXS + kXPad;
  // one dynamic LDS array: two chunk buffers, then the per-row scalars
  extern __shared__ __attribute__((aligned(16))) _Float16 lds[];
  float* s_rs = reinterpret_cast<float*>(lds + 2 * BUF);
  float* s_tot = s_rs + kXM;
  float(*s_ss)[kXM] = reinterpret_cast<float(*)[kXM]>(s_tot + kXM);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;  // rows wr*32*MR + [0,32*MR), tiles wc*CT + [0,CT)
  const int hl = lane >> 5, cl = lane & 31;
  const int64_t n0 = static_cast<int64_t>(blockIdx.x) * kXM;
  const float* rscale = aux + 2 * N;

  if (tid < kXM) s_rs[tid] = (n0 + tid < N) ? rscale[n0 + tid] : 1.f;
  __syncthreads();

  f32x16 acc[MR][CT];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][t][r] = 0.f;

  // Software pipeline over K chunks of kXK, two LDS buffers, one barrier per
  // chunk.  Iteration c: the fragments of both k-steps of chunk c are read
  // from buffer c&1 up front, the first k-step's MFMAs run while the
  // registers holding chunk c+1 are converted and stored into the other
  // buffer and the global loads of B(c+2) and A(c+3) are issued, then the
  // second k-step's MFMAs.  A (the s rows, streamed once from HBM) is
  // prefetched through a ring of two register sets, B (the split weights,
  // L2-resident) through one.  Loads are unconditional (rows clamped to N-1,
  // chunks past the end re-read the last) so no load is branched around; A
  // loads are non-temporal to spare L2 for B.
  f32x4 pa0[AQ], pa1[AQ];
  u32x4 pb[BQ];
  const float* arow[AQ];
  const _Float16* bcol[BQ];
#pragma unroll
  for (int q = 0; q < AQ; ++q) {
    const int idx = tid + kXT * q;
    const int64_t row = min(n0 + (idx >> 3), N - 1);
    arow[q] = S + row * Kp + (idx & 7) * 4;
  }
#pragma unroll
  for (int q = 0; q < BQ; ++q) {
    const int idx = tid + kXT * q;
    const int col = idx >> 3, part = idx & 7;
    bcol[q] = ((part >> 2) ? wtl : wth) + static_cast<int64_t>(col) * Kp + (part & 3) * 8;
  }
  const int nch = Kp / kXK;
  auto load_a = [&](f32x4(&pa)[AQ], int c) {
    const int k = min(c, nch - 1) * kXK;
#pragma unroll
    for (int q = 0; q < AQ; ++q)
      pa[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(arow[q] + k));
  };
  auto load_b = [&](int c) {
    const int k = min(c, nch - 1) * kXK;
#pragma unroll
    for (int q = 0; q < BQ; ++q) pb[q] = *reinterpret_cast<const u32x4*>(bcol[q] + k);
  };
  auto stage = [&](const f32x4(&pa)[AQ], _Float16* buf) {
    // A: 128 rows x 32 fp32 -> row-scaled fp16 hi/lo
#pragma unroll
    for (int q = 0; q < AQ; ++q) {
      const int idx = tid + kXT * q;
      const int row = idx >> 3, c4 = idx & 7;
      const float sc = s_rs[row];
      half4 h, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = pa[q][e] * sc;
        h[e] = static_cast<_Float16>(x);
        l[e] = static_cast<_Float16>(x - static_cast<float>(h[e]));
      }
      *reinterpret_cast<half4*>(buf + OA + row * kXS + c4 * 4) = h;
      *reinterpret_cast<half4*>(buf + OAL + row * kXS + c4 * 4) = l;
    }
    // B: LDW columns x 32 halves per plane = 4 x 16 B per column per plane
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
      const int idx = tid + kXT * q;
      const int col = idx >> 3, part = idx & 7;
      *reinterpret_cast<u32x4*>(buf + ((part >> 2) ? OBL : OB) + col * kXS + (part & 3) * 8) =
          pb[q];
    }
  };
  struct Frag {
    half8 ah[MR], al[MR], bh[CT], bl[CT];
  };
  auto read_frag = [&](const _Float16* buf, int s, Frag& f) {
    const int ko = 16 * s + 8 * hl;
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int row = (wr * MR + i) * 32 + cl;
      f.ah[i] = *reinterpret_cast<const half8*>(buf + OA + row * kXS + ko);
      f.al[i] = *reinterpret_cast<const half8*>(buf + OAL + row * kXS + ko);
    }
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int col = (wc * CT + t) * 32 + cl;
      f.bh[t] = *reinterpret_cast<const half8*>(buf + OB + col * kXS + ko);
      f.bl[t] = *reinterpret_cast<const half8*>(buf + OBL + col * kXS + ko);
    }
  };
  auto mfma = [&](const Frag& f) {
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.ah[i], f.bh[t], acc[i][t], 0, 0, 0);
        acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.ah[i], f.bl[t], acc[i][t], 0, 0, 0);
        acc[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.al[i], f.bh[t], acc[i][t], 0, 0, 0);
      }
  };
  // iteration c: buffer `cur` holds chunk c, `nxt` holds A(c+1) (pb holds
  // B(c+1)), the other ring set holds A(c+2) in flight
  auto iter = [&](int c, f32x4(&nxt)[AQ], const _Float16* cur, _Float16* oth) {
    Frag f0, f1;
    read_frag(cur, 0, f0);
    read_frag(cur, 1, f1);
    mfma(f0);
    stage(nxt, oth);
    load_b(c + 2);
    load_a(nxt, c + 3);
    mfma(f1);
    __syncthreads();
  };
  _Float16* buf0 = lds;
  _Float16* buf1 = lds + BUF;
  load_a(pa0, 0);
  load_b(0);
  load_a(pa1, 1);
  stage(pa0, buf0);
  load_b(1);
  load_a(pa0, 2);
  __syncthreads();
  int c = 0;
  for (; c + 1 < nch; c += 2) {
    iter(c, pa1, buf0, buf1);
    iter(c + 1, pa0, buf1, buf0);
  }
  if (c < nch) iter(c, pa1, buf0, buf1);

  // epilogue (as mm2_project_kernel): unscale, add weighted text sum + c0,
  // divide by the total weight (column D), L2-normalise the row
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    const int col = (wc * CT + t) * 32 + cl;
    const float ci = col_inv[col];
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = (wr * MR + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const int64_t row = n0 + rl;
        float y = acc[i][t][r] * (ci / s_rs[rl]);
        if (row < N) {
          if (col < D) y += num[row * D + col] + c0[col];
          else if (col == D) y += aux[N + row] + c0[D];
        }
        acc[i][t][r] = y;
        if (col == D) s_tot[rl] = y;
      }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    float ss[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) ss[r] = 0.f;
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int col = (wc * CT + t) * 32 + cl;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = (wr * MR + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const float cs = acc[i][t][r] / s_tot[rl];
        acc[i][t][r] = cs;
        if (col < D) ss[r] = fmaf(cs, cs, ss[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float sum = half_sum(ss[r]);
      if (cl == 0) s_ss[wc][(wr * MR + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl] = sum;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = (wr * MR + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
      const int64_t row = n0 + rl;
      const float inv = 1.f / sqrtf(s_ss[0][rl] + s_ss[1][rl]);
      if (row < N) {
#pragma unroll
        for (int t = 0; t < CT; ++t) {
          const int col = (wc * CT + t) * 32 + cl;
          if (col < D) out[row * D + col] = acc[i][t][r] * inv;
        }
      }
    }
}

template <int CT, int MR = 1>
static int launch_project_x3(const float* s, const float* num, const float* aux,
                             const _Float16* wth, const _Float16* wtl, const float* ci,
                             const float* c0, int64_t n, int kp, int d, float* out,
                             hipStream_t stream) {
  const int grid = static_cast<int>(ceil_div(n, kXM));
  constexpr size_t lds = x3_lds_bytes<CT>();
  static_assert(lds <= 160 * 1024, "x3 chunk buffers exceed LDS");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&mm2_project_x3_kernel<CT, MR>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    attr = true;
  }
  mm2_project_x3_kernel<CT, MR><<<grid, x3_threads<MR>(), lds, stream>>>(s, num, aux, wth, wtl, ci,
                                                                        c0, n, kp, d, out);
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
  mm2_prepare_c0_kernel<<<ldw / 64, 1024, 0, stream>>>(p);
  MMB_LAUNCH_CHECK();
  if (wsplit) {
    _Float16* wth = static_cast<_Float16*>(wsplit);
    _Float16* wtl = wth + static_cast<size_t>(ldw) * p.Kp;
    float* ci = reinterpret_cast<float*>(wtl + static_cast<size_t>(ldw) * p.Kp);
    mm2_split_wm_kernel<<<ldw, 256, 0, stream>>>(wm, p.Kp, ldw, wth, wtl, ci);
    MMB_LAUNCH_CHECK();
  }
  return MMB_OK;
}

extern "C" int mmb_mm2_project_x3(const float* s, const float* num, const float* aux,
                                  const void* wsplit, int ldw, const float* c0, int64_t n, int k,
                                  int d, float* out, hipStream_t stream) {
  MMB_REQUIRE(s && num && aux && wsplit && c0 && out && n >= 0 && d > 0);
  MMB_REQUIRE(ldw == mmb_mm2_ldw(d) && k % 32 == 0);
  MMB_REQUIRE((reinterpret_cast<uintptr_t>(s) & 15) == 0 && (reinterpret_cast<uintptr_t>(wsplit) & 15) == 0);
  if (n == 0) return MMB_OK;
  const _Float16* wth = static_cast<const _Float16*>(wsplit);
  const _Float16* wtl = wth + static_cast<size_t>(ldw) * k;
  const float* ci = reinterpret_cast<const float*>(wtl + static_cast<size_t>(ldw) * k);
  switch (ldw / 64) {
    case 1: return launch_project_x3<1>(s, num, aux, wth, wtl, ci, c0, n, k, d, out, stream);
    case 2: return launch_project_x3<2>(s, num, aux, wth, wtl, ci, c0, n, k, d, out, stream);
    case 3: return launch_project_x3<3>(s, num, aux, wth, wtl, ci, c0, n, k, d, out, stream);
    case 4: return launch_project_x3<4>(s, num, aux, wth, wtl, ci, c0, n, k, d, out, stream);
    case 5: return launch_project_x3<5>(s, num, aux, wth, wtl, ci, c0, n, k, d, out, stream);
    default: return MMB_EINVAL;  // d >= 320: two chunk buffers exceed the 160 KB LDS
  }
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
