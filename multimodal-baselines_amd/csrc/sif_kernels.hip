// SIF word-weight gather (a1), weighted gather-reduce (a2) and the fused
// text+audio+visual per-utterance sums of the closed-form MMB2 (a6/a7/a8 stream).
//
// Design (MI355X): one workgroup of 320 threads (5 waves) owns one utterance at
// a time (grid-stride over utterances).  A 300-wide f32 row is 75 float4 column
// units; 4 row slots x 75 units = 300 active lanes, so every wave-instruction
// issues 16 B/lane loads that cover contiguous 1 KiB runs of a frame row or a
// gathered table row.  The utterance's token ids and weights are staged in LDS
// (broadcast reads), the per-slot partial sums are combined through one LDS
// image per accumulator in a fixed order (deterministic), and only the
// reductions leave the chip: the [N,L,300] gathered text tensor the reference
// materialises (simplesif.py:319-340, :871) never exists.
#include <cstdlib>

#include "mmb_common.h"

namespace mmb {

constexpr int kNT = 320;              // threads per utterance workgroup
constexpr int kTokChunk = 512;        // tokens staged per LDS chunk
constexpr int kRedFloats = kNT * 4;   // one accumulator image: R*F <= NT*VEC

struct StreamArgs {
  const int32_t* ids;
  const float* table;
  int64_t V;
  const float* wtab;        // f32 weight table (gather mode without w_dense)
  const float* w_dense;     // [N,L] given weights
  const float* text_dense;  // [N,L,D] dense text frames (MMB2 drop-in mode)
  const float* emb_dense;   // [N,L,D] rows for the weighted sum (may alias text_dense)
  const float* audio;       // [N,L,A]
  const float* visual;      // [N,L,Vd]
  int64_t N;
  int L, D, A, Vd, Kp;
  float* x_out;
  float* num_out;
  float* cnt_out;
  float* s_out;     // [N][Kp] fp32, or with s_half [N][2][Kp] fp16 (hi | lo, row-scaled)
  float* aux_out;
  int32_t* flag;
  int s_half;
  float* cmax_part;  // per-wave (wave kernel) / per-workgroup running max |x| rows [P][D], or null
};

template <int VEC>
__device__ __forceinline__ void ldv(const float* p, float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    const float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
    v[0] = *p;
  }
}
// the same, non-temporal: for the read-once frame streams
template <int VEC>
__device__ __forceinline__ void ldv_nt(const float* p, float (&v)[VEC]) {
  if constexpr (VEC == 4) {
    using f4 = float __attribute__((ext_vector_type(4)));
    const f4 q = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
    v[0] = __builtin_nontemporal_load(p);
  }
}

// Power-of-2 scale that brings a row's max |value| into [2^14, 2^15): the
// projection GEMM splits the sums into fp16 hi/lo pairs (mm2_kernels.hip) and
// needs them in fp16's full-precision range.  Exact (a power of two).
__device__ __forceinline__ float row_scale(float m) {
  if (!(m > 0.f) || !isfinite(m)) return 1.f;
  int ex;
  frexpf(m, &ex);  // m = f * 2^ex, f in [0.5, 1)
  return ldexpf(1.f, 15 - ex);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Resolve token t of utterance i: element offset of its text row (or -1) and
// its SIF weight.  Semantics of sif_functions.py:8-15 (weight gather, id<0 ->
// 0) and numpy/torch fancy indexing for the row (negative ids wrap).
__device__ __forceinline__ void stage_token(const StreamArgs& a, int64_t i, int t, int64_t& off,
                                            float& w) {
  const int64_t ft = i * a.L + t;
  if (a.ids) {
    int64_t id = a.ids[ft];
    if (a.w_dense) {
      w = a.w_dense[ft];
    } else {
      w = (id >= 0 && id < a.V) ? a.wtab[id] : 0.f;
    }
    if (id < 0) id += a.V;
    if (id < 0 || id >= a.V) {
      if (a.flag) atomicOr(a.flag, MMB_FLAG_ID_RANGE);
      off = -1;
      w = 0.f;
    } else {
      off = id * a.D;
    }
  } else {
    w = a.w_dense ? a.w_dense[ft] : 0.f;
    off = ft * a.D;
  }
}

// Token staging of the workgroup kernel.  In gather mode the tokens whose
// row is table row 0 (id 0: the reference's pad / OOV index, ~72 % of a POM
// transcript) are not staged: they are counted (c0) and their weights summed
// (w0), and row 0 enters the sums once at the end as w0 * E0, c0 * E0,
// c0 * E0^2 -- one load instead of c0.  The other tokens are compacted in
// token order (wave ballots + a fixed-order prefix over the waves), so the
// text loop runs over rows that carry new bytes only.  Out-of-range ids
// (flagged) are dropped: they contribute nothing (sif_functions.py:8-15).
constexpr int kStageIters = (kTokChunk + kNT - 1) / kNT;

template <bool MM2, int VT, int VA, int VV>
__global__ __launch_bounds__(kNT) void utt_stream_kernel(StreamArgs a) {
  __shared__ int64_t s_off[kTokChunk];
  __shared__ float s_w[kTokChunk];
  __shared__ float s_red[(MM2 ? 4 : 1) * kRedFloats];
  __shared__ float s_cnt[kNT / kWave], s_sw[kNT / kWave];
  __shared__ float s_c0[kNT / kWave], s_w0[kNT / kWave];
  __shared__ int s_keep[kStageIters][kNT / kWave];

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1), wave = tid / kWave;
  // text lane map: CT column units of VT floats, RT row slots
  const int CT = a.D / VT;
  const int RT = kNT / CT;
  const int rT = tid / CT, cT = tid - (tid / CT) * CT;
  const bool actT = rT < RT;
  // audio / visual lane maps
  const int CA = MM2 ? a.A / VA : 1, RA = kNT / CA;
  const int rA = tid / CA, cA = tid - rA * CA;
  const int CV = MM2 ? a.Vd / VV : 1, RV = kNT / CV;
  const int rV = tid / CV, cV = tid - rV * CV;
  const float* tsrc = a.ids ? a.table : a.text_dense;
  const float* esrc = a.ids ? a.table : a.emb_dense;
  const bool split_emb = MM2 && (esrc != tsrc);

  const bool gather = a.ids != nullptr;
  float cmx0 = 0.f, cmx1 = 0.f;  // running max |x| of columns tid, tid + kNT (MMB2)
  for (int64_t i = blockIdx.x; i < a.N; i += gridDim.x) {
    float num[VT], sx[VT], sxx[VT];
#pragma unroll
    for (int e = 0; e < VT; ++e) num[e] = sx[e] = sxx[e] = 0.f;
    float cntp = 0.f, swp = 0.f, c0p = 0.f, w0p = 0.f;

    for (int t0 = 0; t0 < a.L; t0 += kTokChunk) {
      const int tl = min(kTokChunk, a.L - t0);
      int64_t off_k[kStageIters];
      float w_k[kStageIters];
      int rank_k[kStageIters];
      bool keep_k[kStageIters];
#pragma unroll
      for (int k = 0; k < kStageIters; ++k) {
        const int t = tid + k * kNT;
        int64_t off = -1;
        float w = 0.f;
        if (t < tl) {
          stage_token(a, i, t0 + t, off, w);
          cntp += (w != 0.f) ? 1.f : 0.f;
          swp += w;
          if (gather && off == 0) {
            c0p += 1.f;
            w0p += w;
          }
        }
        const bool keep = t < tl && (gather ? off > 0 : true);
        const unsigned long long bal = __ballot(keep);
        rank_k[k] = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) s_keep[k][wave] = __popcll(bal);
        off_k[k] = off;
        w_k[k] = w;
        keep_k[k] = keep;
      }
      __syncthreads();
      int nkeep = 0;
#pragma unroll
      for (int k = 0; k < kStageIters; ++k) {
        for (int v = 0; v < kNT / kWave; ++v) {
          if (keep_k[k] && v == wave) s_off[nkeep + rank_k[k]] = off_k[k];
          if (keep_k[k] && v == wave) s_w[nkeep + rank_k[k]] = w_k[k];
          nkeep += s_keep[k][v];
        }
      }
      __syncthreads();
      if (actT) {
        // branch-free: a negative offset (negative or flagged id) loads row
        // 0 and contributes nothing, so the unrolled iterations keep their
        // loads in flight together (a `continue` per token would wait on
        // each load right after its branch)
#pragma unroll 4
        for (int t = rT; t < nkeep; t += RT) {
          const float w = s_w[t];
          const int64_t off = s_off[t];
          const bool ok = off >= 0;
          const int64_t o = ok ? off : 0;
          float v[VT];
          ldv<VT>(tsrc + o + cT * VT, v);
#pragma unroll
          for (int e = 0; e < VT; ++e) v[e] = ok ? v[e] : 0.f;
          if (split_emb) {
            float u[VT];
            ldv<VT>(esrc + o + cT * VT, u);
#pragma unroll
            for (int e = 0; e < VT; ++e) num[e] = fmaf(w, ok ? u[e] : 0.f, num[e]);
          } else {
#pragma unroll
            for (int e = 0; e < VT; ++e) num[e] = fmaf(w, v[e], num[e]);
          }
          if constexpr (MM2) {
#pragma unroll
            for (int e = 0; e < VT; ++e) {
              sx[e] += v[e];
              sxx[e] = fmaf(v[e], v[e], sxx[e]);
            }
          }
        }
      }
      __syncthreads();
    }

    // audio / visual frame sums (MMB2 only): sum_t x and sum_t x^2 per feature
    float sa[VA], saa[VA], sv[VV], svv[VV];
#pragma unroll
    for (int e = 0; e < VA; ++e) sa[e] = saa[e] = 0.f;
#pragma unroll
    for (int e = 0; e < VV; ++e) sv[e] = svv[e] = 0.f;
    if constexpr (MM2) {
      if (rA < RA) {
        const float* base = a.audio + (i * a.L) * a.A + cA * VA;
#pragma unroll 4
        for (int t = rA; t < a.L; t += RA) {
          float v[VA];
          ldv_nt<VA>(base + static_cast<int64_t>(t) * a.A, v);
#pragma unroll
          for (int e = 0; e < VA; ++e) {
            sa[e] += v[e];
            saa[e] = fmaf(v[e], v[e], saa[e]);
          }
        }
      }
      if (rV < RV) {
        const float* base = a.visual + (i * a.L) * a.Vd + cV * VV;
#pragma unroll 4
        for (int t = rV; t < a.L; t += RV) {
          float v[VV];
          ldv_nt<VV>(base + static_cast<int64_t>(t) * a.Vd, v);
#pragma unroll
          for (int e = 0; e < VV; ++e) {
            sv[e] += v[e];
            svv[e] = fmaf(v[e], v[e], svv[e]);
          }
        }
      }
    }

    // count_nonzero(w) and sum(w) (and the row-0 token count / weight sum):
    // wave shuffle then fixed-order wave sum
    cntp = wave_sum(cntp);
    swp = wave_sum(swp);
    c0p = wave_sum(c0p);
    w0p = wave_sum(w0p);
    if (lane == 0) {
      s_cnt[wave] = cntp;
      s_sw[wave] = swp;
      s_c0[wave] = c0p;
      s_w0[wave] = w0p;
    }
    // round 1: text accumulators
    if (actT) {
#pragma unroll
      for (int e = 0; e < VT; ++e) {
        const int f = rT * a.D + cT * VT + e;
        s_red[f] = num[e];
        if constexpr (MM2) {
          s_red[kRedFloats + f] = sx[e];
          s_red[2 * kRedFloats + f] = sxx[e];
        }
      }
    }
    __syncthreads();
    float cnt = 0.f, sw = 0.f, c0 = 0.f, w0 = 0.f;
#pragma unroll
    for (int w = 0; w < kNT / kWave; ++w) {
      cnt += s_cnt[w];
      sw += s_sw[w];
      c0 += s_c0[w];
      w0 += s_w0[w];
    }
    float smax = 0.f;  // max |sum| of this thread's part of the row (MMB2)
    for (int f = tid; f < a.D; f += kNT) {
      float n_ = 0.f;
      for (int r = 0; r < RT; ++r) n_ += s_red[r * a.D + f];
      // row 0 once for its c0 tokens (gather mode; c0 = 0 otherwise)
      const float e0 = (c0 > 0.f) ? a.table[f] : 0.f;
      n_ = fmaf(w0, e0, n_);
      if constexpr (MM2) {
        float x1 = 0.f, x2 = 0.f;
        for (int r = 0; r < RT; ++r) {
          x1 += s_red[kRedFloats + r * a.D + f];
          x2 += s_red[2 * kRedFloats + r * a.D + f];
        }
        x1 = fmaf(c0, e0, x1);
        x2 = fmaf(c0 * e0, e0, x2);
        const float xf = n_ / cnt;
        a.num_out[i * a.D + f] = xf;  // x = the a2 row (sif_functions.py:55)
        if (f < kNT) cmx0 = fmaxf(cmx0, fabsf(xf)); else cmx1 = fmaxf(cmx1, fabsf(xf));
        a.s_out[i * a.Kp + f] = x1;
        a.s_out[i * a.Kp + a.D + f] = x2;
        smax = fmaxf(smax, fmaxf(fabsf(x1), fabsf(x2)));
      } else {
        if (a.num_out) a.num_out[i * a.D + f] = n_;
        if (a.x_out) a.x_out[i * a.D + f] = n_ / cnt;
      }
    }
    if (tid == 0) {
      if (cnt == 0.f && a.flag) atomicOr(a.flag, MMB_FLAG_ZERO_WEIGHTS);
      if constexpr (MM2) {
        a.aux_out[i] = cnt;         // planar [3][N]: row 0 doubles as the SIF count
        a.aux_out[a.N + i] = sw;
      } else {
        if (a.cnt_out) a.cnt_out[i] = cnt;
      }
    }
    if constexpr (MM2) {
      __syncthreads();
      // round 2: audio and visual accumulators
      if (rA < RA) {
#pragma unroll
        for (int e = 0; e < VA; ++e) {
          const int f = rA * a.A + cA * VA + e;
          s_red[f] = sa[e];
          s_red[kRedFloats + f] = saa[e];
        }
      }
      if (rV < RV) {
#pragma unroll
        for (int e = 0; e < VV; ++e) {
          const int f = rV * a.Vd + cV * VV + e;
          s_red[2 * kRedFloats + f] = sv[e];
          s_red[3 * kRedFloats + f] = svv[e];
        }
      }
      __syncthreads();
      float* srow = a.s_out + i * a.Kp + 2 * a.D;
      for (int f = tid; f < a.A; f += kNT) {
        float x1 = 0.f, x2 = 0.f;
        for (int r = 0; r < RA; ++r) {
          x1 += s_red[r * a.A + f];
          x2 += s_red[kRedFloats + r * a.A + f];
        }
        srow[f] = x1;
        srow[a.A + f] = x2;
        smax = fmaxf(smax, fmaxf(fabsf(x1), fabsf(x2)));
      }
      for (int f = tid; f < a.Vd; f += kNT) {
        float x1 = 0.f, x2 = 0.f;
        for (int r = 0; r < RV; ++r) {
          x1 += s_red[2 * kRedFloats + r * a.Vd + f];
          x2 += s_red[3 * kRedFloats + r * a.Vd + f];
        }
        srow[2 * a.A + f] = x1;
        srow[2 * a.A + a.Vd + f] = x2;
        smax = fmaxf(smax, fmaxf(fabsf(x1), fabsf(x2)));
      }
      const int k = 2 * (a.D + a.A + a.Vd);
      for (int f = k + tid; f < a.Kp; f += kNT) a.s_out[i * a.Kp + f] = 0.f;
      smax = wave_max(smax);
      if (lane == 0) s_cnt[wave] = smax;
      __syncthreads();
      if (tid == 0) {
        float m = 0.f;
        for (int w = 0; w < kNT / kWave; ++w) m = fmaxf(m, s_cnt[w]);
        a.aux_out[2 * a.N + i] = row_scale(m);
      }
    }
    __syncthreads();
  }
  if (MM2 && a.cmax_part) {  // this workgroup's column bounds (mmb_gram_i8)
    float* pr = a.cmax_part + static_cast<int64_t>(blockIdx.x) * a.D;
    if (tid < a.D) pr[tid] = cmx0;
    if (tid + kNT < a.D) pr[tid + kNT] = cmx1;
  }
}

// ---------------------------------------------------------------------------
// Wave-per-utterance variant (tokens/frames <= 64, widths % 4 == 0, <= 512):
// the fast path for MOSI / synthetic shapes.  One wave owns one utterance:
// lane t stages token t (id, weight) in registers and the loop broadcasts it
// with v_readlane, lane l owns float4 columns l and l+64 of every row for the
// whole utterance, so there is no LDS, no barrier and no cross-lane reduction
// of the sums — only independent 16-B loads (3 rows per frame in MMB2 mode)
// that the compiler keeps in flight across unrolled frames.
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
using nf4 = float __attribute__((ext_vector_type(4)));
// Frame streams are read exactly once: NT=true marks them non-temporal so they
// do not evict the (Zipf-hot) word-table rows from L2 / Infinity Cache.
template <bool NT>
__device__ __forceinline__ float4 ldnt4(const float* p) {
  if constexpr (NT) {
    const nf4 v = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  } else {
    return *reinterpret_cast<const float4*>(p);
  }
}
__device__ __forceinline__ void fma4(float4& acc, float w, float4 v) {
  acc.x = fmaf(w, v.x, acc.x); acc.y = fmaf(w, v.y, acc.y);
  acc.z = fmaf(w, v.z, acc.z); acc.w = fmaf(w, v.w, acc.w);
}
__device__ __forceinline__ void add4(float4& acc, float4 v) {
  acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
}
__device__ __forceinline__ void sq4(float4& acc, float4 v) {
  acc.x = fmaf(v.x, v.x, acc.x); acc.y = fmaf(v.y, v.y, acc.y);
  acc.z = fmaf(v.z, v.z, acc.z); acc.w = fmaf(v.w, v.w, acc.w);
}
__device__ __forceinline__ float amax4(float4 v) {
  return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
}
__device__ __forceinline__ float4 div4(float4 v, float c) {
  return make_float4(v.x / c, v.y / c, v.z / c, v.w / c);
}
using h4 = _Float16 __attribute__((ext_vector_type(4)));
// Output rows (x, s planes) are written once and read back by a later kernel,
// far beyond what L2 / Infinity Cache hold: NTS=true writes them non-temporal.
template <bool NTS>
__device__ __forceinline__ void stnt4(float* p, float4 v) {
  if constexpr (NTS) {
    __builtin_nontemporal_store(nf4{v.x, v.y, v.z, v.w}, reinterpret_cast<nf4*>(p));
  } else {
    *reinterpret_cast<float4*>(p) = v;
  }
}
// x * rs (rs a power of two: exact) as fp16 hi + fp16 lo = the residual
template <bool NTS = false>
__device__ __forceinline__ void split_store4(_Float16* hi, _Float16* lo, float4 v, float rs) {
  const float x[4] = {v.x * rs, v.y * rs, v.z * rs, v.w * rs};
  h4 h, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = static_cast<_Float16>(x[e]);
    l[e] = static_cast<_Float16>(x[e] - static_cast<float>(h[e]));
  }
  if constexpr (NTS) {
    __builtin_nontemporal_store(h, reinterpret_cast<h4*>(hi));
    __builtin_nontemporal_store(l, reinterpret_cast<h4*>(lo));
  } else {
    *reinterpret_cast<h4*>(hi) = h;
    *reinterpret_cast<h4*>(lo) = l;
  }
}

template <bool MM2, int CT, int CA, int CV, int UNR = 2, bool NT = false, bool SPLIT = false,
          bool NTS = false>
__global__ __launch_bounds__(256) void utt_wave_kernel(StreamArgs a) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wid = static_cast<int64_t>(blockIdx.x) * (blockDim.x / kWave) + threadIdx.x / kWave;
  const int64_t nw = static_cast<int64_t>(gridDim.x) * (blockDim.x / kWave);
  const int UT = a.D >> 2, UA = a.A >> 2, UV = a.Vd >> 2;
  const float* tsrc = a.ids ? a.table : a.text_dense;
  const float* esrc = a.ids ? a.table : a.emb_dense;
  constexpr bool split_emb = MM2 && SPLIT;  // weighted sum over a different dense tensor
  const bool gather = a.ids != nullptr;

  float4 cmx[CT];  // running max |x| of this lane's columns (MMB2, mmb_gram_i8)
#pragma unroll
  for (int c = 0; c < CT; ++c) cmx[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = wid; i < a.N; i += nw) {
    // stage: lane t <- token t (row id or -1, weight)
    int rid = -1;
    float w = 0.f;
    if (lane < a.L) {
      int64_t off;
      stage_token(a, i, lane, off, w);
      rid = off < 0 ? -1 : (gather ? static_cast<int>(off / a.D) : lane);
    }
    const float cnt = wave_sum((w != 0.f) ? 1.f : 0.f);
    const float sw = wave_sum(w);
    // every weight 0: x is 0/0 = NaN (numpy's answer); the reference's
    // TruncatedSVD then rejects the split -- report it through the flag word
    if (lane == 0 && cnt == 0.f && a.flag) atomicOr(a.flag, MMB_FLAG_ZERO_WEIGHTS);

    float4 num[CT], sx[CT], sxx[CT], sa[CA], saa[CA], sv[CV], svv[CV];
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int c = 0; c < CT; ++c) num[c] = sx[c] = sxx[c] = z4;
#pragma unroll
    for (int c = 0; c < CA; ++c) sa[c] = saa[c] = z4;
#pragma unroll
    for (int c = 0; c < CV; ++c) sv[c] = svv[c] = z4;
    const float* abase = a.audio + i * a.L * a.A;
    const float* vbase = a.visual + i * a.L * a.Vd;
    const int64_t dbase = i * a.L;

    // Column offsets clamped into the row so every lane loads unconditionally:
    // lanes past a row's width read a valid duplicate and never store it.  A
    // group of UNR frames issues ALL its loads before any accumulation — no
    // branch separates them, so UNR frames x (CT+CA+CV) 16-B loads per lane
    // are in flight together (a guarded load per lane would be waited on
    // right after its branch: one load in flight per wave).
    int ct[CT], ca[CA], cv[CV];
#pragma unroll
    for (int c = 0; c < CT; ++c) ct[c] = 4 * min(lane + kWave * c, UT - 1);
#pragma unroll
    for (int c = 0; c < CA; ++c) ca[c] = 4 * min(lane + kWave * c, MM2 ? UA - 1 : 0);
#pragma unroll
    for (int c = 0; c < CV; ++c) cv[c] = 4 * min(lane + kWave * c, MM2 ? UV - 1 : 0);
    auto frame = [&](int t, float4 (&vt)[CT], float4 (&ve)[CT], float4 (&va)[CA],
                     float4 (&vv)[CV], float& wt, bool& ok) {
      const int r = __builtin_amdgcn_readlane(rid, t);
      wt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), t));
      ok = r >= 0;  // an out-of-range id (flagged) contributes a zero row
      const int64_t o = (gather ? static_cast<int64_t>(ok ? r : 0) : dbase + t) * a.D;
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        vt[c] = ld4(tsrc + o + ct[c]);
        if (split_emb) ve[c] = ld4(esrc + o + ct[c]);
      }
      if constexpr (MM2) {
#pragma unroll
        for (int c = 0; c < CA; ++c) va[c] = ldnt4<NT>(abase + static_cast<int64_t>(t) * a.A + ca[c]);
#pragma unroll
        for (int c = 0; c < CV; ++c) vv[c] = ldnt4<NT>(vbase + static_cast<int64_t>(t) * a.Vd + cv[c]);
      }
    };
    auto accum = [&](float4 (&vt)[CT], float4 (&ve)[CT], float4 (&va)[CA], float4 (&vv)[CV],
                     float wt, bool ok) {
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        const float4 v = ok ? vt[c] : z4;
        fma4(num[c], wt, split_emb ? (ok ? ve[c] : z4) : v);
        if constexpr (MM2) {
          add4(sx[c], v);
          sq4(sxx[c], v);
        }
      }
      if constexpr (MM2) {
#pragma unroll
        for (int c = 0; c < CA; ++c) {
          add4(sa[c], va[c]);
          sq4(saa[c], va[c]);
        }
#pragma unroll
        for (int c = 0; c < CV; ++c) {
          add4(sv[c], vv[c]);
          sq4(svv[c], vv[c]);
        }
      }
    };
    int t = 0;
    for (; t + UNR <= a.L; t += UNR) {
      float4 vt[UNR][CT], ve[UNR][CT], va[UNR][CA], vv[UNR][CV];
      float wt[UNR];
      bool ok[UNR];
#pragma unroll
      for (int q = 0; q < UNR; ++q) frame(t + q, vt[q], ve[q], va[q], vv[q], wt[q], ok[q]);
#pragma unroll
      for (int q = 0; q < UNR; ++q) accum(vt[q], ve[q], va[q], vv[q], wt[q], ok[q]);
    }
    for (; t < a.L; ++t) {
      float4 vt[CT], ve[CT], va[CA], vv[CV];
      float wt;
      bool ok;
      frame(t, vt, ve, va, vv, wt, ok);
      accum(vt, ve, va, vv, wt, ok);
    }

    if constexpr (MM2) {
      float m = 0.f;
#pragma unroll
      for (int c = 0; c < CT; ++c) m = fmaxf(m, fmaxf(amax4(sx[c]), amax4(sxx[c])));
#pragma unroll
      for (int c = 0; c < CA; ++c) m = fmaxf(m, fmaxf(amax4(sa[c]), amax4(saa[c])));
#pragma unroll
      for (int c = 0; c < CV; ++c) m = fmaxf(m, fmaxf(amax4(sv[c]), amax4(svv[c])));
      const float rs = row_scale(wave_max(m));
      // one sums row: fp32, or fp16 hi | lo planes of the row-scaled sums (the
      // projection GEMM's A operand, ready for direct global->LDS staging)
      float* srow = a.s_out + i * a.Kp;
      _Float16* hrow = reinterpret_cast<_Float16*>(a.s_out) + i * 2 * a.Kp;
      auto put = [&](int f, float4 v) {
        if (a.s_half) {
          split_store4<NTS>(hrow + f, hrow + a.Kp + f, v, rs);
        } else {
          stnt4<NTS>(srow + f, v);
        }
      };
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        const int u = lane + kWave * c;
        if (u < UT) {
          const float4 xr = div4(num[c], cnt);
          stnt4<NTS>(a.num_out + i * a.D + 4 * u, xr);  // x = the a2 row
          cmx[c] = make_float4(fmaxf(cmx[c].x, fabsf(xr.x)), fmaxf(cmx[c].y, fabsf(xr.y)),
                               fmaxf(cmx[c].z, fabsf(xr.z)), fmaxf(cmx[c].w, fabsf(xr.w)));
          put(4 * u, sx[c]);
          put(a.D + 4 * u, sxx[c]);
        }
      }
#pragma unroll
      for (int c = 0; c < CA; ++c) {
        const int u = lane + kWave * c;
        if (u < UA) {
          put(2 * a.D + 4 * u, sa[c]);
          put(2 * a.D + a.A + 4 * u, saa[c]);
        }
      }
#pragma unroll
      for (int c = 0; c < CV; ++c) {
        const int u = lane + kWave * c;
        if (u < UV) {
          put(2 * (a.D + a.A) + 4 * u, sv[c]);
          put(2 * (a.D + a.A) + a.Vd + 4 * u, svv[c]);
        }
      }
      const int k = 2 * (a.D + a.A + a.Vd);
      for (int f = k + lane; f < a.Kp; f += kWave) {
        if (a.s_half) {
          hrow[f] = hrow[a.Kp + f] = static_cast<_Float16>(0.f);
        } else {
          srow[f] = 0.f;
        }
      }
      if (lane == 0) {
        a.aux_out[i] = cnt;  // planar [3][N]: count | sum w | fp16 row scale
        a.aux_out[a.N + i] = sw;
        a.aux_out[2 * a.N + i] = rs;
      }
    } else {
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        const int u = lane + kWave * c;
        if (u < UT) {
          if (a.num_out) st4(a.num_out + i * a.D + 4 * u, num[c]);
          if (a.x_out) st4(a.x_out + i * a.D + 4 * u, div4(num[c], cnt));
        }
      }
      if (lane == 0 && a.cnt_out) a.cnt_out[i] = cnt;
    }
  }
  if (MM2 && a.cmax_part) {  // this wave's column bounds (mmb_gram_i8)
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const int u = lane + kWave * c;
      if (u < UT) st4(a.cmax_part + wid * a.D + 4 * u, cmx[c]);
    }
  }
}

// colmax[f] = max over the P partial rows (float bits; non-negative floats
// order like their bits), fixed order.  16 row groups per column, LDS reduce.
__global__ __launch_bounds__(1024) void colmax_reduce_kernel(const float* __restrict__ part, int P,
                                                            int D, unsigned* __restrict__ colmax) {
  __shared__ float s_m[16][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int f = blockIdx.x * 64 + c;
  float m = 0.f;
  if (f < D) {
    // 8 independent loads in flight per thread (a single chain is latency-bound)
    float mm[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int r = g;
    for (; r + 7 * 16 < P; r += 8 * 16) {
#pragma unroll
      for (int u = 0; u < 8; ++u) mm[u] = fmaxf(mm[u], part[static_cast<int64_t>(r + 16 * u) * D + f]);
    }
    for (; r < P; r += 16) mm[0] = fmaxf(mm[0], part[static_cast<int64_t>(r) * D + f]);
#pragma unroll
    for (int u = 0; u < 8; ++u) m = fmaxf(m, mm[u]);
  }
  s_m[g][c] = m;
  __syncthreads();
  if (g == 0 && f < D) {
    for (int k = 1; k < 16; ++k) m = fmaxf(m, s_m[k][c]);
    colmax[f] = __float_as_uint(m);
  }
}

// Load/store policy of the MMB2 wave kernel: bit 0 = frame loads
// non-temporal, bit 1 = output stores non-temporal, bit 2 = 4 frames per load
// group instead of 2.  Default 5 (4-frame groups, non-temporal frame loads):
// measured on MI355X at 1M x 40 x 3 x 300-d, Zipf ids (tools/policy_sweep.sh):
// policy 0/1/2/3/4/5/6/7 = 20.65/20.62/21.00/19.94/20.54/19.80/20.57/20.09 ms;
// uniform ids 26.87 (0) -> 24.23 (5).  MMB_STREAM_POLICY overrides it (read
// once) for such sweeps.
static int stream_policy() {
  static const int p = [] {
    const char* e = getenv("MMB_STREAM_POLICY");
    return e ? atoi(e) : 5;
  }();
  return p;
}

template <bool MM2, int CT, int CA, int CV, int UNR, bool NT, bool NTS>
static void launch_wave_v(const StreamArgs& a, int grid, hipStream_t stream) {
  if (MM2 && a.ids == nullptr && a.emb_dense != a.text_dense) {
    utt_wave_kernel<MM2, CT, CA, CV, UNR, NT, true, NTS><<<grid, 256, 0, stream>>>(a);
  } else {
    utt_wave_kernel<MM2, CT, CA, CV, UNR, NT, false, NTS><<<grid, 256, 0, stream>>>(a);
  }
}

// Workgroups per CU of the grid-stride wave kernel: 2 = exactly the resident
// waves at its occupancy (2 waves / SIMD), one even share of utterances per
// wave.  Measured (tools/grid_sweep.sh, MI355X): 2/4/8/16/32 = 20.88/20.94/
// 21.04/21.01/21.18 ms.  MMB_STREAM_GRID_MULT overrides it (read once).
static int stream_grid_mult() {
  static const int m = [] {
    const char* e = getenv("MMB_STREAM_GRID_MULT");
    const int v = e ? atoi(e) : 2;
    return v > 0 ? v : 2;
  }();
  return m;
}

// rows of the column-bound partials (one per wave / workgroup of a launch)
constexpr int kCmaxRows = 8192;

template <bool MM2, int CT, int CA, int CV>
static int launch_wave(const StreamArgs& a, hipStream_t stream, int* parts = nullptr) {
  const int64_t blocks = ceil_div(a.N, 4);
  int grid_cap = stream_grid_mult() * stream_cu_count(stream);
  if (a.cmax_part && grid_cap > kCmaxRows / 4) grid_cap = kCmaxRows / 4;
  const int grid = static_cast<int>(blocks < grid_cap ? blocks : grid_cap);
  if (parts) *parts = grid * 4;
  switch (MM2 ? stream_policy() & 7 : 0) {
    case 1: launch_wave_v<MM2, CT, CA, CV, 2, true, false>(a, grid, stream); break;
    case 2: launch_wave_v<MM2, CT, CA, CV, 2, false, true>(a, grid, stream); break;
    case 3: launch_wave_v<MM2, CT, CA, CV, 2, true, true>(a, grid, stream); break;
    case 4: launch_wave_v<MM2, CT, CA, CV, 4, false, false>(a, grid, stream); break;
    case 5: launch_wave_v<MM2, CT, CA, CV, 4, true, false>(a, grid, stream); break;
    case 6: launch_wave_v<MM2, CT, CA, CV, 4, false, true>(a, grid, stream); break;
    case 7: launch_wave_v<MM2, CT, CA, CV, 4, true, true>(a, grid, stream); break;
    default: launch_wave_v<MM2, CT, CA, CV, 2, false, false>(a, grid, stream); break;
  }
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

__global__ void seq2weight_kernel(const int32_t* __restrict__ seq, const uint8_t* __restrict__ sel,
                                  int64_t total, const double* __restrict__ wtab, int64_t V,
                                  float* __restrict__ w, int32_t* flag) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int32_t id = seq[k];
    float out = 0.f;
    if ((sel == nullptr || sel[k]) && id >= 0) {
      if (id < V) {
        out = static_cast<float>(wtab[id]);  // f64 -> f32, round to nearest (sif_functions.py:13)
      } else if (flag) {
        atomicOr(flag, MMB_FLAG_ID_RANGE);
      }
    }
    w[k] = out;
  }
}

__global__ void calc_weights_kernel(const float* __restrict__ x, int64_t total, int F,
                                    const float* __restrict__ bm, const float* __restrict__ bl,
                                    float* __restrict__ qm, float* __restrict__ qs) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < total;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int f = static_cast<int>(k % F);
    const float d = x[k] - bm[f];
    const float e = expf(2.f * bl[f]);
    qm[k] = d / e;
    qs[k] = d * d / e - 1.f;
  }
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int stream_cu_count(hipStream_t stream) {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    return 256;
  }
  if (stream == nullptr) return n;
  uint32_t mask[32] = {};
  if (hipExtStreamGetCUMask(stream, 32, mask) != hipSuccess) {
    (void)hipGetLastError();  // a query failure is not a launch error
    return n;
  }
  int c = 0;
  for (int b = 0; b < n && b < 32 * 32; ++b) c += (mask[b >> 5] >> (b & 31)) & 1;
  return (c > 0 && c < n) ? c : n;
}

template <bool MM2, int VT, int VA, int VV>
static int launch_stream(const StreamArgs& a, hipStream_t stream, int* parts = nullptr) {
  int grid = stream_grid(a.N, 6, stream);
  if (a.cmax_part && grid > kCmaxRows) grid = kCmaxRows;
  if (parts) *parts = grid;
  utt_stream_kernel<MM2, VT, VA, VV><<<grid, kNT, 0, stream>>>(a);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

}  // namespace mmb

using namespace mmb;

extern "C" int mmb_version(void) { return 100; }

extern "C" int mmb_cu_count(int device, int* out) {
  MMB_REQUIRE(out);
  const hipError_t e = hipDeviceGetAttribute(out, hipDeviceAttributeMultiprocessorCount, device);
  return e == hipSuccess ? MMB_OK : static_cast<int>(e);
}

extern "C" int mmb_stream_create_cu_mask(const uint32_t* cu_mask, int mask_words,
                                         hipStream_t* out) {
  MMB_REQUIRE(cu_mask && mask_words > 0 && out);
  const hipError_t e =
      hipExtStreamCreateWithCUMask(out, static_cast<uint32_t>(mask_words), cu_mask);
  return e == hipSuccess ? MMB_OK : static_cast<int>(e);
}

extern "C" int mmb_stream_destroy(hipStream_t stream) {
  MMB_REQUIRE(stream);
  const hipError_t e = hipStreamDestroy(stream);
  return e == hipSuccess ? MMB_OK : static_cast<int>(e);
}

extern "C" int mmb_seq2weight(const int32_t* seq, const uint8_t* sel, int64_t n, int64_t l,
                              const double* wtab64, int64_t v, float* w_out, int32_t* flag,
                              hipStream_t stream) {
  MMB_REQUIRE(n >= 0 && l >= 0 && v > 0 && seq && wtab64 && w_out);
  const int64_t total = n * l;
  if (total == 0) return MMB_OK;
  const int grid = static_cast<int>(std::min<int64_t>(ceil_div(total, 256), 256 * 16));
  seq2weight_kernel<<<grid, 256, 0, stream>>>(seq, sel, total, wtab64, v, w_out, flag);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_sif_wavg(const float* table, int64_t v, int d, const int32_t* ids, int64_t n,
                            int l, const float* w, const float* wtab32, float* x_out,
                            float* num_out, float* cnt_out, int32_t* flag, hipStream_t stream) {
  MMB_REQUIRE(table && ids && v > 0 && d > 0 && n >= 0 && l >= 0);
  MMB_REQUIRE(w || wtab32);
  MMB_REQUIRE(x_out || num_out || cnt_out);
  if (n == 0) return MMB_OK;
  StreamArgs a{};
  a.ids = ids; a.table = table; a.V = v; a.wtab = wtab32; a.w_dense = w;
  a.N = n; a.L = l; a.D = d;
  a.x_out = x_out; a.num_out = num_out; a.cnt_out = cnt_out; a.flag = flag;
  const bool v4 = (d % 4 == 0) && aligned16(table);
  if (v4 && l <= kWave && d <= 512 && (x_out == nullptr || aligned16(x_out)) &&
      (num_out == nullptr || aligned16(num_out))) {
    return d <= 256 ? launch_wave<false, 1, 1, 1>(a, stream) : launch_wave<false, 2, 1, 1>(a, stream);
  }
  MMB_REQUIRE(d / (v4 ? 4 : 1) <= kNT && d <= kRedFloats);
  return v4 ? launch_stream<false, 4, 1, 1>(a, stream) : launch_stream<false, 1, 1, 1>(a, stream);
}

extern "C" int mmb_calc_weights(const float* x, int64_t rows, int f, const float* b_mean,
                                const float* b_log_sigma, float* q_mean, float* q_sigma,
                                hipStream_t stream) {
  MMB_REQUIRE(x && b_mean && b_log_sigma && q_mean && q_sigma && rows >= 0 && f > 0);
  const int64_t total = rows * f;
  if (total == 0) return MMB_OK;
  const int grid = static_cast<int>(std::min<int64_t>(ceil_div(total, 256), 256 * 16));
  calc_weights_kernel<<<grid, 256, 0, stream>>>(x, total, f, b_mean, b_log_sigma, q_mean, q_sigma);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_mm2_k(int d, int a, int vd) {
  const int k = 2 * (d + a + vd);
  return (k + 31) / 32 * 32;
}

// The workgroup stream kernel writes fp32 sums; for the fp16 hi/lo format a
// second pass splits each row in place (one workgroup per row, the row staged
// in LDS).  Only the fallback shapes (tokens > 64, widths not % 4) take it.
__global__ __launch_bounds__(256) void split_rows_kernel(float* __restrict__ s,
                                                         const float* __restrict__ rscale,
                                                         int Kp) {
  extern __shared__ float srow[];
  const int64_t i = blockIdx.x;
  float* row = s + i * Kp;
  for (int f = threadIdx.x; f < Kp; f += blockDim.x) srow[f] = row[f];
  __syncthreads();
  const float rs = rscale[i];
  _Float16* hi = reinterpret_cast<_Float16*>(row);
  for (int f = threadIdx.x; f < Kp; f += blockDim.x) {
    const float x = srow[f] * rs;
    const _Float16 h = static_cast<_Float16>(x);
    hi[f] = h;
    hi[Kp + f] = static_cast<_Float16>(x - static_cast<float>(h));
  }
}

extern "C" size_t mmb_mm2_colmax_ws_bytes(int d) {
  return static_cast<size_t>(kCmaxRows) * (d > 0 ? d : 0) * sizeof(float);
}

extern "C" int mmb_mm2_stream(const int32_t* ids, const float* table, int64_t v,
                              const float* wtab32, const float* text_dense,
                              const float* emb_dense, const float* w_dense, const float* audio,
                              const float* visual, int64_t n, int t, int d, int a_, int vd,
                              float* num_out, void* s_out, int s_half, float* aux_out,
                              int32_t* flag, uint32_t* colmax, void* colmax_ws,
                              hipStream_t stream) {
  MMB_REQUIRE(n >= 0 && t > 0 && d > 0 && a_ > 0 && vd > 0);
  MMB_REQUIRE(colmax == nullptr || (colmax_ws != nullptr && d <= 2 * kNT));
  MMB_REQUIRE(audio && visual && num_out && s_out && aux_out && (s_half == 0 || s_half == 1));
  if (ids) {
    MMB_REQUIRE(table && v > 0 && (wtab32 || w_dense));
  } else {
    MMB_REQUIRE(text_dense && emb_dense && w_dense);
  }
  if (n == 0) {
    if (colmax) {
      const hipError_t e = hipMemsetAsync(colmax, 0, sizeof(uint32_t) * d, stream);
      if (e != hipSuccess) return static_cast<int>(e);
    }
    return MMB_OK;
  }
  StreamArgs s{};
  s.cmax_part = colmax ? static_cast<float*>(colmax_ws) : nullptr;
  int parts = 0;
  // the column bounds: max over the launch's per-wave / per-workgroup rows
  auto reduce_colmax = [&](int rc) {
    if (rc != MMB_OK || !colmax) return rc;
    colmax_reduce_kernel<<<static_cast<unsigned>(ceil_div(d, 64)), 1024, 0, stream>>>(
        static_cast<const float*>(colmax_ws), parts, d, colmax);
    MMB_LAUNCH_CHECK();
    return static_cast<int>(MMB_OK);
  };
  s.ids = ids; s.table = table; s.V = v; s.wtab = wtab32; s.w_dense = w_dense;
  s.text_dense = text_dense; s.emb_dense = emb_dense; s.audio = audio; s.visual = visual;
  s.N = n; s.L = t; s.D = d; s.A = a_; s.Vd = vd; s.Kp = mmb_mm2_k(d, a_, vd);
  s.num_out = num_out; s.s_out = static_cast<float*>(s_out); s.aux_out = aux_out; s.flag = flag;
  s.s_half = s_half;
  const bool vt = (d % 4 == 0) && (ids ? aligned16(table) : (aligned16(text_dense) && aligned16(emb_dense)));
  const bool va = (a_ % 4 == 0) && aligned16(audio);
  const bool vv = (vd % 4 == 0) && aligned16(visual);
  if (vt && va && vv && t <= kWave && d <= 512 && a_ <= 512 && vd <= 512 && aligned16(num_out) &&
      aligned16(s_out)) {
    const int sel = (d > 256 ? 4 : 0) | (a_ > 256 ? 2 : 0) | (vd > 256 ? 1 : 0);
    switch (sel) {
      case 7: return reduce_colmax(launch_wave<true, 2, 2, 2>(s, stream, &parts));
      case 6: return reduce_colmax(launch_wave<true, 2, 2, 1>(s, stream, &parts));
      case 5: return reduce_colmax(launch_wave<true, 2, 1, 2>(s, stream, &parts));
      case 4: return reduce_colmax(launch_wave<true, 2, 1, 1>(s, stream, &parts));
      case 3: return reduce_colmax(launch_wave<true, 1, 2, 2>(s, stream, &parts));
      case 2: return reduce_colmax(launch_wave<true, 1, 2, 1>(s, stream, &parts));
      case 1: return reduce_colmax(launch_wave<true, 1, 1, 2>(s, stream, &parts));
      default: return reduce_colmax(launch_wave<true, 1, 1, 1>(s, stream, &parts));
    }
  }
  MMB_REQUIRE(d / (vt ? 4 : 1) <= kNT && a_ / (va ? 4 : 1) <= kNT && vd / (vv ? 4 : 1) <= kNT);
  s.s_half = 0;
  const int sel = (vt ? 4 : 0) | (va ? 2 : 0) | (vv ? 1 : 0);
  int rc;
  switch (sel) {
    case 7: rc = launch_stream<true, 4, 4, 4>(s, stream, &parts); break;
    case 6: rc = launch_stream<true, 4, 4, 1>(s, stream, &parts); break;
    case 5: rc = launch_stream<true, 4, 1, 4>(s, stream, &parts); break;
    case 4: rc = launch_stream<true, 4, 1, 1>(s, stream, &parts); break;
    case 3: rc = launch_stream<true, 1, 4, 4>(s, stream, &parts); break;
    case 2: rc = launch_stream<true, 1, 4, 1>(s, stream, &parts); break;
    case 1: rc = launch_stream<true, 1, 1, 4>(s, stream, &parts); break;
    default: rc = launch_stream<true, 1, 1, 1>(s, stream, &parts); break;
  }
  rc = reduce_colmax(rc);
  if (rc != MMB_OK || !s_half) return rc;
  split_rows_kernel<<<static_cast<unsigned>(n), 256, s.Kp * sizeof(float), stream>>>(
      s.s_out, aux_out + 2 * n, s.Kp);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}
