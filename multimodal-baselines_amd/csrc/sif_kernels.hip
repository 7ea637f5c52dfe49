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
#include <algorithm>
#include <cstdlib>
#include <type_traits>

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

// max of two column bounds |x| >= 0 on their bits: for non-negative floats the
// unsigned order is the float order, and a NaN (|NaN| = 0x7fc00000..) ranks
// above inf -- so a non-finite x reaches the bound (and mmb_gram_i8 then
// writes NaN into G, as the f64 Gram would), where fmaxf would drop a NaN
__device__ __forceinline__ float bmax(float a, float b) {
  return __uint_as_float(max(__float_as_uint(a), __float_as_uint(b)));
}
__device__ __forceinline__ float4 bmax4(float4 m, float4 x) {
  return make_float4(bmax(m.x, fabsf(x.x)), bmax(m.y, fabsf(x.y)), bmax(m.z, fabsf(x.z)),
                     bmax(m.w, fabsf(x.w)));
}

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

// The text rows of a staged token chunk (workgroup kernels): row slot rT
// of the chunk's nkeep kept tokens, CT column units of VT floats at cT.
// Branch-free per row (a negative offset loads row 0 and contributes
// nothing) and SPLIT (the weighted sum over a different dense tensor) a
// template argument, so the TU unrolled rows' loads issue together: a
// runtime `split_emb` test per row put a branch and a wait for that row's
// load after every load (r06: the gfx950 ISA of the split-part kernel).
template <bool MM2, bool SPLIT, int VT, int TU>
__device__ __forceinline__ void text_rows(const float* tsrc, const float* esrc, const int64_t* s_off,
                                          const float* s_w, int nkeep, int rT, int RT, int cT,
                                          float (&num)[VT], float (&sx)[VT], float (&sxx)[VT]) {
#pragma unroll TU
  for (int t = rT; t < nkeep; t += RT) {
    const float w = s_w[t];
    const int64_t off = s_off[t];
    const bool ok = off >= 0;
    const int64_t o = ok ? off : 0;
    float v[VT];
    ldv<VT>(tsrc + o + cT * VT, v);
#pragma unroll
    for (int e = 0; e < VT; ++e) v[e] = ok ? v[e] : 0.f;
    if constexpr (SPLIT) {
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

// FU: frame rows (and TU: text rows) per thread in flight -- 4 / 4 when the
// grid fills the chip (occupancy hides the latency); for a few hundred long
// rows (dataset splits: one workgroup per CU at most, so one workgroup's
// loads in flight set the time; POM's 100-row valid split spent 0.18 ms in 68
// rounds of 4 frame loads per thread) NT = 1024 threads with 8 / 4.  NT
// changes the f32 order of the row sums (RT = NT / CT row slots).
template <bool MM2, int VT, int VA, int VV, int FU = 4, int TU = 4, int NT = kNT>
__global__ __launch_bounds__(NT) void utt_stream_kernel(StreamArgs a) {
  constexpr int kRF = NT * 4;  // one accumulator image: R*F <= NT*VEC
  constexpr int kSI = (kTokChunk + NT - 1) / NT;
  __shared__ int64_t s_off[kTokChunk];
  __shared__ float s_w[kTokChunk];
  __shared__ float s_red[(MM2 ? 4 : 1) * kRF];
  __shared__ float s_cnt[NT / kWave], s_sw[NT / kWave];
  __shared__ float s_c0[NT / kWave], s_w0[NT / kWave];
  __shared__ int s_keep[kSI][NT / kWave];

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1), wave = tid / kWave;
  // text lane map: CT column units of VT floats, RT row slots
  const int CT = a.D / VT;
  const int RT = NT / CT;
  const int rT = tid / CT, cT = tid - (tid / CT) * CT;
  const bool actT = rT < RT;
  // audio / visual lane maps
  const int CA = MM2 ? a.A / VA : 1, RA = NT / CA;
  const int rA = tid / CA, cA = tid - rA * CA;
  const int CV = MM2 ? a.Vd / VV : 1, RV = NT / CV;
  const int rV = tid / CV, cV = tid - rV * CV;
  const float* tsrc = a.ids ? a.table : a.text_dense;
  const float* esrc = a.ids ? a.table : a.emb_dense;
  const bool split_emb = MM2 && (esrc != tsrc);

  const bool gather = a.ids != nullptr;
  float cmx0 = 0.f, cmx1 = 0.f;  // running max |x| of columns tid, tid + NT (MMB2)
  for (int64_t i = blockIdx.x; i < a.N; i += gridDim.x) {
    float num[VT], sx[VT], sxx[VT];
#pragma unroll
    for (int e = 0; e < VT; ++e) num[e] = sx[e] = sxx[e] = 0.f;
    float cntp = 0.f, swp = 0.f, c0p = 0.f, w0p = 0.f;

    for (int t0 = 0; t0 < a.L; t0 += kTokChunk) {
      const int tl = min(kTokChunk, a.L - t0);
      int64_t off_k[kSI];
      float w_k[kSI];
      int rank_k[kSI];
      bool keep_k[kSI];
#pragma unroll
      for (int k = 0; k < kSI; ++k) {
        const int t = tid + k * NT;
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
      for (int k = 0; k < kSI; ++k) {
        for (int v = 0; v < NT / kWave; ++v) {
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
        if (split_emb)
          text_rows<MM2, true, VT, TU>(tsrc, esrc, s_off, s_w, nkeep, rT, RT, cT, num, sx, sxx);
        else
          text_rows<MM2, false, VT, TU>(tsrc, esrc, s_off, s_w, nkeep, rT, RT, cT, num, sx, sxx);
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
#pragma unroll FU
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
#pragma unroll FU
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
          s_red[kRF + f] = sx[e];
          s_red[2 * kRF + f] = sxx[e];
        }
      }
    }
    __syncthreads();
    float cnt = 0.f, sw = 0.f, c0 = 0.f, w0 = 0.f;
#pragma unroll
    for (int w = 0; w < NT / kWave; ++w) {
      cnt += s_cnt[w];
      sw += s_sw[w];
      c0 += s_c0[w];
      w0 += s_w0[w];
    }
    float smax = 0.f;  // max |sum| of this thread's part of the row (MMB2)
    for (int f = tid; f < a.D; f += NT) {
      float n_ = 0.f;
      for (int r = 0; r < RT; ++r) n_ += s_red[r * a.D + f];
      // row 0 once for its c0 tokens (gather mode; c0 = 0 otherwise)
      const float e0 = (c0 > 0.f) ? a.table[f] : 0.f;
      n_ = fmaf(w0, e0, n_);
      if constexpr (MM2) {
        float x1 = 0.f, x2 = 0.f;
        for (int r = 0; r < RT; ++r) {
          x1 += s_red[kRF + r * a.D + f];
          x2 += s_red[2 * kRF + r * a.D + f];
        }
        x1 = fmaf(c0, e0, x1);
        x2 = fmaf(c0 * e0, e0, x2);
        const float xf = n_ / cnt;
        a.num_out[i * a.D + f] = xf;  // x = the a2 row (sif_functions.py:55)
        if (f < NT) cmx0 = bmax(cmx0, fabsf(xf)); else cmx1 = bmax(cmx1, fabsf(xf));
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
          s_red[kRF + f] = saa[e];
        }
      }
      if (rV < RV) {
#pragma unroll
        for (int e = 0; e < VV; ++e) {
          const int f = rV * a.Vd + cV * VV + e;
          s_red[2 * kRF + f] = sv[e];
          s_red[3 * kRF + f] = svv[e];
        }
      }
      __syncthreads();
      float* srow = a.s_out + i * a.Kp + 2 * a.D;
      for (int f = tid; f < a.A; f += NT) {
        float x1 = 0.f, x2 = 0.f;
        for (int r = 0; r < RA; ++r) {
          x1 += s_red[r * a.A + f];
          x2 += s_red[kRF + r * a.A + f];
        }
        srow[f] = x1;
        srow[a.A + f] = x2;
        smax = fmaxf(smax, fmaxf(fabsf(x1), fabsf(x2)));
      }
      for (int f = tid; f < a.Vd; f += NT) {
        float x1 = 0.f, x2 = 0.f;
        for (int r = 0; r < RV; ++r) {
          x1 += s_red[2 * kRF + r * a.Vd + f];
          x2 += s_red[3 * kRF + r * a.Vd + f];
        }
        srow[2 * a.A + f] = x1;
        srow[2 * a.A + a.Vd + f] = x2;
        smax = fmaxf(smax, fmaxf(fabsf(x1), fabsf(x2)));
      }
      const int k = 2 * (a.D + a.A + a.Vd);
      for (int f = k + tid; f < a.Kp; f += NT) a.s_out[i * a.Kp + f] = 0.f;
      smax = wave_max(smax);
      if (lane == 0) s_cnt[wave] = smax;
      __syncthreads();
      if (tid == 0) {
        float m = 0.f;
        for (int w = 0; w < NT / kWave; ++w) m = fmaxf(m, s_cnt[w]);
        a.aux_out[2 * a.N + i] = row_scale(m);
      }
    }
    __syncthreads();
  }
  if (MM2 && a.cmax_part) {  // this workgroup's column bounds (mmb_gram_i8)
    float* pr = a.cmax_part + static_cast<int64_t>(blockIdx.x) * a.D;
    if (tid < a.D) pr[tid] = cmx0;
    if (tid + NT < a.D) pr[tid + NT] = cmx1;
  }
}

// ---------------------------------------------------------------------------
// Few long rows split over workgroups (r06; POM's splits: 100 / 203
// transcripts of 1089 / 1357 aligned tokens).  One workgroup per utterance
// (utt_stream_kernel) puts 100 / 203 workgroups on 256 CUs, each a
// 1,089-1,357-frame chain: 0.21 / 0.42 of 8 TB/s.  Here every utterance is
// cut into P ranges of Lc tokens / frames and each range has a text and a
// frame workgroup, in ONE launch: the text workgroups (blocks [0, N Pt):
// token staging, the kept rows' gather, the counts) first, then the frame
// workgroups (one modality each, audio then visual: pure streams, no
// staging, no barrier before their reduction), each writing PARTIAL sums; utt_split_finish_kernel adds
// an utterance's partials in fixed part order and finishes the row as
// utt_stream_kernel does (x = num / count, the s row, aux, the row scale,
// the column bounds) -- writing the fp16 hi / lo planes directly, so the
// s_half path needs no split_rows pass.  Deterministic; against the
// one-workgroup kernel only the f32 order of the token and frame sums
// differs (with one range it is the same order: bit-identical).
//
// Workspace (floats): text partials [N][Pt][Wt] = [num (D) | Sx_e (D) |
// Sxx_e (D) | count_nonzero(w), sum w, row-0 tokens, their weight sum] (row
// 0 excluded from the sums, as utt_stream_kernel), then frame partials
// [N][Pf][Wf] = [Sx_a (A) | Sxx_a (A) | Sx_v (Vd) | Sxx_v (Vd)].
struct SplitPlan {
  int Pt, Lt, Pf, Lf;  // text / frame parts per utterance and their lengths
  int Wt, Wf;          // partial row strides (floats, multiples of 4)
};
// A/B build constants of the split kernel (tools/ab_libs/build_split.sh):
// text ranges per frame range of the automatic plan (MMB_SPLIT_TEXT_X; an
// explicit part count keeps them equal), text / frame rows unrolled per
// thread group (MMB_SPLIT_TU / MMB_SPLIT_FU; the sums' order is the same).
// Alternated twice on POM's real splits (r06, profiles/r06/splitab*,
// valid / test stream ms): TU 8 FU 16 0.0556-0.0567 / 0.126-0.128; FU 8
// 0.0545-0.0551 / 0.123-0.125 (kept); FU 4 0.067 / 0.146; FU 32 0.065 /
// 0.141; TU 16 0.072 / 0.151; TU 4 FU 8 0.067 / 0.116; two text ranges per
// frame range 0.058 / 0.131 -- the text workgroups are not the long pole
#ifndef MMB_SPLIT_TEXT_X
#define MMB_SPLIT_TEXT_X 1
#endif
#ifndef MMB_SPLIT_TU
#define MMB_SPLIT_TU 8
#endif
#ifndef MMB_SPLIT_FU
#define MMB_SPLIT_FU 8
#endif
inline SplitPlan split_plan_of(int t, int d, int a, int vd, int Pf, int text_x = 1) {
  SplitPlan q;
  q.Lf = (t + Pf - 1) / Pf;
  q.Pf = (t + q.Lf - 1) / q.Lf;  // no empty part
  // the text ranges are the frame ranges (over kTokChunk tokens they are
  // staged chunk by chunk): with one range the sums run in the one-workgroup
  // kernel's order.  One LDS chunk per text workgroup instead measured no
  // faster (POM valid 57.5 vs 55.3 us, r06 tools/split_ab.py)
  q.Lt = (t + q.Pf * text_x - 1) / (q.Pf * text_x);
  q.Pt = (t + q.Lt - 1) / q.Lt;
  q.Wt = (3 * d + 4 + 3) / 4 * 4;
  q.Wf = (2 * a + 2 * vd + 3) / 4 * 4;
  return q;
}

template <int VT, int VA, int VV, int FU = 16, int TU = 8>
__global__ __launch_bounds__(kNT) void utt_split_part_kernel(StreamArgs a, SplitPlan q,
                                                             float* __restrict__ part) {
  constexpr int NT = kNT;
  constexpr int kRF = NT * 4;
  constexpr int kSI = (kTokChunk + NT - 1) / NT;
  __shared__ int64_t s_off[kTokChunk];
  __shared__ float s_w[kTokChunk];
  __shared__ float s_red[4 * kRF];
  __shared__ float s_sc[4][NT / kWave];
  __shared__ int s_keep[kSI][NT / kWave];

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1), wave = tid / kWave;
  const int64_t ntext = a.N * q.Pt;
  if (static_cast<int64_t>(blockIdx.x) < ntext) {
    // ---- a token range: staging, the kept rows, the counts
    const int64_t i = blockIdx.x / q.Pt;
    const int p = static_cast<int>(blockIdx.x - i * q.Pt);
    const int tb = p * q.Lt, te = min(a.L, tb + q.Lt);
    const int CT = a.D / VT, RT = NT / CT;
    const int rT = tid / CT, cT = tid - rT * CT;
    const bool actT = rT < RT;
    const float* tsrc = a.ids ? a.table : a.text_dense;
    const float* esrc = a.ids ? a.table : a.emb_dense;
    const bool gather = a.ids != nullptr;
    float num[VT], sx[VT], sxx[VT];
#pragma unroll
    for (int e = 0; e < VT; ++e) num[e] = sx[e] = sxx[e] = 0.f;
    float cntp = 0.f, swp = 0.f, c0p = 0.f, w0p = 0.f;
    for (int t0 = tb; t0 < te; t0 += kTokChunk) {  // the range in LDS chunks
      const int tl = min(kTokChunk, te - t0);
      int64_t off_k[kSI];
      float w_k[kSI];
      int rank_k[kSI];
      bool keep_k[kSI];
#pragma unroll
      for (int k = 0; k < kSI; ++k) {
        const int t = tid + k * NT;
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
      for (int k = 0; k < kSI; ++k) {
        for (int v = 0; v < NT / kWave; ++v) {
          if (keep_k[k] && v == wave) {
            s_off[nkeep + rank_k[k]] = off_k[k];
            s_w[nkeep + rank_k[k]] = w_k[k];
          }
          nkeep += s_keep[k][v];
        }
      }
      __syncthreads();
      if (actT) {
        if (esrc != tsrc)
          text_rows<true, true, VT, TU>(tsrc, esrc, s_off, s_w, nkeep, rT, RT, cT, num, sx, sxx);
        else
          text_rows<true, false, VT, TU>(tsrc, esrc, s_off, s_w, nkeep, rT, RT, cT, num, sx, sxx);
      }
      __syncthreads();
    }
    cntp = wave_sum(cntp);
    swp = wave_sum(swp);
    c0p = wave_sum(c0p);
    w0p = wave_sum(w0p);
    if (lane == 0) {
      s_sc[0][wave] = cntp;
      s_sc[1][wave] = swp;
      s_sc[2][wave] = c0p;
      s_sc[3][wave] = w0p;
    }
    if (actT) {
#pragma unroll
      for (int e = 0; e < VT; ++e) {
        const int f = rT * a.D + cT * VT + e;
        s_red[f] = num[e];
        s_red[kRF + f] = sx[e];
        s_red[2 * kRF + f] = sxx[e];
      }
    }
    __syncthreads();
    float* prow = part + (i * q.Pt + p) * static_cast<int64_t>(q.Wt);
    for (int f = tid; f < a.D; f += NT) {  // the row slots summed in order
      float n_ = 0.f, x1 = 0.f, x2 = 0.f;
      for (int r = 0; r < RT; ++r) {
        n_ += s_red[r * a.D + f];
        x1 += s_red[kRF + r * a.D + f];
        x2 += s_red[2 * kRF + r * a.D + f];
      }
      prow[f] = n_;
      prow[a.D + f] = x1;
      prow[2 * a.D + f] = x2;
    }
    if (tid < 4) {
      float sc = 0.f;
#pragma unroll
      for (int w = 0; w < NT / kWave; ++w) sc += s_sc[tid][w];
      prow[3 * a.D + tid] = sc;
    }
    return;
  }
  // ---- a frame range of ONE modality (audio workgroups, then visual)
  const int64_t b = blockIdx.x - ntext;
  const bool vis = b >= a.N * q.Pf;
  const int64_t bm = vis ? b - a.N * q.Pf : b;
  const int64_t i = bm / q.Pf;
  const int p = static_cast<int>(bm - i * q.Pf);
  const int tb = p * q.Lf, te = min(a.L, tb + q.Lf);
  float* prow = part + ntext * q.Wt + (i * q.Pf + p) * static_cast<int64_t>(q.Wf);
  auto stream = [&](const float* src, int F, float* out, auto vec) {
    constexpr int VF = decltype(vec)::value;
    const int CF = F / VF, RF = NT / CF;
    const int rF = tid / CF, cF = tid - rF * CF;
    float sm[VF], sq[VF];
#pragma unroll
    for (int e = 0; e < VF; ++e) sm[e] = sq[e] = 0.f;
    if (rF < RF) {
      const float* base = src + (i * a.L) * F + cF * VF;
#pragma unroll FU
      for (int t = tb + rF; t < te; t += RF) {
        float v[VF];
        ldv_nt<VF>(base + static_cast<int64_t>(t) * F, v);
#pragma unroll
        for (int e = 0; e < VF; ++e) {
          sm[e] += v[e];
          sq[e] = fmaf(v[e], v[e], sq[e]);
        }
      }
#pragma unroll
      for (int e = 0; e < VF; ++e) {
        const int f = rF * F + cF * VF + e;
        s_red[f] = sm[e];
        s_red[kRF + f] = sq[e];
      }
    }
    __syncthreads();
    for (int f = tid; f < F; f += NT) {  // the row slots summed in order
      float x1 = 0.f, x2 = 0.f;
      for (int r = 0; r < RF; ++r) {
        x1 += s_red[r * F + f];
        x2 += s_red[kRF + r * F + f];
      }
      out[f] = x1;
      out[F + f] = x2;
    }
  };
  if (vis)
    stream(a.visual, a.Vd, prow + 2 * a.A, std::integral_constant<int, VV>{});
  else
    stream(a.audio, a.A, prow, std::integral_constant<int, VA>{});
}

// The partials of utterance i (blockIdx.x) in part order, then the row's
// epilogue of utt_stream_kernel: row 0 once for its tokens, x, the s row
// (fp32, or the fp16 hi / lo planes of s * rs), aux, the column bounds of
// this workgroup (grid = N <= kCmaxRows rows of cmax_part).  Thread tid owns
// columns f = tid + NT j (j < kSplitJ) of [num | Sx_e | Sxx_e | frame sums]
// and walks each kind's parts in order, all kSplitJ loads of a part issued
// together (a loop over the parts per column was a chain of P dependent L2
// round trips per column).
constexpr int kSplitJ = 7;  // ceil((3 * 320 + 4 * 320) / kNT): every partial column
__global__ __launch_bounds__(kNT) void utt_split_finish_kernel(StreamArgs a, SplitPlan q,
                                                               const float* __restrict__ part) {
  constexpr int NT = kNT;
  extern __shared__ float s_row[];  // s_half: the fp32 row before the split
  __shared__ float s_m[NT / kWave];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  const int64_t i = blockIdx.x;
  const int K = 2 * (a.D + a.A + a.Vd);
  const int D3 = 3 * a.D, W = a.D + K;  // text columns; all partial columns
  const float* pt = part + i * q.Pt * static_cast<int64_t>(q.Wt);
  const float* pf = part + a.N * q.Pt * static_cast<int64_t>(q.Wt) + i * q.Pf * static_cast<int64_t>(q.Wf);
  float acc[kSplitJ], sc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < kSplitJ; ++j) acc[j] = 0.f;
#pragma unroll 2
  for (int p = 0; p < q.Pt; ++p) {
    const float* pr = pt + static_cast<int64_t>(p) * q.Wt;
    float v[kSplitJ], u[4];
#pragma unroll
    for (int j = 0; j < kSplitJ; ++j) {
      const int f = tid + NT * j;
      v[j] = f < D3 ? pr[f] : 0.f;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) u[c] = pr[D3 + c];  // (a broadcast: every lane the same word)
#pragma unroll
    for (int j = 0; j < kSplitJ; ++j) acc[j] += v[j];
#pragma unroll
    for (int c = 0; c < 4; ++c) sc[c] += u[c];
  }
#pragma unroll 2
  for (int p = 0; p < q.Pf; ++p) {
    const float* pr = pf + static_cast<int64_t>(p) * q.Wf - D3;
    float v[kSplitJ];
#pragma unroll
    for (int j = 0; j < kSplitJ; ++j) {
      const int f = tid + NT * j;
      v[j] = (f >= D3 && f < W) ? pr[f] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < kSplitJ; ++j) acc[j] += v[j];
  }
  const float cnt = sc[0], sw = sc[1], c0 = sc[2], w0 = sc[3];
  float cmx0 = 0.f, cmx1 = 0.f, smax = 0.f;
#pragma unroll
  for (int j = 0; j < kSplitJ; ++j) {
    const int f = tid + NT * j;
    if (f >= W) continue;
    float v = acc[j];
    if (f < a.D) {  // the weighted text sum: row 0 once for its c0 tokens (gather mode)
      const float e0 = (c0 > 0.f) ? a.table[f] : 0.f;
      v = fmaf(w0, e0, v);
      const float xf = v / cnt;
      a.num_out[i * a.D + f] = xf;
      if (f < NT) cmx0 = bmax(cmx0, fabsf(xf)); else cmx1 = bmax(cmx1, fabsf(xf));
      continue;
    }
    const int g = f - a.D;  // s column
    if (g < 2 * a.D) {
      const float e0 = (c0 > 0.f) ? a.table[g < a.D ? g : g - a.D] : 0.f;
      v = g < a.D ? fmaf(c0, e0, v) : fmaf(c0 * e0, e0, v);
    }
    smax = fmaxf(smax, fabsf(v));
    if (a.s_half) s_row[g] = v; else a.s_out[i * a.Kp + g] = v;
  }
  smax = wave_max(smax);
  if (lane == 0) s_m[wave] = smax;
  __syncthreads();
  float m = 0.f;
#pragma unroll
  for (int w = 0; w < NT / kWave; ++w) m = fmaxf(m, s_m[w]);
  const float rs = row_scale(m);
  if (a.s_half) {
    _Float16* hi = reinterpret_cast<_Float16*>(a.s_out) + i * 2 * static_cast<int64_t>(a.Kp);
    for (int f = tid; f < a.Kp; f += NT) {
      const float x = f < K ? s_row[f] * rs : 0.f;
      const _Float16 h = static_cast<_Float16>(x);
      hi[f] = h;
      hi[a.Kp + f] = static_cast<_Float16>(x - static_cast<float>(h));
    }
  } else {
    for (int f = K + tid; f < a.Kp; f += NT) a.s_out[i * a.Kp + f] = 0.f;
  }
  if (tid == 0) {
    if (cnt == 0.f && a.flag) atomicOr(a.flag, MMB_FLAG_ZERO_WEIGHTS);
    a.aux_out[i] = cnt;
    a.aux_out[a.N + i] = sw;
    a.aux_out[2 * a.N + i] = rs;
  }
  if (a.cmax_part) {
    float* pr = a.cmax_part + i * a.D;
    if (tid < a.D) pr[tid] = cmx0;
    if (tid + NT < a.D) pr[tid + NT] = cmx1;
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

// Per-utterance sums of the wave-per-utterance kernels (utt_wave_kernel,
// utt_fused_kernel): lane t stages token t, the frame loop broadcasts it with
// v_readlane, lane l owns float4 columns l + 64 c of every row.
template <int CT, int CA, int CV>
struct UttSums {
  float4 num[CT], sx[CT], sxx[CT], sa[CA], saa[CA], sv[CV], svv[CV];
  float cnt, sw;
};

template <bool MM2, int CT, int CA, int CV, int UNR, bool NT, bool SPLIT>
__device__ __forceinline__ void utt_sums(const StreamArgs& a, int64_t i, int lane,
                                         UttSums<CT, CA, CV>& u) {
  const int UT = a.D >> 2, UA = a.A >> 2, UV = a.Vd >> 2;
  const float* tsrc = a.ids ? a.table : a.text_dense;
  const float* esrc = a.ids ? a.table : a.emb_dense;
  constexpr bool split_emb = MM2 && SPLIT;  // weighted sum over a different dense tensor
  const bool gather = a.ids != nullptr;
  // stage: lane t <- token t (row id or -1, weight)
  int rid = -1;
  float w = 0.f;
  if (lane < a.L) {
    int64_t off;
    stage_token(a, i, lane, off, w);
    rid = off < 0 ? -1 : (gather ? static_cast<int>(off / a.D) : lane);
  }
  u.cnt = wave_sum((w != 0.f) ? 1.f : 0.f);
  u.sw = wave_sum(w);
  // every weight 0: x is 0/0 = NaN (numpy's answer); the reference's
  // TruncatedSVD then rejects the split -- report it through the flag word
  if (lane == 0 && u.cnt == 0.f && a.flag) atomicOr(a.flag, MMB_FLAG_ZERO_WEIGHTS);

  float4 (&num)[CT] = u.num;
  float4 (&sx)[CT] = u.sx;
  float4 (&sxx)[CT] = u.sxx;
  float4 (&sa)[CA] = u.sa;
  float4 (&saa)[CA] = u.saa;
  float4 (&sv)[CV] = u.sv;
  float4 (&svv)[CV] = u.svv;
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
}

template <bool MM2, int CT, int CA, int CV, int UNR = 2, bool NT = false, bool SPLIT = false,
          bool NTS = false, int OCC = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void utt_wave_kernel(
    StreamArgs a) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wid = static_cast<int64_t>(blockIdx.x) * (blockDim.x / kWave) + threadIdx.x / kWave;
  const int64_t nw = static_cast<int64_t>(gridDim.x) * (blockDim.x / kWave);
  const int UT = a.D >> 2, UA = a.A >> 2, UV = a.Vd >> 2;

  float4 cmx[CT];  // running max |x| of this lane's columns (MMB2, mmb_gram_i8)
#pragma unroll
  for (int c = 0; c < CT; ++c) cmx[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = wid; i < a.N; i += nw) {
    UttSums<CT, CA, CV> u;
    utt_sums<MM2, CT, CA, CV, UNR, NT, SPLIT>(a, i, lane, u);
    const float cnt = u.cnt, sw = u.sw;
    float4 (&num)[CT] = u.num;
    float4 (&sx)[CT] = u.sx;
    float4 (&sxx)[CT] = u.sxx;
    float4 (&sa)[CA] = u.sa;
    float4 (&saa)[CA] = u.saa;
    float4 (&sv)[CV] = u.sv;
    float4 (&svv)[CV] = u.svv;

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
          cmx[c] = bmax4(cmx[c], xr);
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

// ------------------------------------------------------ narrow-frame stream
// MMB2 stream kernel for narrow frame rows (MOSI: COVAREP A = 76, FACET
// Vd = 48 -- 19 and 12 float4 units).  utt_wave_kernel gives every frame row
// its own wave-instruction, so at these widths 19 / 12 of the 64 lanes load
// (304 / 192 B per instruction) and a wave moves ~2 KB per HBM round trip:
// latency-bound at ~2.9 TB/s.  Here a wave-instruction covers P = 64 / U
// consecutive frame rows (lane -> frame slot f = lane / U, unit c = lane % U:
// 3 rows = 912 contiguous bytes of audio, 5 rows = 960 B of visual; lanes past
// P U load a duplicate), and ALL of an utterance's frame instructions (7 + 4
// at T = 20) are issued together, before its text groups: one HBM round trip
// per utterance for ~10 KB.  The token ids of the next utterance are loaded
// one utterance ahead and its weights gathered before the loop turns, so a
// text group waits for nothing but the (L2-resident at MOSI's V = 3016) table
// rows.  (The last iteration resolves its own ids a second time: an
// out-of-range id sets the same flag bit again.)
// Sums: the text sums (and so x, aux's count and weight sum, the column
// bounds) are utt_wave_kernel's operations in its order: bit-identical.  The
// frame sums (FR = 1, the product) are per-lane partials over the rows of one
// slot (f, f + P, f + 2P, ...) added slot 0 + 1 + ... at the end -- another
// f32 summation order than the wave kernel's t = 0, 1, ... (within f32
// rounding of it; the reference's torch sum over T fixes no order either).
// FR = 0 gathers every frame across the packed lanes (ds_bpermute) in t order
// instead: bit-identical to the wave kernel, 0.5 ms slower at MOSI (r03z).
// GA / GV: frame instructions per modality issued at once (7 + 4 = all of a
// T = 20 MOSI utterance; longer utterances take further groups after the text)
// ABL (tools build, timing-only ablations with wrong outputs): bit 0 skips the
// text rows, bit 1 the frames, bit 2 the row stores (kept live behind a test
// no value passes)
// FR: 0 = frames gathered frame by frame (ds_bpermute, the wave kernel's
// order), 1 = per-lane slot partials combined slot 0 + 1 + ... at the end.
// ORD: 0 = utterances round robin over the waves, 1 = a contiguous range per
// wave (neighbouring x / s / aux rows written by one wave: whole lines).
template <int CT, int UNR, int GA_MAX, int GV_MAX, int OCC = 2, int ABL = 0, int FR = 0, int ORD = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void utt_narrow_kernel(StreamArgs a) {
  const int lane = threadIdx.x & (kWave - 1);
  // the wave index made visibly wave-uniform: utterance bases stay in SGPRs
  const int64_t wid = static_cast<int64_t>(blockIdx.x) * (blockDim.x / kWave) +
                      __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t nw = static_cast<int64_t>(gridDim.x) * (blockDim.x / kWave);
  const int L = a.L, D = a.D;
  const int UT = D >> 2, UA = a.A >> 2, UV = a.Vd >> 2;
  const int PA = kWave / UA, PV = kWave / UV;  // frame rows per instruction (>= 2)
  const int GA = (L + PA - 1) / PA, GV = (L + PV - 1) / PV;
  // Loads go through buffer descriptors: a scalar offset per row / per packed
  // instruction and a fixed per-lane column offset -- no 64-bit address
  // arithmetic in VGPRs.  A row id < 0 (out of range, flagged) reads past the
  // table's record count, which returns zeros (a zero row, as the wave
  // kernel's select).  Text column offsets clamped into the row (lanes past
  // unit 74 read a duplicate the L1 coalesces and never store it).
  int vt[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) vt[c] = 16 * min(lane + kWave * c, UT - 1);
  const int tbytes = static_cast<int>(a.V * D * 4);
  const auto trsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.table), 0, tbytes, 0x00020000);
  // lane f U + c of a packed frame instruction: frame row f, unit c
  const int voa = ((lane / UA) * a.A + 4 * (lane % UA)) * 4;
  const int vov = ((lane / UV) * a.Vd + 4 * (lane % UV)) * 4;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 cmx[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) cmx[c] = z4;

  // token t of utterance i on lane t: the raw id (prefetched one utterance
  // ahead), then stage_token's semantics
  auto ld_id = [&](int64_t i) -> int { return (i < a.N && lane < L) ? a.ids[i * L + lane] : -1; };
  // (the weight gather is issued here and first waited for by the text loop,
  // behind the frame loads: the wave sums of the weights come after the text;
  // an id outside [0, V) -- a negative one wraps for its ROW only -- reads
  // past the weight table's record count: weight 0 with no select)
  const auto wrsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.wtab), 0,
                                                       static_cast<int>(a.V * 4), 0x00020000);
  auto resolve = [&](int raw, int& rid, float& w) {
    rid = -1;
    w = 0.f;
    if (lane < L) {
      int64_t id = raw;
      const bool in = id >= 0 && id < a.V;
      w = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                        wrsrc, in ? static_cast<int>(id) * 4 : static_cast<int>(a.V * 4), 0, 0));
      if (id < 0) id += a.V;
      if (id < 0 || id >= a.V) {
        if (a.flag) atomicOr(a.flag, MMB_FLAG_ID_RANGE);
      } else {
        rid = static_cast<int>(id);
      }
    }
  };
  const int64_t chunk = (a.N + nw - 1) / nw;
  const int64_t i_beg = ORD ? wid * chunk : wid;
  const int64_t i_end = ORD ? min(a.N, i_beg + chunk) : a.N;
  const int64_t i_step = ORD ? 1 : nw;
  // The next utterance's ids are loaded at the top of an iteration and
  // resolved (row ids, weight gather issued) at its end BEFORE its row stores:
  // with loads and stores both pending, gfx9's one vmcnt counter makes any
  // wait a wait for everything (s_waitcnt vmcnt(0)), so an iteration that
  // began by waiting for its ids waited for the previous row's stores too.
  int rid_n, raw = -1;
  float w_n;
  resolve(i_beg < i_end ? ld_id(i_beg) : -1, rid_n, w_n);
  for (int64_t i = i_beg; i < i_end; i += i_step) {
    const int rid = rid_n;
    float w = w_n;
    if (i + i_step < i_end) raw = ld_id(i + i_step);  // in flight through this utterance

    // frames: the first GA_MAX / GV_MAX packed instructions per modality
    // issued before the text loop (rows past L read zeros past the record count)
    const auto arsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.audio + i * L * a.A), 0,
                                                         L * a.A * 4, 0x00020000);
    const auto vrsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.visual + i * L * a.Vd), 0,
                                                         L * a.Vd * 4, 0x00020000);
    float4 sa = z4, saa = z4, sv = z4, svv = z4;
    auto frames = [&](auto gmax, auto rsrc, int vo, int W, int U, int P, int g0, float4& s1, float4& s2) {
      constexpr int GM = decltype(gmax)::value;
      float4 v[GM > 0 ? GM : 1];
#pragma unroll
      for (int g = 0; g < GM; ++g)  // non-temporal: read-once streams
        v[g] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo, (g0 + g) * P * W * 4, 2));
      // frame t = g P + q of unit c sits on lane q U + c: lane c < U adds the
      // frames in order t = 0, 1, ... (ds_bpermute), the order of
      // utt_wave_kernel / the fused kernel's frame_piece -- bit-identical sums
      const int c = lane % U;
      const bool mine = lane < P * U;
      return [=, &s1, &s2]() {
#pragma unroll
        for (int g = 0; g < GM; ++g) {
          if constexpr (FR == 1) {  // rows past L read zeros
            if (mine) {
              add4(s1, v[g]);
              sq4(s2, v[g]);
            }
            continue;
          }
          for (int q = 0; q < P; ++q) {
            if ((g0 + g) * P + q >= L) break;
            const int src = min(q * U + c, kWave - 1);
            float4 x;
            x.x = __shfl(v[g].x, src, kWave);
            x.y = __shfl(v[g].y, src, kWave);
            x.z = __shfl(v[g].z, src, kWave);
            x.w = __shfl(v[g].w, src, kWave);
            add4(s1, x);
            sq4(s2, x);
          }
        }
      };
    };
    using GAc = std::integral_constant<int, GA_MAX>;
    using GVc = std::integral_constant<int, GV_MAX>;
    using G0 = std::integral_constant<int, 0>;
    auto acc_a = frames(std::conditional_t<(ABL & 2) != 0, G0, GAc>{}, arsrc, voa, a.A, UA, PA, 0, sa, saa);
    auto acc_v = frames(std::conditional_t<(ABL & 2) != 0, G0, GVc>{}, vrsrc, vov, a.Vd, UV, PV, 0, sv, svv);

    // text: utt_sums' text half, the same operations in the same order
    float4 num[CT], sx[CT], sxx[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c) num[c] = sx[c] = sxx[c] = z4;
    auto row = [&](int t, float4 (&v)[CT]) {
      const int r = __builtin_amdgcn_readlane(rid, t);
      const int so = r >= 0 ? r * D * 4 : tbytes;  // out of range: a zero row
#pragma unroll
      for (int c = 0; c < CT; ++c)
        v[c] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(trsrc, vt[c], so, 0));
    };
    // (the weight is read at accumulation: its gather is waited for there)
    auto accum = [&](int t, const float4 (&v)[CT]) {
      const float wt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), t));
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        fma4(num[c], wt, v[c]);
        add4(sx[c], v[c]);
        sq4(sxx[c], v[c]);
      }
    };
    int t = (ABL & 1) ? L : 0;
    for (; t + UNR <= L; t += UNR) {
      float4 v[UNR][CT];
#pragma unroll
      for (int u = 0; u < UNR; ++u) row(t + u, v[u]);
#pragma unroll
      for (int u = 0; u < UNR; ++u) accum(t + u, v[u]);
    }
    for (; t < L; ++t) {
      float4 v[CT];
      row(t, v);
      accum(t, v);
    }
    acc_a();
    acc_v();
    const float cnt = wave_sum((w != 0.f) ? 1.f : 0.f);
    const float sw = wave_sum(w);
    if (lane == 0 && cnt == 0.f && a.flag) atomicOr(a.flag, MMB_FLAG_ZERO_WEIGHTS);
    if constexpr ((ABL & 2) == 0)
    for (int g0 = GA_MAX; g0 < GA; g0 += GA_MAX) frames(GAc{}, arsrc, voa, a.A, UA, PA, g0, sa, saa)();
    if constexpr ((ABL & 2) == 0)
    for (int g0 = GV_MAX; g0 < GV; g0 += GV_MAX) frames(GVc{}, vrsrc, vov, a.Vd, UV, PV, g0, sv, svv)();
    if constexpr (FR == 1) {  // slot partials -> unit totals on lanes < U, slot 0 + 1 + ...
      auto slots = [&](float4& acc, int U, int P) {
        float4 r = acc;
        for (int f = 1; f < P; ++f) {
          const int src = min(lane + f * U, kWave - 1);
          float4 o;
          o.x = __shfl(acc.x, src, kWave);
          o.y = __shfl(acc.y, src, kWave);
          o.z = __shfl(acc.z, src, kWave);
          o.w = __shfl(acc.w, src, kWave);
          add4(r, o);
        }
        acc = r;
      };
      slots(sa, UA, PA);
      slots(saa, UA, PA);
      slots(sv, UV, PV);
      slots(svv, UV, PV);
    }
    // lanes past a modality's units summed duplicates: keep them out of the row max
    if (lane >= UA) sa = saa = z4;
    if (lane >= UV) sv = svv = z4;

    float m = fmaxf(fmaxf(amax4(sa), amax4(saa)), fmaxf(amax4(sv), amax4(svv)));
#pragma unroll
    for (int c = 0; c < CT; ++c) m = fmaxf(m, fmaxf(amax4(sx[c]), amax4(sxx[c])));
    const float rs = row_scale(wave_max(m));
    resolve(raw, rid_n, w_n);  // the next utterance's (see above)
    if ((ABL & 4) != 0 && rs != 3.f) continue;  // (never 3: a power of two)
    _Float16* hrow = reinterpret_cast<_Float16*>(a.s_out) + i * 2 * a.Kp;
    auto put = [&](int f, float4 v) { split_store4<false>(hrow + f, hrow + a.Kp + f, v, rs); };
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const int u = lane + kWave * c;
      if (u < UT) {
        const float4 xr = div4(num[c], cnt);
        st4(a.num_out + i * D + 4 * u, xr);  // x = the a2 row
        cmx[c] = bmax4(cmx[c], xr);
        put(4 * u, sx[c]);
        put(D + 4 * u, sxx[c]);
      }
    }
    if (lane < UA) {
      put(2 * D + 4 * lane, sa);
      put(2 * D + a.A + 4 * lane, saa);
    }
    if (lane < UV) {
      put(2 * (D + a.A) + 4 * lane, sv);
      put(2 * (D + a.A) + a.Vd + 4 * lane, svv);
    }
    for (int f = 2 * (D + a.A + a.Vd) + lane; f < a.Kp; f += kWave)
      hrow[f] = hrow[a.Kp + f] = static_cast<_Float16>(0.f);
    if (lane == 0) {
      a.aux_out[i] = cnt;  // planar [3][N]: count | sum w | fp16 row scale
      a.aux_out[a.N + i] = sw;
      a.aux_out[2 * a.N + i] = rs;
    }
  }
  if (a.cmax_part) {  // this wave's column bounds (mmb_gram_i8)
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const int u = lane + kWave * c;
      if (u < UT) st4(a.cmax_part + wid * D + 4 * u, cmx[c]);
    }
  }
}

// the narrow kernel's shapes: gathered ids with the weight table, fp16 s,
// text rows of 65-128 float4 units (CT = 2; the MOSI / bench D = 300), frame
// rows of at most 32 units (two or more rows per instruction), T <= 64
static bool narrow_ok(const StreamArgs& a) {
  return a.ids && a.wtab && !a.w_dense && a.s_half && a.D > 256 && a.D <= 512 &&
         a.A <= 128 && a.Vd <= 128 && a.L <= kWave && a.V * a.D * 4 < (int64_t{1} << 31);
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
      for (int u = 0; u < 8; ++u) mm[u] = bmax(mm[u], part[static_cast<int64_t>(r + 16 * u) * D + f]);
    }
    for (; r < P; r += 16) mm[0] = bmax(mm[0], part[static_cast<int64_t>(r) * D + f]);
#pragma unroll
    for (int u = 0; u < 8; ++u) m = bmax(m, mm[u]);
  }
  s_m[g][c] = m;
  __syncthreads();
  if (g == 0 && f < D) {
    for (int k = 1; k < 16; ++k) m = bmax(m, s_m[k][c]);
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
// Read per launch (in-process A/B sweeps flip it).  Bit 3 (policy 13):
// the default variant compiled for two waves per SIMD (amdgpu_waves_per_eu).
// The sweep knobs (this one, MMB_STREAM_GRID_MULT, the fused kernel's
// MMB_FUSED_*, the projection's MMB_PROJ_*, MMB_GRAM_DIAG, MMB_PC_REMOVE_R)
// exist only in the tools build (libmmb_diag.so, tools/diag/): at each
// MMB_HOOK_* point below the product library compiles its default and reads
// no environment variable.

template <bool MM2, int CT, int CA, int CV, int UNR, bool NT, bool NTS, int OCC = 1>
static void launch_wave_v(const StreamArgs& a, int grid, hipStream_t stream) {
  if (MM2 && a.ids == nullptr && a.emb_dense != a.text_dense) {
    utt_wave_kernel<MM2, CT, CA, CV, UNR, NT, true, NTS, OCC><<<grid, 256, 0, stream>>>(a);
  } else {
    utt_wave_kernel<MM2, CT, CA, CV, UNR, NT, false, NTS, OCC><<<grid, 256, 0, stream>>>(a);
  }
}

// Workgroups per CU of the grid-stride wave kernel: 2 = exactly the resident
// waves at its occupancy (2 waves / SIMD), one even share of utterances per
// wave.  Measured (tools/grid_sweep.sh, MI355X): 2/4/8/16/32 = 20.88/20.94/
// 21.04/21.01/21.18 ms.  MMB_STREAM_GRID_MULT overrides it (tools build).
#ifndef MMB_HOOK_STREAM_GRID_MULT
#define MMB_HOOK_STREAM_GRID_MULT 2
#endif
static int stream_grid_mult() { return MMB_HOOK_STREAM_GRID_MULT; }

// rows of the column-bound partials (one per wave / workgroup of a launch)
constexpr int kCmaxRows = 8192;

// Narrow-frame kernel variant (MMB_STREAM_NARROW, tools build; the product
// runs 10).  Measured (r03z, MOSI 1M x 20, A = 76, Vd = 48, V = 3016, same
// process, stream kernel ms): utt_wave_kernel (0) 5.04; frames gathered frame
// by frame, 4 / 5 text rows per load group (2 / 3) 4.41 / 4.34; 10 rows at
// occupancy 2 (4) 4.74; 5 rows forced to 4 waves per SIMD (5, spills) 5.15;
// slot-partial frame sums (10) 3.81; contiguous utterance ranges per wave (11
// = 3, 12 = 10 with it) no change; 8-row groups (13, occupancy 2) 4.41;
// not kept (removed after measuring): the text rows' last column load on
// its 11 live lanes only 3.87 vs 3.87; the last 11 units of 5 text rows in
// ONE packed instruction (16 instead of 40 text loads per utterance) 3.89 vs
// 3.85 with 5-row groups, 4.44 with 10; the next utterance's ids resolved
// before the row stores (kept: no iteration starts by waiting for the
// previous row's stores) 3.87 vs 3.81; slot partials with 7 / 10 text rows
// per group (occupancy 2) 4.31 / 3.90, 7 rows forced to occupancy 3 (7 VGPRs
// spilled) 4.09 vs 3.84.
// Timing-only ablations of 3 (wrong rows): no text 3.14 (6), no frames 2.32
// (7), no row stores 3.61 (8), neither text nor frames 1.41 (9).
#ifndef MMB_HOOK_NARROW_VARIANT
#define MMB_HOOK_NARROW_VARIANT 10
#endif
static int narrow_variant() { return MMB_HOOK_NARROW_VARIANT; }

static int launch_narrow(const StreamArgs& a, hipStream_t stream, int* parts) {
  const int var = narrow_variant();
  // resident workgroups of 4 waves per CU at each variant's occupancy
  const int per_cu = (var == 4 || var == 13) ? 2 : var == 5 ? 4 : 3;
  const int64_t blocks = ceil_div(a.N, 4);
  int grid_cap = per_cu * stream_cu_count(stream);
  if (a.cmax_part && grid_cap > kCmaxRows / 4) grid_cap = kCmaxRows / 4;
  const int grid = static_cast<int>(blocks < grid_cap ? blocks : grid_cap);
  if (parts) *parts = grid * 4;
#ifndef MMB_HOOK_NARROW_LAUNCH  // (tools/diag: the variant sweep)
#define MMB_HOOK_NARROW_LAUNCH false
#endif
  if (!(MMB_HOOK_NARROW_LAUNCH)) utt_narrow_kernel<2, 5, 7, 4, 2, 0, 1, 0><<<grid, 256, 0, stream>>>(a);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

template <bool MM2, int CT, int CA, int CV>
static int launch_wave(const StreamArgs& a, hipStream_t stream, int* parts = nullptr) {
  if (MM2 && narrow_ok(a) && narrow_variant() > 0) return launch_narrow(a, stream, parts);
  const int64_t blocks = ceil_div(a.N, 4);
  int grid_cap = stream_grid_mult() * stream_cu_count(stream);
  if (a.cmax_part && grid_cap > kCmaxRows / 4) grid_cap = kCmaxRows / 4;
  const int grid = static_cast<int>(blocks < grid_cap ? blocks : grid_cap);
  if (parts) *parts = grid * 4;
#ifndef MMB_HOOK_WAVE_LAUNCH  // (tools/diag: the stream-policy sweep)
#define MMB_HOOK_WAVE_LAUNCH false
#endif
  if (!(MMB_HOOK_WAVE_LAUNCH)) {
    if constexpr (MM2) {  // policy 5: 4-frame groups, non-temporal frame loads
      launch_wave_v<MM2, CT, CA, CV, 4, true, false>(a, grid, stream);
    } else {
      launch_wave_v<MM2, CT, CA, CV, 2, false, false>(a, grid, stream);
    }
  }
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

// ---------------------------------------------------------------- fused step
// Stream + projection in ONE kernel (the bench step's MMB2 path): the frame
// sums s of an utterance never leave the chip.  One persistent workgroup per
// CU, 8 waves (two per SIMD):
//   waves 0-3 (streamers)  stream the utterances of a batch of 48 consecutive
//     rows modality by modality (text pass: gathered rows, the a2 row x, aux,
//     the column bounds; then the audio pass, then the visual pass), leaving
//     each (row, modality) piece of sums -- [Sx_m | Sxx_m], fp16 hi | lo of
//     the piece scaled by a power of two -- in an LDS ring slot
//   waves 4-7 (projectors) per piece of a batch: [48, 2 w_m] x [2 w_m, 320]
//     fp16 x3 products (v_mfma_f32_16x16x32_f16, 3 row tiles x 5 column tiles
//     per wave) with A from the ring and B straight from L2 (the piece-ordered
//     weight split, mmb_mm2_split_pieces); the accumulators carry over from
//     piece to piece (rescaled exactly by the ratio of the pieces' power-of-2
//     scales); after the third piece the epilogue of mm2_project_x3b_kernel
//     (text sum, total weight, L2 norm) on 80 columns per wave, the row totals
//     and norms exchanged through LDS
// Why piece-major 48-row batches: every batch re-reads the whole 2.3 MB weight
// image from L2, and that L2 traffic is what competes with the HBM stream
// (r02 ablation: 16-row whole-row batches -- 146 GB of L2 reads per 1M rows --
// took the kernel from 20.2 ms, stream alone, to 26.0 ms).  LDS cannot hold 48
// whole rows (7.3 KB each), but it holds 60 single-modality pieces (2.5 KB):
// the projectors read piece m of the batch while the streamers fill piece m+1.
// Hand-over through LDS counters (the two groups run at their own pace):
//   fill[p % 4]  piece-rows of piece p (= 3 batch + modality) written
//   consumed     projector waves done reading a piece (the streamers wait
//                before overwriting a slot)
//   pbar         the projectors' own exchange points (two per batch)
// Every wait is bounded: after ~0.5 s without progress it raises
// MMB_FLAG_SYNC_TIMEOUT and every later wait returns at once, so a broken
// hand-over ends the kernel (wrong rows, flagged) instead of hanging the GPU.
constexpr int kGR = 48;                 // rows per batch
constexpr int kGRT = kGR / 16;          // MFMA row tiles per batch
constexpr int kGSlots = 62;             // ring slots (piece-rows), at most (fused_lds_bytes)
constexpr int kGUnits = 80;             // 16-byte units per plane (piece <= 640 sums; XOR-16 headroom)
constexpr int kGPlane = kGUnits * 8;    // halves per plane
constexpr int kGSlot = 2 * kGPlane;     // halves per slot (hi | lo)
constexpr int kFTiles = 5;              // 16-column tiles per projector (ldw = 320)
constexpr int kFLdw = 320;
constexpr int kFThreads = 512;
// ring [SL slots] | irs [SL] | counters [8] | cnt, tw [2][48] each | tot [2][48] | ssq [2][4][48]
// | the dynamic schedule's batch and tag slots [8] each
__host__ __device__ constexpr size_t fused_lds_bytes(int sl) {
  return static_cast<size_t>(sl) * kGSlot * sizeof(_Float16) + sl * 4 + 8 * 4 + 2 * 2 * kGR * 4 +
         2 * kGR * 4 + 2 * 4 * kGR * 4 + 2 * 8 * 4;
}
static_assert(fused_lds_bytes(kGSlots) <= 160 * 1024, "fused ring exceeds LDS");
static_assert((kGSlot * 2) % 256 == 0 && (kGPlane * 2) % 256 == 0,
              "slot and plane strides keep the XOR swizzle conflict-free");

struct FusedArgs {
  StreamArgs s;
  const _Float16* img;     // piece-ordered B image (mmb_mm2_split_pieces), ldw = 320
  const float* col_inv;    // [320] 1 / column scale
  const float* c0;         // [320]
  float* out;              // mmb2 [N][D]
  int64_t nb;              // batches = ceil(N / 48)
  int kq[3];               // padded piece widths (multiples of 32)
  int balanced;            // rows past the last full round split evenly over the workgroups
  unsigned* sched;         // the launch's batch counter, zero at launch (nullable: static order)
  int64_t big, nu;         // dynamic order: units [0, big) are 48-row batches, the rest 12 rows
};

// the bounded waits' budget (tools/diag: a test shortens it to drive the
// timeout path)
#ifndef MMB_HOOK_FUSED_WAIT_ITERS
#define MMB_HOOK_FUSED_WAIT_ITERS (1 << 23)
#endif
__device__ __forceinline__ int fused_wait_iters() { return MMB_HOOK_FUSED_WAIT_ITERS; }

// bounded wait for *p >= target (workgroup scope); false once anything timed out
__device__ __forceinline__ bool fused_wait(int* p, int target, int* abort_flag, int32_t* gflag) {
  const int iters = fused_wait_iters();
  for (int it = 0; it < iters; ++it) {
    if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      return true;
    }
    if (__hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
    __builtin_amdgcn_s_sleep(2);
  }
  __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (gflag && (threadIdx.x & (kWave - 1)) == 0) atomicOr(gflag, MMB_FLAG_SYNC_TIMEOUT);
  return false;
}
// one increment per wave, ordered after this wave's earlier LDS / global writes
__device__ __forceinline__ void fused_signal(int* p) {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if ((threadIdx.x & (kWave - 1)) == 0)
    __hip_atomic_fetch_add(p, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// the same without waiting for this wave's global loads / stores (the
// pipelined streamer: its next frame groups stay in flight); the LDS writes it
// orders are complete before the increment (lgkmcnt), and LDS operations of
// one wave retire in order
__device__ __forceinline__ void fused_signal_lds(int* p) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if ((threadIdx.x & (kWave - 1)) == 0)
    __hip_atomic_fetch_add(p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Text piece of utterance i (one wave, lane l owns float4 columns l, l + 64):
// the weighted sum num = sum_t w_t E_t, Sx, Sxx of the gathered rows, the
// count of nonzero weights and their sum (utt_sums' text half).
template <int UNR>
__device__ __forceinline__ void text_piece(const StreamArgs& a, int64_t i, int lane, float4 (&num)[2],
                                           float4 (&sx)[2], float4 (&sxx)[2], float& cnt, float& sw) {
  const int UT = a.D >> 2;
  const float* tsrc = a.ids ? a.table : a.text_dense;
  const bool gather = a.ids != nullptr;
  int rid = -1;
  float w = 0.f;
  if (lane < a.L) {
    int64_t off;
    stage_token(a, i, lane, off, w);
    rid = off < 0 ? -1 : (gather ? static_cast<int>(off / a.D) : lane);
  }
  cnt = wave_sum((w != 0.f) ? 1.f : 0.f);
  sw = wave_sum_dpp_f32(w);  // DPP rows, as the pipelined streamers (bit-identical variants)
  if (lane == 0 && cnt == 0.f && a.flag) atomicOr(a.flag, MMB_FLAG_ZERO_WEIGHTS);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int c = 0; c < 2; ++c) num[c] = sx[c] = sxx[c] = z4;
  const int64_t dbase = i * a.L;
  const int ct0 = 4 * min(lane, UT - 1), ct1 = 4 * min(lane + kWave, UT - 1);
  auto frame = [&](int t, float4 (&v)[2], float& wt, bool& ok) {
    const int r = __builtin_amdgcn_readlane(rid, t);
    wt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), t));
    ok = r >= 0;
    const int64_t o = (gather ? static_cast<int64_t>(ok ? r : 0) : dbase + t) * a.D;
    v[0] = ld4(tsrc + o + ct0);
    v[1] = ld4(tsrc + o + ct1);
  };
  auto accum = [&](const float4 (&v)[2], float wt, bool ok) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float4 x = ok ? v[c] : z4;
      fma4(num[c], wt, x);
      add4(sx[c], x);
      sq4(sxx[c], x);
    }
  };
  int t = 0;
  for (; t + UNR <= a.L; t += UNR) {
    float4 v[UNR][2];
    float wt[UNR];
    bool ok[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) frame(t + u, v[u], wt[u], ok[u]);
#pragma unroll
    for (int u = 0; u < UNR; ++u) accum(v[u], wt[u], ok[u]);
  }
  for (; t + 4 <= a.L; t += 4) {  // tail groups: keep loads in flight
    float4 v[4][2];
    float wt[4];
    bool ok[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) frame(t + u, v[u], wt[u], ok[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) accum(v[u], wt[u], ok[u]);
  }
  for (; t < a.L; ++t) {
    float4 v[2];
    float wt;
    bool ok;
    frame(t, v, wt, ok);
    accum(v, wt, ok);
  }
}

// Audio / visual piece: Sx, Sxx over the L frames [L][W] at `base`
// (read-once streams: non-temporal loads).
template <int UNR, bool NT>
__device__ __forceinline__ void frame_piece(const float* base, int W, int L, int lane,
                                            float4 (&sx)[2], float4 (&sxx)[2]) {
  const int UW = W >> 2;
  const int c0 = 4 * min(lane, UW - 1), c1 = 4 * min(lane + kWave, UW - 1);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  sx[0] = sx[1] = sxx[0] = sxx[1] = z4;
  int t = 0;
  for (; t + UNR <= L; t += UNR) {
    float4 v[UNR][2];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      v[u][0] = ldnt4<NT>(base + static_cast<int64_t>(t + u) * W + c0);
      v[u][1] = ldnt4<NT>(base + static_cast<int64_t>(t + u) * W + c1);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        add4(sx[c], v[u][c]);
        sq4(sxx[c], v[u][c]);
      }
  }
  for (; t + 4 <= L; t += 4) {  // tail groups: keep loads in flight
    float4 v[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      v[u][0] = ldnt4<NT>(base + static_cast<int64_t>(t + u) * W + c0);
      v[u][1] = ldnt4<NT>(base + static_cast<int64_t>(t + u) * W + c1);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        add4(sx[c], v[u][c]);
        sq4(sxx[c], v[u][c]);
      }
  }
  for (; t < L; ++t) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float4 x = ldnt4<NT>(base + static_cast<int64_t>(t) * W + (c ? c1 : c0));
      add4(sx[c], x);
      sq4(sxx[c], x);
    }
  }
}

// DIAG (timing-only builds, MMB_FUSED_DIAG; wrong MMB2 rows): bit 7 the
// epilogue without its x re-read, bit 8 without its MMB2 stores; bit 4 every B
// chunk read from the piece's first chunk, bit 5 no B loads; bit 0 the
// projectors only hand the slots back (no loads, MFMAs or epilogue), bit 1
// no MFMAs (B loads kept live), bit 2 no epilogue, bit 3 the streamers skip
// the frames (constant sums: the projectors alone)
// per-workgroup wall-clock marks of the fused kernel (tools/diag defines
// them: mmb_diag_fused_probe)
#ifndef FUSED_PROBE
#define FUSED_PROBE(slot) \
  do {                    \
  } while (0)
#endif

template <int UNR, bool NT, int DIAG = 0, int PIPE = 0, int SL = kGSlots>
__global__ __launch_bounds__(kFThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void utt_fused_kernel(
    FusedArgs f) {
  const StreamArgs& a = f.s;
  extern __shared__ __attribute__((aligned(16))) _Float16 flds[];
  _Float16* ring = flds;
  float* s_irs = reinterpret_cast<float*>(flds + SL * kGSlot);
  int* ctr = reinterpret_cast<int*>(s_irs + SL);   // fill[4], consumed, pbar, abort, -
  float* s_cnt = reinterpret_cast<float*>(ctr + 8);     // [2][48]
  float* s_tw = s_cnt + 2 * kGR;                        // [2][48]
  float* s_tot = s_tw + 2 * kGR;                        // [2][48]
  float* s_ssq = s_tot + 2 * kGR;                       // [2][4][48]
  int* s_bat = reinterpret_cast<int*>(s_ssq + 2 * 4 * kGR);  // [8] global batch of local batch j (slot j & 7)
  int* s_tag = s_bat + 8;                                // [8] j + 1 once slot j & 7 holds batch j
  int* fill = ctr;
  int* consumed = ctr + 4;
  int* pbar = ctr + 5;
  int* abort_flag = ctr + 6;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid >> 6;
  if (tid < 8) {
    ctr[tid] = 0;
    s_tag[tid] = 0;
  }
  if (tid == 0) FUSED_PROBE(0);
  __syncthreads();
  const int64_t N = a.N;
  const int G = gridDim.x;
  const int D = a.D;
  // This workgroup's batches of 48 rows: batch blockIdx.x + j G of the row
  // space (round robin: the CUs stream neighbouring rows -- contiguous
  // per-CU ranges measured 23.07 vs 22.32 ms).  With f.balanced the rows
  // past the last full round (N mod 48 G) are split evenly over the
  // workgroups instead of being whole batches of a few of them (a CU with
  // one batch more than another runs ~0.28 ms longer).
  const int64_t full = N / (static_cast<int64_t>(kGR) * G);  // full rounds
  // Dynamic schedule (r05; the pipelined streamer with a counter): local
  // batch j is whatever global batch the streamers' wave 0 drew from the
  // launch's counter for it (one batch ahead of its own use), so a CU that
  // streams faster takes more batches.  The static round robin left the
  // workgroups' finishing times 0.3-0.7 ms apart at 1M rows (the even XCDs
  // slower; tools/fused_balance.py, gpurun_out r05ab).  Neighbouring CUs
  // still draw neighbouring batches.
  const bool dyn = PIPE == 2 && f.sched != nullptr;
  auto batch = [&](int64_t j, int64_t& row0, int64_t& rend) -> bool {
    if (dyn) {
      int64_t u = blockIdx.x + j * G;  // local batches 0 and 1: the round robin's units
      if (j >= 2) {
        if (!fused_wait(&s_tag[j & 7], static_cast<int>(j) + 1, abort_flag, a.flag)) return false;
        u = s_bat[j & 7];
      }
      if (u >= f.nu) return false;
      // the last round's worth of rows in quarter batches: the end of the
      // kernel waits for one 12-row unit, not one 48-row batch (~0.3 ms)
      row0 = u < f.big ? u * kGR : f.big * kGR + (u - f.big) * (kGR / 4);
      rend = min<int64_t>(N, row0 + (u < f.big ? kGR : kGR / 4));
      return true;
    }
    if (f.balanced && j >= full) {
      if (j > full) return false;
      const int64_t t0 = full * kGR * G, tail = N - t0, b = blockIdx.x;
      const int64_t per = tail / G, rem = tail % G;
      row0 = t0 + b * per + (b < rem ? b : rem);
      rend = row0 + per + (b < rem ? 1 : 0);
      return row0 < rend;
    }
    const int64_t Bj = blockIdx.x + j * G;
    row0 = Bj * kGR;
    rend = min<int64_t>(N, row0 + kGR);
    return Bj < f.nb;
  };

  if (wave < 4) {
    // ------------------------------------------------------------ streamer
    const int wdt[3] = {a.D, a.A, a.Vd};
    float4 cmx[2];
    cmx[0] = cmx[1] = make_float4(0.f, 0.f, 0.f, 0.f);
    // Row q (utterance i) of batch j, modality m summed: its power-of-2 scale,
    // the text row's x / aux / column bounds, then the scaled fp16 hi | lo
    // sums into the ring slot (once the slot's previous piece-row was read by
    // every projector) and one fill increment.  DRAIN: the increment waits for
    // every earlier global access of this wave (the group-at-a-time streamer);
    // the pipelined streamer waits only for its LDS writes, its next loads
    // stay in flight (its x / aux stores are drained once per batch, before
    // the audio piece's first increment -- the projectors read x only after
    // the visual piece).
    auto finish_row = [&](auto drain_c, int64_t j, int m, int q, int64_t i, const float4 (&num)[2],
                          const float4 (&sx)[2], const float4 (&sxx)[2], float cnt, float sw) {
      const int W = wdt[m], U = W >> 2;
      const int p = 3 * static_cast<int>(j) + m;  // piece sequence number
      float mx = 0.f;
#pragma unroll
      for (int c = 0; c < 2; ++c) mx = fmaxf(mx, fmaxf(amax4(sx[c]), amax4(sxx[c])));
      const float rs = row_scale(wave_max_dpp_f32(mx));
      if (m == 0) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int uu = lane + kWave * c;
          if (uu < U) {
            const float4 xr = div4(num[c], cnt);
            st4(a.num_out + i * D + 4 * uu, xr);  // x = the a2 row
            cmx[c] = bmax4(cmx[c], xr);
          }
        }
        if (lane == 0) {
          a.aux_out[i] = cnt;  // planar [3][N]: count | sum w | text-piece scale
          a.aux_out[N + i] = sw;
          a.aux_out[2 * N + i] = rs;
          s_cnt[(j & 1) * kGR + q] = cnt;
          s_tw[(j & 1) * kGR + q] = sw;
        }
      }
      // the slot's previous piece-row (pos - 60) must have been read by every projector
      const int pos = p * kGR + q;
      const int slot = pos % SL;
      // (DIAG 64, timing only: never wait -- the ring's back-pressure removed)
      if ((DIAG & 64) == 0 && pos >= SL)
        fused_wait(consumed, ((pos - SL) / kGR + 1) * 4, abort_flag, a.flag);
      _Float16* srow = ring + slot * kGSlot;
      const int qx = q & 15;  // row within its MFMA row tile: the XOR swizzle key
      auto put = [&](int k, float4 v) {
        const float x4[4] = {v.x * rs, v.y * rs, v.z * rs, v.w * rs};
        h4 h, l;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          h[e] = static_cast<_Float16>(x4[e]);
          l[e] = static_cast<_Float16>(x4[e] - static_cast<float>(h[e]));
        }
        const int o = (((k >> 3) ^ qx) << 3) + (k & 7);
        *reinterpret_cast<h4*>(srow + o) = h;
        *reinterpret_cast<h4*>(srow + kGPlane + o) = l;
      };
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int uu = lane + kWave * c;
        if (uu < U) {
          put(4 * uu, sx[c]);
          put(W + 4 * uu, sxx[c]);
        }
      }
      for (int k = 2 * W + 4 * lane; k < f.kq[m]; k += 4 * kWave) put(k, make_float4(0.f, 0.f, 0.f, 0.f));
      if (lane == 0) s_irs[slot] = 1.f / rs;  // a power of two: exact
      if constexpr (decltype(drain_c)::value) {
        fused_signal(&fill[p & 3]);
      } else {
        fused_signal_lds(&fill[p & 3]);
      }
    };

    if constexpr (PIPE == 0) {
      for (int64_t j = 0;; ++j) {
        int64_t row0, rend;
        if (!batch(j, row0, rend)) break;
#pragma unroll 1
        for (int m = 0; m < 3; ++m) {
          const int W = wdt[m];
#pragma unroll 1
          for (int r = 0; r < kGR / 4; ++r) {
            const int q = wave + 4 * r;
            const int64_t i = row0 + q;
            if (i >= rend) break;
            float4 num[2], sx[2], sxx[2];
            float cnt = 0.f, sw = 0.f;
            if constexpr ((DIAG & 8) != 0) {
              const float4 o4 = make_float4(1.f, 1.f, 1.f, 1.f);
              num[0] = num[1] = sx[0] = sx[1] = sxx[0] = sxx[1] = o4;
              cnt = sw = 1.f;
            } else if (m == 0) {
              text_piece<UNR>(a, i, lane, num, sx, sxx, cnt, sw);
            } else {
              const float* base = m == 1 ? a.audio + i * a.L * a.A : a.visual + i * a.L * a.Vd;
              frame_piece<UNR, NT>(base, W, a.L, lane, sx, sxx);
            }
            finish_row(std::true_type{}, j, m, q, i, num, sx, sxx, cnt, sw);
          }
        }
      }
    } else {
      // Pipelined streamer: the (row, frame group) sequence of one (batch,
      // modality) piece -- this wave's rows i0 + 4 r, ceil(L / UNR) groups of
      // UNR frames each -- as ONE load pipeline two groups deep: group g + 1's
      // 2 UNR loads are issued before group g is summed (alternating register
      // sets b0 / b1; the compiler's counted vmcnt waits only for the older
      // group), so loads stay in flight across group and row boundaries where
      // the group-at-a-time streamer drained them.  Text rows: row r + 1's ids
      // are loaded while row r's first group is summed, its weights gathered
      // (wtab[id]) at the second -- the next row's first group is issued after
      // that (>= 3 groups per row, launch_fused).  Per lane the frames are
      // summed in the same order as text_piece / frame_piece: bit-identical.
      // (A pipeline running on across piece and batch boundaries, one issue /
      // consume pair for all three modalities, measured 29.4 vs 22.1 ms: the
      // shared register sets made the compiler drain every group, vmcnt(0).)
      const bool gather = a.ids != nullptr;
      const int L = a.L;
      // the wave index made visibly wave-uniform (SGPR): rows, loop bounds and
      // buffer descriptors derive from it (a descriptor in VGPRs would be
      // waterfall-looped around every load)
      const int uw = __builtin_amdgcn_readfirstlane(wave);
      auto tok_issue = [&](int64_t i, int& raw, float& wd) {
        raw = -1;
        wd = 0.f;
        if (lane < L) {
          const int64_t ft = i * L + lane;
          if (gather) raw = a.ids[ft];
          if (a.w_dense) wd = a.w_dense[ft];
        }
      };
      auto tok_resolve = [&](int raw, float wd, int& rid, float& w) {  // stage_token's semantics
        rid = -1;
        w = 0.f;
        if (lane < L) {
          if (gather) {
            int64_t id = raw;
            w = a.w_dense ? wd : ((id >= 0 && id < a.V) ? a.wtab[id] : 0.f);
            if (id < 0) id += a.V;
            if (id < 0 || id >= a.V) {
              if (a.flag) atomicOr(a.flag, MMB_FLAG_ID_RANGE);
              w = 0.f;
            } else {
              rid = static_cast<int>(id);
            }
          } else {
            w = wd;
            rid = lane;
          }
        }
      };
      auto piece = [&](auto text_c, int64_t j, int m, int64_t i0, int nrows) {
        constexpr bool TEXT = decltype(text_c)::value;
        const int W = wdt[m], UW = W >> 2;
        const int c0 = 4 * min(lane, UW - 1), c1 = 4 * min(lane + kWave, UW - 1);
        const int ngr = (L + UNR - 1) / UNR, ng = nrows * ngr;
        const float* src = TEXT ? (gather ? a.table : a.text_dense) : (m == 1 ? a.audio : a.visual);
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        int cur = 0;                        // the row being summed
        int rid_c = -1, rid_n = -1, raw_n = -1;
        float w_c = 0.f, w_n = 0.f, wd_n = 0.f;
        float4 num[2], sx[2], sxx[2];
        float cnt = 0.f, sw = 0.f;
        if constexpr (TEXT) {
          int raw;
          float wd;
          tok_issue(i0, raw, wd);
          tok_resolve(raw, wd, rid_c, w_c);
        }
        // loads through buffer descriptors: one scalar offset per frame (the
        // gathered row's or the frame's), per-lane column offsets vo0 / vo1 --
        // no 64-bit address arithmetic in VGPRs.  (The second column load
        // issued on its 11 live lanes only, the others zeroed, measured 23.37
        // vs 22.24 ms: the divergent branch costs more than the clamped
        // duplicate addresses, which the L1 coalesces.)
        const int vo0 = 4 * c0, vo1 = 4 * c1;
        auto issue = [&](int g, float4 (&v)[UNR][2]) {
          const int rr = g / ngr, t0 = (g - rr * ngr) * UNR;
          const int64_t i = i0 + 4 * rr;
          int rid = 0;
          if constexpr (TEXT) rid = rr == cur ? rid_c : rid_n;
          const bool rowbase = !TEXT || !gather;  // frames [L][W] of row i
          const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
              const_cast<float*>(rowbase ? src + i * L * W : src), 0,
              rowbase ? L * W * 4 : static_cast<int>(a.V * D * 4), 0x00020000);
#pragma unroll
          for (int u = 0; u < UNR; ++u) {
            const int t = min(t0 + u, L - 1);
            int so;
            if constexpr (TEXT) {
              const int r = __builtin_amdgcn_readlane(rid, t);
              so = gather ? (r >= 0 ? r : 0) * D * 4 : t * W * 4;
            } else {
              so = t * W * 4;
            }
            constexpr int pol = (!TEXT && NT) ? 2 : 0;  // non-temporal frame streams
            v[u][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo0, so, pol));
            v[u][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo1, so, pol));
          }
        };
        auto sum_frame = [&](int t, const float4 (&v)[2]) {
          if constexpr (TEXT) {
            const int r = __builtin_amdgcn_readlane(rid_c, t);
            const float wt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w_c), t));
            const bool ok = r >= 0;  // an out-of-range id (flagged) contributes a zero row
#pragma unroll
            for (int c = 0; c < 2; ++c) {
              const float4 x = ok ? v[c] : z4;
              fma4(num[c], wt, x);
              add4(sx[c], x);
              sq4(sxx[c], x);
            }
          } else {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
              add4(sx[c], v[c]);
              sq4(sxx[c], v[c]);
            }
          }
        };
        auto consume = [&](int g, const float4 (&v)[UNR][2]) {
          const int rr = g / ngr, gg = g - rr * ngr, t0 = gg * UNR;
          if (gg == 0) {
#pragma unroll
            for (int c = 0; c < 2; ++c) num[c] = sx[c] = sxx[c] = z4;
            if constexpr (TEXT) {
              cnt = static_cast<float>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(w_c != 0.f)));
              sw = wave_sum_dpp_f32(w_c);
              // every weight 0: x is 0/0 = NaN (numpy's answer); TruncatedSVD
              // would reject the split -- report it through the flag word
              if (lane == 0 && cnt == 0.f && a.flag) atomicOr(a.flag, MMB_FLAG_ZERO_WEIGHTS);
              if (rr + 1 < nrows) tok_issue(i0 + 4 * (rr + 1), raw_n, wd_n);
            }
          }
          if constexpr (TEXT) {
            if (gg == 1 && rr + 1 < nrows) tok_resolve(raw_n, wd_n, rid_n, w_n);
          }
          if (t0 + UNR <= L) {
#pragma unroll
            for (int u = 0; u < UNR; ++u) sum_frame(t0 + u, v[u]);
          } else {
#pragma unroll
            for (int u = 0; u < UNR; ++u)
              if (t0 + u < L) sum_frame(t0 + u, v[u]);
          }
          if (gg == ngr - 1) {
            const int q = uw + 4 * rr;
            finish_row(std::false_type{}, j, m, q, i0 + 4 * rr, num, sx, sxx, cnt, sw);
            cur = rr + 1;
            if constexpr (TEXT) {
              rid_c = rid_n;
              w_c = w_n;
            }
          }
        };
        float4 b0[UNR][2], b1[UNR][2];
        issue(0, b0);
        int g = 0;
#pragma unroll 1
        for (; g + 2 < ng; g += 2) {
          issue(g + 1, b1);
          consume(g, b0);
          issue(g + 2, b0);
          consume(g + 1, b1);
        }
        if (g + 1 < ng) {
          issue(g + 1, b1);
          consume(g, b0);
          consume(g + 1, b1);
        } else {
          consume(g, b0);
        }
      };
      // PIPE == 2: the same pipeline, and each piece's tail also issues the
      // NEXT piece's first group (text -> audio -> visual -> the next batch's
      // text) once its own next-to-last group is summed, so loads stay in
      // flight across piece and batch boundaries too; the next batch's first
      // text row is staged during the visual piece's last groups.  Pieces with
      // an odd group count drain as before.
      float4 pb0[UNR][2], pb1[UNR][2];
      bool pre = false;  // pb0 holds this piece's group 0 (issued by the previous piece)
      int rid_pre = -1, raw_p = -1;
      float w_pre = 0.f, wd_p = 0.f;
      auto piece2 = [&](auto m_c, int64_t j, int64_t i0, int nrows, int64_t ni0, int nnr) {
        constexpr int M = decltype(m_c)::value;
        constexpr bool TEXT = M == 0;
        const int W = wdt[M], UW = W >> 2;
        const int ngr = (L + UNR - 1) / UNR, ng = nrows * ngr;
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        const bool has_next = M < 2 || nnr > 0;
        if constexpr (M == 2) {
          // the text piece's x / aux stores complete before any visual
          // increment (the projectors read x after the visual piece): with
          // group 0 in flight the 16 newest operations are its loads
          if (pre) {
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
          } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
        }
        int cur = 0;
        int rid_c = -1, rid_n = -1, raw_n = -1;
        float w_c = 0.f, w_n = 0.f, wd_n = 0.f;
        float4 num[2], sx[2], sxx[2];
        float cnt = 0.f, sw = 0.f;
        if constexpr (TEXT) {
          if (pre) {
            rid_c = rid_pre;
            w_c = w_pre;
          } else {
            int raw;
            float wd;
            tok_issue(i0, raw, wd);
            tok_resolve(raw, wd, rid_c, w_c);
          }
        }
        const int vo0 = 16 * min(lane, UW - 1), vo1 = 16 * min(lane + kWave, UW - 1);
        // group g of this piece (or, NX, group 0 of the next piece) into v
        auto load_group = [&](auto nx_c, int g, float4 (&v)[UNR][2]) {
          constexpr bool NX = decltype(nx_c)::value;
          constexpr int MM = NX ? (M + 1) % 3 : M;
          constexpr bool T2 = MM == 0;
          const int rr = NX ? 0 : g / ngr, t0 = NX ? 0 : (g - rr * ngr) * UNR;
          const int64_t i = NX ? (M == 2 ? ni0 : i0) : i0 + 4 * rr;
          const int W2 = wdt[MM], U2 = W2 >> 2;
          const float* s2 = T2 ? (gather ? a.table : a.text_dense) : (MM == 1 ? a.audio : a.visual);
          const int o0 = NX ? 16 * min(lane, U2 - 1) : vo0, o1 = NX ? 16 * min(lane + kWave, U2 - 1) : vo1;
          int rid = 0;
          if constexpr (T2) rid = NX ? rid_pre : (rr == cur ? rid_c : rid_n);
          const bool rowbase = !T2 || !gather;
          const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
              const_cast<float*>(rowbase ? s2 + i * L * W2 : s2), 0,
              rowbase ? L * W2 * 4 : static_cast<int>(a.V * D * 4), 0x00020000);
#pragma unroll
          for (int u = 0; u < UNR; ++u) {
            const int t = min(t0 + u, L - 1);
            int so;
            if constexpr (T2) {
              const int r = __builtin_amdgcn_readlane(rid, t);
              so = gather ? (r >= 0 ? r : 0) * D * 4 : t * W2 * 4;
            } else {
              so = t * W2 * 4;
            }
            constexpr int pol = (!T2 && NT) ? 2 : 0;  // non-temporal frame streams
            v[u][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, o0, so, pol));
            v[u][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, o1, so, pol));
          }
        };
        auto issue = [&](int g, float4 (&v)[UNR][2]) { load_group(std::false_type{}, g, v); };
        auto sum_frame = [&](int t, const float4 (&v)[2]) {
          if constexpr (TEXT) {
            const int r = __builtin_amdgcn_readlane(rid_c, t);
            const float wt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w_c), t));
            const bool ok = r >= 0;  // an out-of-range id (flagged) contributes a zero row
#pragma unroll
            for (int c = 0; c < 2; ++c) {
              const float4 x = ok ? v[c] : z4;
              fma4(num[c], wt, x);
              add4(sx[c], x);
              sq4(sxx[c], x);
            }
          } else {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
              add4(sx[c], v[c]);
              sq4(sxx[c], v[c]);
            }
          }
        };
        auto consume = [&](int g, const float4 (&v)[UNR][2]) {
          const int rr = g / ngr, gg = g - rr * ngr, t0 = gg * UNR;
          if (gg == 0) {
#pragma unroll
            for (int c = 0; c < 2; ++c) num[c] = sx[c] = sxx[c] = z4;
            if constexpr (TEXT) {
              cnt = static_cast<float>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(w_c != 0.f)));
              sw = wave_sum_dpp_f32(w_c);
              // every weight 0: x is 0/0 = NaN (numpy's answer); TruncatedSVD
              // would reject the split -- report it through the flag word
              if (lane == 0 && cnt == 0.f && a.flag) atomicOr(a.flag, MMB_FLAG_ZERO_WEIGHTS);
              if (rr + 1 < nrows) tok_issue(i0 + 4 * (rr + 1), raw_n, wd_n);
            }
          }
          if constexpr (TEXT) {
            if (gg == 1 && rr + 1 < nrows) tok_resolve(raw_n, wd_n, rid_n, w_n);
          }
          if constexpr (M == 2) {  // the next batch's first text row
            if (has_next && ng >= 4 && g == ng - 4) tok_issue(ni0, raw_p, wd_p);
            if (has_next && ng >= 4 && g == ng - 3) tok_resolve(raw_p, wd_p, rid_pre, w_pre);
          }
          if (t0 + UNR <= L) {
#pragma unroll
            for (int u = 0; u < UNR; ++u) sum_frame(t0 + u, v[u]);
          } else {
#pragma unroll
            for (int u = 0; u < UNR; ++u)
              if (t0 + u < L) sum_frame(t0 + u, v[u]);
          }
          if (gg == ngr - 1) {
            const int q = uw + 4 * rr;
            finish_row(std::false_type{}, j, M, q, i0 + 4 * rr, num, sx, sxx, cnt, sw);
            cur = rr + 1;
            if constexpr (TEXT) {
              rid_c = rid_n;
              w_c = w_n;
            }
          }
        };
        if (!pre) issue(0, pb0);
        int g = 0;
#pragma unroll 1
        for (; g + 2 < ng; g += 2) {
          issue(g + 1, pb1);
          consume(g, pb0);
          issue(g + 2, pb0);
          consume(g + 1, pb1);
        }
        if (g + 1 < ng) {
          issue(g + 1, pb1);
          consume(g, pb0);
          if (has_next) {
            if constexpr (M == 2) {
              if (ng < 4) {  // too few groups to stage the tokens on the way
                tok_issue(ni0, raw_p, wd_p);
                tok_resolve(raw_p, wd_p, rid_pre, w_pre);
              }
            }
            load_group(std::true_type{}, 0, pb0);
          }
          consume(g + 1, pb1);
          pre = has_next;
        } else {
          consume(g, pb0);
          pre = false;
        }
      };
      // Local batches 0 and 1 are the round robin's units (every workgroup
      // drawing at once at the start queued 512 atomics on one word); from 2
      // on, streamer wave 0 draws local batch j + 2's unit at the top of batch
      // j and publishes it after the batch's text piece, so the atomic's
      // return is not waited for where it is issued; the other waves need it
      // at the top of batch j + 1, the projectors later still
      unsigned drawn = 0;
      auto draw_issue = [&]() {
        if (dyn && uw == 0 && lane == 0)
          drawn = __hip_atomic_fetch_add(f.sched, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      };
      auto draw_commit = [&](int64_t j) {  // publishes local batch j + 2
        if (dyn && uw == 0 && lane == 0) {
          const unsigned b = 2u * G + drawn;
          s_bat[(j + 2) & 7] = static_cast<int>(b < 0x7fffffffu ? b : 0x7fffffffu);
          __hip_atomic_store(&s_tag[(j + 2) & 7], static_cast<int>(j) + 3, __ATOMIC_RELEASE,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      };
      auto rows_of = [&](int64_t jb, int64_t& i0) -> int {
        int64_t row0, rend;
        if (!batch(jb, row0, rend)) {
          i0 = 0;
          return dyn ? -1 : 0;  // (dynamic: -1 = no batch, 0 = a batch without this wave's rows)
        }
        i0 = row0 + uw;
        return i0 < rend ? static_cast<int>(min<int64_t>(kGR / 4, (rend - i0 + 3) / 4)) : 0;
      };
      // dynamic order: every wave counts kGR / 4 fill increments per piece,
      // its rows' and the rest as padding after them, so the projectors'
      // targets stay kGR per piece whatever the unit's rows (a 12-row unit
      // followed by more units would otherwise leave the next targets short)
      auto pad = [&](int64_t j, int m, int nrows) {
        if (dyn && nrows < kGR / 4 && lane == 0) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __hip_atomic_fetch_add(&fill[(3 * static_cast<int>(j) + m) & 3], kGR / 4 - nrows, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      };
      if constexpr (PIPE == 2) {
        int64_t i0, ni0;
        int nrows = rows_of(0, i0);
        for (int64_t j = 0; nrows > 0 || (dyn && nrows == 0); ++j) {
          draw_issue();
          const int nnr = rows_of(j + 1, ni0);
          if (nrows > 0) {
            const int nn = nnr > 0 ? nnr : 0;
            piece2(std::integral_constant<int, 0>{}, j, i0, nrows, ni0, nn);
            draw_commit(j);
            pad(j, 0, nrows);
            piece2(std::integral_constant<int, 1>{}, j, i0, nrows, ni0, nn);
            pad(j, 1, nrows);
            piece2(std::integral_constant<int, 2>{}, j, i0, nrows, ni0, nn);
            pad(j, 2, nrows);
          } else {  // a unit without rows for this wave (its last < 4 rows)
            pre = false;
            draw_commit(j);
            for (int m = 0; m < 3; ++m) pad(j, m, 0);
          }
          i0 = ni0;
          nrows = nnr;
        }
      } else {
        for (int64_t j = 0;; ++j) {
          int64_t row0, rend;
          if (!batch(j, row0, rend)) break;
          const int64_t i0 = row0 + uw;
          const int nrows = i0 < rend ? static_cast<int>(min<int64_t>(kGR / 4, (rend - i0 + 3) / 4)) : 0;
          if (nrows == 0) continue;
          piece(std::true_type{}, j, 0, i0, nrows);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // x / aux stores before the audio increments
          piece(std::false_type{}, j, 1, i0, nrows);
          piece(std::false_type{}, j, 2, i0, nrows);
        }
      }
    }
    if (a.cmax_part) {  // this wave's column bounds (mmb_gram_i8)
      const int64_t wid = static_cast<int64_t>(blockIdx.x) * 4 + wave;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int uu = lane + kWave * c;
        if (uu < (D >> 2)) st4(a.cmax_part + wid * D + 4 * uu, cmx[c]);
      }
    }
    FUSED_PROBE(1 + wave);
    return;
  }

  // -------------------------------------------------------------- projector
  const int pw = wave - 4;
  const int q = lane & 15, g = lane >> 4;  // A row / B column in a tile; k group
  constexpr int CH = 2 * kFLdw * 32, PL = kFLdw * 32;  // B image chunk / plane (halves)
  const int nch = (f.kq[0] + f.kq[1] + f.kq[2]) / 32;
  const int cb[3] = {0, f.kq[0] / 32, (f.kq[0] + f.kq[1]) / 32};
  const auto brsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(f.img), 0, nch * CH * 2,
                                                       0x00020000);
  int boff[kFTiles];
  float cinv[kFTiles], cadd[kFTiles];
#pragma unroll
  for (int t = 0; t < kFTiles; ++t) {
    const int col = 16 * (kFTiles * pw + t) + q;
    boff[t] = col * 32 + ((g ^ x3_swz(col)) << 3);
    cinv[t] = f.col_inv[col];
    cadd[t] = f.c0[col];
  }
  // column D (the total weight) lives in projector tD_w, tile tD_t, lane q == tD_q
  const int tD = D >> 4, tD_w = tD / kFTiles, tD_t = tD % kFTiles, tD_q = D & 15;
  // this projector's tiles holding columns <= D (the rest of the 320 are
  // zero); 256 <= D < 320 leaves at most one dead tile, on projector 3
  const int ntiles = max(kFTiles - 1, min(kFTiles, tD + 1 - kFTiles * pw));
  int ep = 0;  // projector exchange points passed
  for (int64_t j = 0;; ++j) {
    int64_t row0, rend;
    if (!batch(j, row0, rend)) break;
    const int nvalid = static_cast<int>(rend - row0);
    f32x4 acc[kGRT][kFTiles];
#pragma unroll
    for (int rt = 0; rt < kGRT; ++rt)
#pragma unroll
      for (int t = 0; t < kFTiles; ++t) acc[rt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float irs[kGRT][4];
#pragma unroll 1
    for (int m = 0; m < 3; ++m) {
      const int p = 3 * static_cast<int>(j) + m;
      fused_wait(&fill[p & 3], kGR * (p >> 2) + (dyn ? kGR : nvalid), abort_flag, a.flag);
      if constexpr ((DIAG & 1) != 0) {
        fused_signal(consumed);
        continue;
      }
      // this piece's power-of-2 scales of the lane's output rows 16 rt + 4 g + jj;
      // the running sums move to this piece's scale (exact: ratios of powers of 2)
#pragma unroll
      for (int rt = 0; rt < kGRT; ++rt)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const float v = s_irs[(p * kGR + 16 * rt + 4 * g + jj) % SL];
          if (m > 0) {
            const float ratio = irs[rt][jj] / v;
#pragma unroll
            for (int t = 0; t < kFTiles; ++t) acc[rt][t][jj] *= ratio;
          }
          irs[rt][jj] = v;
        }
      const _Float16* arow[kGRT];
#pragma unroll
      for (int rt = 0; rt < kGRT; ++rt) arow[rt] = ring + ((p * kGR + 16 * rt + q) % SL) * kGSlot;
      const int npc = f.kq[m] / 32, c0g = cb[m];
      // the K loop for NT live column tiles (tiles past column D hold zero
      // padding: projector 3 at D = 300 skips their loads and MFMAs)
      auto kloop = [&](auto nt_c) {
        constexpr int NL = decltype(nt_c)::value;
        half8 bh[2][NL], bl[2][NL];
        auto ld_b = [&](int c, half8 (&h)[NL], half8 (&l)[NL]) {
          // DIAG 16: every chunk reads the piece's chunk 0 (a 20 KB L2 footprint)
          const int so = (DIAG & 16) ? c0g * CH * 2 : (c0g + (c < npc ? c : npc - 1)) * CH * 2;
#pragma unroll
          for (int t = 0; t < NL; ++t) {
            if constexpr ((DIAG & 32) != 0) {  // no B loads at all
              h[t] = l[t] = half8{1, 1, 1, 1, 1, 1, 1, 1};
            } else {
              h[t] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(brsrc, boff[t] * 2, so, 0));
              l[t] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(brsrc, (boff[t] + PL) * 2, so, 0));
            }
          }
        };
        auto chunk = [&](int c, const half8 (&h)[NL], const half8 (&l)[NL]) {
          const int o = (((4 * c + g) ^ q) << 3);
#pragma unroll
          for (int rt = 0; rt < kGRT; ++rt) {
            const half8 ah = *reinterpret_cast<const half8*>(arow[rt] + o);
            const half8 al = *reinterpret_cast<const half8*>(arow[rt] + kGPlane + o);
            if constexpr ((DIAG & 2) != 0) {
              asm volatile("" ::"v"(ah), "v"(al));
#pragma unroll
              for (int t = 0; t < NL; ++t) asm volatile("" ::"v"(h[t]), "v"(l[t]));
            } else {
#pragma unroll
              for (int t = 0; t < NL; ++t) {
                acc[rt][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, h[t], acc[rt][t], 0, 0, 0);
                acc[rt][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, l[t], acc[rt][t], 0, 0, 0);
                acc[rt][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, h[t], acc[rt][t], 0, 0, 0);
              }
            }
          }
        };
        ld_b(0, bh[0], bl[0]);
        ld_b(1, bh[1], bl[1]);
#pragma unroll 1
        for (int c = 0; c < npc; c += 2) {
          chunk(c, bh[0], bl[0]);
          ld_b(c + 2, bh[0], bl[0]);
          if (c + 1 < npc) {
            chunk(c + 1, bh[1], bl[1]);
            ld_b(c + 3, bh[1], bl[1]);
          }
        }
      };
      if (ntiles == kFTiles) {
        kloop(std::integral_constant<int, kFTiles>{});
      } else {
        kloop(std::integral_constant<int, kFTiles - 1>{});
      }
      // this projector's LDS reads of the piece's slots are done (lgkmcnt
      // only: its weight-image loads in flight and the previous epilogue's
      // MMB2 stores do not guard the slots; 22.48 -> 22.45 ms, r02z)
      fused_signal_lds(consumed);
    }
    if constexpr ((DIAG & 5) != 0) {
#pragma unroll
      for (int rt = 0; rt < kGRT; ++rt)
#pragma unroll
        for (int t = 0; t < kFTiles; ++t) asm volatile("" ::"v"(acc[rt][t]));
      continue;
    }

    // epilogue: lane value (rt, t, jj) = row 16 rt + 4 g + jj, column 16 (5 pw + t) + q
    const float* cntb = s_cnt + (j & 1) * kGR;
    const float* twb = s_tw + (j & 1) * kGR;
    float* tot = s_tot + (j & 1) * kGR;
    float* ssq = s_ssq + (j & 1) * 4 * kGR;
#pragma unroll
    for (int rt = 0; rt < kGRT; ++rt) {
      float xv[kFTiles][4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int64_t rowc = min(row0 + 16 * rt + 4 * g + jj, N - 1);
#pragma unroll
        for (int t = 0; t < kFTiles; ++t) {
          const int col = 16 * (kFTiles * pw + t) + q;
          if constexpr ((DIAG & 128) != 0) {  // timing only: no x re-read
            xv[t][jj] = static_cast<float>(col);
          } else {
            xv[t][jj] = a.num_out[rowc * D + min(col, D - 1)];
          }
        }
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int r = 16 * rt + 4 * g + jj;
        const float cn = cntb[r], tw = twb[r];
#pragma unroll
        for (int t = 0; t < kFTiles; ++t) {
          const int col = 16 * (kFTiles * pw + t) + q;
          const float add = col < D ? text_sum(xv[t][jj], cn) : (col == D ? tw : 0.f);
          acc[rt][t][jj] = acc[rt][t][jj] * (cinv[t] * irs[rt][jj]) + add + cadd[t];
        }
        if (pw == tD_w && q == tD_q) {
#pragma unroll
          for (int t = 0; t < kFTiles; ++t)
            if (t == tD_t) tot[r] = acc[rt][t][jj];
        }
      }
    }
    fused_signal_lds(pbar);  // the row totals exchanged through LDS only
    fused_wait(pbar, 4 * ++ep, abort_flag, a.flag);
#pragma unroll
    for (int rt = 0; rt < kGRT; ++rt) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int r = 16 * rt + 4 * g + jj;
        const float rtot = 1.f / tot[r];
        float ss = 0.f;
#pragma unroll
        for (int t = 0; t < kFTiles; ++t) {
          const int col = 16 * (kFTiles * pw + t) + q;
          acc[rt][t][jj] *= rtot;
          if (col < D) ss = fmaf(acc[rt][t][jj], acc[rt][t][jj], ss);
        }
        ss = row16_sum(ss);
        if (q == 0) ssq[pw * kGR + r] = ss;
      }
    }
    fused_signal_lds(pbar);
    fused_wait(pbar, 4 * ++ep, abort_flag, a.flag);
#pragma unroll
    for (int rt = 0; rt < kGRT; ++rt) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int r = 16 * rt + 4 * g + jj;
        const float inv = 1.f / sqrtf((ssq[r] + ssq[kGR + r]) + (ssq[2 * kGR + r] + ssq[3 * kGR + r]));
        if (r < nvalid) {
          float* orow = f.out + (row0 + r) * D;
#pragma unroll
          for (int t = 0; t < kFTiles; ++t) {
            const int col = 16 * (kFTiles * pw + t) + q;
            if constexpr ((DIAG & 256) != 0) {  // timing only: no MMB2 stores
              asm volatile("" ::"v"(acc[rt][t][jj] * inv));
            } else {
              if (col < D) orow[col] = acc[rt][t][jj] * inv;
            }
          }
        }
      }
    }
  }
  FUSED_PROBE(1 + wave);
}

template <int DIAG, int UNR = 8, int PIPE = 0, int SL = kGSlots>
static void launch_fused_v(const FusedArgs& f, int grid, hipStream_t stream) {
  constexpr size_t lds = fused_lds_bytes(SL);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&utt_fused_kernel<UNR, true, DIAG, PIPE, SL>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    attr = true;
  }
  utt_fused_kernel<UNR, true, DIAG, PIPE, SL><<<grid, kFThreads, lds, stream>>>(f);
}
// streamer: 1 = pipelined (two groups in flight: kernel 23.35 -> 22.49 ms,
// step 25.14 -> 24.41 ms in a same-process A/B, r02k); 2 (default) = also
// prefetching across piece and batch boundaries (22.32 -> 22.14 ms, r02y);
// 0 = one group at a time (the fallback for rows of < 3 frame groups or a
// word table >= 2 GB, and the bit-identical reference of the tests)
static bool fused_pipe_ok(const FusedArgs& f, int un) {
  // the pipelined streamer stages a text row's tokens two groups before its
  // first group is issued: >= 3 groups per row; it addresses the word table
  // through one buffer descriptor (< 2^31 bytes)
  return (f.s.L + un - 1) / un >= 3 && (f.s.ids == nullptr || f.s.V * f.s.D * 4 < (int64_t{1} << 31));
}

static int fused_grid(int64_t nb, hipStream_t stream) {
  return static_cast<int>(std::min<int64_t>(nb, std::min(stream_cu_count(stream), kCmaxRows / 4)));
}

static int launch_fused(const FusedArgs& f, hipStream_t stream, int* parts) {
  const int grid = fused_grid(f.nb, stream);
  if (parts) *parts = grid * 4;
#ifndef MMB_HOOK_FUSED_LAUNCH  // (tools/diag: the MMB_FUSED_* sweeps and ablations)
#define MMB_HOOK_FUSED_LAUNCH false
#endif
  if (!(MMB_HOOK_FUSED_LAUNCH)) {
    if (fused_pipe_ok(f, 8)) {
      launch_fused_v<0, 8, 2>(f, grid, stream);
    } else {
      launch_fused_v<0, 8, 0>(f, grid, stream);
    }
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
  if (MM2 && a.N <= stream_cu_count(stream)) {
    // a few long rows (POM's splits: 100 / 203 rows of 1089 / 1357 tokens):
    // 16 frame / 8 text rows in flight per group instead of 4 / 4 (r05
    // tools/splits_ab.py, gpurun_out r05m: stream 0.180 -> 0.148 ms and
    // 0.217 -> 0.188 ms, the same sums bit for bit; 1024 threads x 4 / 4:
    // 0.157 / 0.193 ms)
#ifndef MMB_HOOK_STREAM_SMALL  // (tools/diag: MMB_STREAM_SMALL)
#define MMB_HOOK_STREAM_SMALL false
#endif
    if (!(MMB_HOOK_STREAM_SMALL)) {
      utt_stream_kernel<MM2, VT, VA, VV, 16, 8><<<grid, kNT, 0, stream>>>(a);
    }
  } else
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

// the column-bound partials [kCmaxRows][d], then (mmb_mm2_stream_project)
// the fused kernel's batch counter (16 bytes)
extern "C" size_t mmb_mm2_colmax_ws_bytes(int d) {
  return static_cast<size_t>(kCmaxRows) * (d > 0 ? d : 0) * sizeof(float) + 16;
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
      const hipError_t e = static_cast<hipError_t>(zero_words_async(colmax, static_cast<int64_t>(sizeof(uint32_t) * d) / 4, stream));
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

// Ranges per utterance of the few-long-rows path: about one workgroup per
// CU in all (3 per range: text, audio, visual), no range under
// kSplitMinTok frames.  r06 sweep (tools/split_ab.py, graph-timed, POM's
// real splits): fewer, longer streams win -- valid (100 x 1089) 55.3 / 62.9
// / 64.8 / 64.8 us at 1 / 2 / 3 / 4 ranges, test (203 x 1357) 126 / 135 /
// 125 / 145 us; the one-workgroup kernel 89.7 / 134 us; a plain read of the
// same frame bytes (probe, 512 workgroups) 40.5 / 97 us.
constexpr int kSplitMinTok = 64;
static int split_parts(int64_t n, int t, int cus) {
  if (n <= 0 || t <= 0) return 1;
  const int64_t want = ceil_div(static_cast<int64_t>(cus), 3 * n);
  const int64_t cap = std::max<int64_t>(1, t / kSplitMinTok);
  return static_cast<int>(std::max<int64_t>(1, std::min(want, cap)));
}

extern "C" int mmb_mm2_stream_split_parts(int64_t n, int t) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
    (void)hipGetLastError();
    cus = 256;
  }
  return split_parts(n, t, cus);
}

static size_t split_ws_floats(int64_t n, const SplitPlan& q) {
  return static_cast<size_t>(n) * (static_cast<size_t>(q.Pt) * q.Wt + static_cast<size_t>(q.Pf) * q.Wf);
}

extern "C" size_t mmb_mm2_stream_split_ws_bytes(int64_t n, int t, int d, int a_, int vd, int parts) {
  if (n <= 0 || t <= 0 || d <= 0 || a_ <= 0 || vd <= 0) return 0;
  const int P = parts > 0 ? std::min(parts, t) : mmb_mm2_stream_split_parts(n, t);
  return split_ws_floats(n, split_plan_of(t, d, a_, vd, P, parts > 0 ? 1 : MMB_SPLIT_TEXT_X)) * sizeof(float);
}

template <int VT, int VA, int VV>
static int launch_split(const StreamArgs& a, const SplitPlan& q, float* part, hipStream_t stream) {
  const int64_t grid = a.N * (q.Pt + 2 * q.Pf);
  utt_split_part_kernel<VT, VA, VV, MMB_SPLIT_FU, MMB_SPLIT_TU><<<static_cast<unsigned>(grid), kNT, 0, stream>>>(a, q, part);
  MMB_LAUNCH_CHECK();
  const size_t lds = a.s_half ? static_cast<size_t>(2 * (a.D + a.A + a.Vd)) * sizeof(float) : 0;
  utt_split_finish_kernel<<<static_cast<unsigned>(a.N), kNT, lds, stream>>>(a, q, part);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_mm2_stream_split(const int32_t* ids, const float* table, int64_t v,
                                    const float* wtab32, const float* text_dense,
                                    const float* emb_dense, const float* w_dense, const float* audio,
                                    const float* visual, int64_t n, int t, int d, int a_, int vd,
                                    float* num_out, void* s_out, int s_half, float* aux_out,
                                    int32_t* flag, uint32_t* colmax, void* colmax_ws, int parts,
                                    void* ws, size_t ws_bytes, hipStream_t stream) {
  MMB_REQUIRE(n >= 0 && t > 0 && d > 0 && a_ > 0 && vd > 0 && parts >= 0);
  MMB_REQUIRE(colmax == nullptr || (colmax_ws != nullptr && d <= 2 * kNT && n <= kCmaxRows));
  MMB_REQUIRE(audio && visual && num_out && s_out && aux_out && (s_half == 0 || s_half == 1));
  if (ids) {
    MMB_REQUIRE(table && v > 0 && (wtab32 || w_dense));
  } else {
    MMB_REQUIRE(text_dense && emb_dense && w_dense);
  }
  if (n == 0) {
    if (colmax) {
      const hipError_t e = static_cast<hipError_t>(zero_words_async(colmax, d, stream));
      if (e != hipSuccess) return static_cast<int>(e);
    }
    return MMB_OK;
  }
  const int P = parts > 0 ? std::min(parts, t) : mmb_mm2_stream_split_parts(n, t);
  const SplitPlan q = split_plan_of(t, d, a_, vd, P, parts > 0 ? 1 : MMB_SPLIT_TEXT_X);
  MMB_REQUIRE(ws && ws_bytes >= split_ws_floats(n, q) * sizeof(float));
  MMB_REQUIRE(n * (q.Pt + 2 * q.Pf) <= (int64_t{1} << 31) - 1);
  MMB_REQUIRE(3 * d + 2 * a_ + 2 * vd <= kSplitJ * kNT);  // the finish kernel's columns
  StreamArgs s{};
  s.cmax_part = colmax ? static_cast<float*>(colmax_ws) : nullptr;
  s.ids = ids; s.table = table; s.V = v; s.wtab = wtab32; s.w_dense = w_dense;
  s.text_dense = text_dense; s.emb_dense = emb_dense; s.audio = audio; s.visual = visual;
  s.N = n; s.L = t; s.D = d; s.A = a_; s.Vd = vd; s.Kp = mmb_mm2_k(d, a_, vd);
  s.num_out = num_out; s.s_out = static_cast<float*>(s_out); s.aux_out = aux_out; s.flag = flag;
  s.s_half = s_half;
  const bool vt = (d % 4 == 0) && (ids ? aligned16(table) : (aligned16(text_dense) && aligned16(emb_dense)));
  const bool va = (a_ % 4 == 0) && aligned16(audio);
  const bool vv = (vd % 4 == 0) && aligned16(visual);
  MMB_REQUIRE(d / (vt ? 4 : 1) <= kNT && a_ / (va ? 4 : 1) <= kNT && vd / (vv ? 4 : 1) <= kNT);
  float* part = static_cast<float*>(ws);
  int rc;
  switch ((vt ? 4 : 0) | (va ? 2 : 0) | (vv ? 1 : 0)) {
    case 7: rc = launch_split<4, 4, 4>(s, q, part, stream); break;
    case 6: rc = launch_split<4, 4, 1>(s, q, part, stream); break;
    case 5: rc = launch_split<4, 1, 4>(s, q, part, stream); break;
    case 4: rc = launch_split<4, 1, 1>(s, q, part, stream); break;
    case 3: rc = launch_split<1, 4, 4>(s, q, part, stream); break;
    case 2: rc = launch_split<1, 4, 1>(s, q, part, stream); break;
    case 1: rc = launch_split<1, 1, 4>(s, q, part, stream); break;
    default: rc = launch_split<1, 1, 1>(s, q, part, stream); break;
  }
  if (rc != MMB_OK || !colmax) return rc;
  colmax_reduce_kernel<<<static_cast<unsigned>(ceil_div(d, 64)), 1024, 0, stream>>>(
      static_cast<const float*>(colmax_ws), static_cast<int>(n), d, colmax);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_mm2_stream_project_supported(int t, int d, int a_, int vd) {
  // every piece [Sx | Sxx] of one modality fits a ring slot (2 w <= 640),
  // two float4 columns per lane (w <= 512), the 320-column weight image
  return t > 0 && t <= kWave && d >= 256 && d < 320 && d % 4 == 0 && a_ > 0 && vd > 0 &&
         a_ % 4 == 0 && vd % 4 == 0 && 2 * a_ <= kGPlane && 2 * vd <= kGPlane;
}

extern "C" int mmb_mm2_stream_project(const int32_t* ids, const float* table, int64_t v,
                                      const float* wtab32, const float* text_dense,
                                      const float* w_dense, const float* audio, const float* visual,
                                      int64_t n, int t, int d, int a_, int vd, const void* wpieces,
                                      const float* c0, float* num_out, float* aux_out,
                                      float* mmb2_out, int32_t* flag, uint32_t* colmax,
                                      void* colmax_ws, hipStream_t stream) {
  MMB_REQUIRE(n >= 0 && mmb_mm2_stream_project_supported(t, d, a_, vd));
  MMB_REQUIRE(audio && visual && num_out && aux_out && mmb2_out && wpieces && c0);
  MMB_REQUIRE(colmax == nullptr || colmax_ws != nullptr);
  if (ids) {
    MMB_REQUIRE(table && v > 0 && (wtab32 || w_dense) && aligned16(table));
  } else {
    MMB_REQUIRE(text_dense && w_dense && aligned16(text_dense));
  }
  MMB_REQUIRE(aligned16(audio) && aligned16(visual) && aligned16(num_out) && aligned16(wpieces));
  if (n == 0) {
    if (colmax) {
      const hipError_t e = static_cast<hipError_t>(zero_words_async(colmax, static_cast<int64_t>(sizeof(uint32_t) * d) / 4, stream));
      if (e != hipSuccess) return static_cast<int>(e);
    }
    return MMB_OK;
  }
  FusedArgs f{};
  StreamArgs& s = f.s;
  s.ids = ids; s.table = table; s.V = v; s.wtab = wtab32; s.w_dense = w_dense;
  s.text_dense = text_dense; s.emb_dense = text_dense; s.audio = audio; s.visual = visual;
  s.N = n; s.L = t; s.D = d; s.A = a_; s.Vd = vd; s.Kp = mmb_mm2_k(d, a_, vd);
  s.num_out = num_out; s.aux_out = aux_out; s.flag = flag; s.s_half = 1;
  s.cmax_part = colmax ? static_cast<float*>(colmax_ws) : nullptr;
  const int w3[3] = {d, a_, vd};
  int kq = 0;
  for (int m = 0; m < 3; ++m) {
    f.kq[m] = (2 * w3[m] + 31) / 32 * 32;
    kq += f.kq[m];
  }
  f.img = static_cast<const _Float16*>(wpieces);
  f.col_inv = reinterpret_cast<const float*>(f.img + 2 * static_cast<size_t>(kFLdw) * kq);
  f.c0 = c0;
  f.out = mmb2_out;
  f.nb = ceil_div(n, kGR);
  f.balanced = 1;  // balanced tail: 22.35 -> 22.26 ms (r02s)
  // the dynamic batch schedule's counter, past the column-bound partials
  // (zeroed here by a kernel: no memset node in a captured step)
  f.sched = colmax ? reinterpret_cast<unsigned*>(static_cast<char*>(colmax_ws) +
                                                 static_cast<size_t>(kCmaxRows) * d * sizeof(float))
                   : nullptr;
#ifdef MMB_HOOK_FUSED_ARGS  // (tools/diag: MMB_FUSED_BALANCED / MMB_FUSED_DYN)
  MMB_HOOK_FUSED_ARGS(f);
#endif
  {
    // the dynamic order from 16 rounds of batches on (fewer: the static round
    // robin, whose finishing times spread little there); its units: 48-row
    // batches, then the last ~G batches' rows as 12-row units.  Same-process
    // A/B (tools/fused_dyn_ab.py, r05af/ag, fused kernel ms static ->
    // dynamic): 1M 22.63 -> 22.38, 500k 11.41 -> 11.28, 250k 5.98 -> 5.96;
    // 125k (10 rounds) 2.98 -> 3.06, so it stays static
    const int64_t G = fused_grid(f.nb, stream);
    if (f.nb < 16 * G) f.sched = nullptr;
    if (f.sched) {
      f.big = std::max<int64_t>(0, n - kGR * G) / kGR;
      f.nu = f.big + ceil_div(n - f.big * kGR, kGR / 4);
      const hipError_t e = static_cast<hipError_t>(zero_words_async(f.sched, 1, stream));
      if (e != hipSuccess) return static_cast<int>(e);
    }
  }
  int parts = 0;
  const int rc = launch_fused(f, stream, &parts);
  if (rc != MMB_OK || !colmax) return rc;
  colmax_reduce_kernel<<<static_cast<unsigned>(ceil_div(d, 64)), 1024, 0, stream>>>(
      static_cast<const float*>(colmax_ws), parts, d, colmax);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}


namespace mmb {

// ------------------------------------------------------------------ narrow fused (r04)
// SIF + closed-form MMB2 at narrow frame widths (MOSI: COVAREP A = 76, FACET
// Vd = 48, V = 3016) in ONE kernel: the two-kernel step wrote the frame sums
// s (fp16 hi | lo of 2 (D + A + Vd) = 848 sums, 3.4 KB per utterance) to HBM
// and read them back in a K = 864 projection.  Here the text sums never
// form: the text rows of Wm are applied per vocabulary row (the text cache,
// mmb_mm2_text_cache: P[v] = E_v Wm_t1 + E_v^2 Wm_t2, column D the total
// weight), so an utterance's text term is sum_t P[id_t], gathered beside its
// table rows, and only the audio / visual sums [Sa | Saa | Sv | Svv] (K =
// kq(A) + kq(Vd) <= 256) go through the f16 x3 MFMA -- in the same launch.
//
// One persistent 512-thread workgroup per CU, batches of 32 utterances:
//   stream phase: every wave runs 4 utterances as utt_narrow_kernel does
//     (packed frame instructions issued first, ids one utterance ahead,
//     buffer-descriptor loads), its text rows from LDS for the 32 words of
//     smallest weight (the most frequent; ~58 % of Zipf(1.1) tokens at
//     V = 3016) and from L2 otherwise; it writes x (the a2 row, bit-identical
//     to the narrow kernel's: the same f32 operations in the same order),
//     aux, its column bounds, and into LDS the row's text term T (x-sum + sum
//     of P) and its audio / visual sums as fp16 hi | lo (power-of-2 row scale);
//   MFMA phase (after a barrier): [32 x K] x [K x 320] as fp16 x3 products
//     (v_mfma_f32_16x16x32_f16, the fused kernel's projector arithmetic; B =
//     the audio / visual chunks of the piece-ordered weight image, from L2);
//   epilogue: y = acc * scales + T + c0 into the T rows (LDS), then per row
//     the division by the total weight (column D) and the L2 norm, the MMB2
//     row written with 16-byte stores.
// LDS: hot E rows 38.4 KB + hot P rows 38.9 KB + T 38.9 KB + A 32 KB.
#ifndef NF_UNR
#define NF_UNR 2
#endif
#ifndef NF_HU
#define NF_HU 1
#endif
#ifndef NF_ABL  // timing-only ablations (tools/ab_libs): 1 no MFMA, 2 no frames, 4 no text,
                // 8 no a2 / aux stores, 16 no MMB2 stores, 32 no id / weight loads
#define NF_ABL 0
#endif
#ifndef NF_GA  // audio / visual frame loads issued with the text loads
#define NF_GA 7
#endif
#ifndef NF_GV
#define NF_GV 4
#endif
#ifndef NF_WAVES  // 8 (2 per SIMD, 32-row batches) or 12 (3 per SIMD, 36-row batches)
#define NF_WAVES 8
#endif
constexpr int kNFWaves = NF_WAVES;
constexpr int kNFThreads = kNFWaves * kWave;
constexpr int kNFRpw = kNFWaves == 8 ? 4 : 3;  // utterances per wave and batch (at most)
constexpr int kNFRows = kNFWaves * kNFRpw;     // rows of a batch (at most)
constexpr int kNFRT = (kNFRows + 15) / 16;     // MFMA row tiles
constexpr int kNFHot = 32;                  // = mm2_kernels.hip kTextHot
constexpr int kNFLdp = 304;                 // = kTextLdp (T row stride, floats: y columns and the total)
constexpr int kNFLdq = 608;                 // = kTextLdq (text cache row: E | P, floats)
constexpr int kNFHotRow = 604;              // a hot word's E | P row in LDS (151 float4 units)
constexpr int kNFK = 256;                   // K of the audio / visual GEMM (max)
constexpr int kNFLdw = 320;                 // projection columns
constexpr int kNFCT = kNFLdp / 16;          // 16-column tiles of y and the total (19)
constexpr size_t kNFLdsRows = sizeof(float) * (kNFHot * kNFHotRow + kNFRows * kNFLdp) +
                              sizeof(_Float16) * kNFRows * 2 * kNFK + sizeof(float) * 3 * kNFRows;
static_assert(kNFLdsRows % 16 == 0, "the frame-slot scratch is float4-aligned");
// + 1 KB per wave for the frame-slot sums (12 waves: the utterance's own T
// row, free until T is written, holds them instead)
constexpr size_t kNFLds = kNFLdsRows + (kNFWaves == 8 ? 16 * kWave * kNFWaves : 0) + 16;  // + team counters

struct NarrowFusedArgs {
  StreamArgs s;        // ids, table, V, wtab, audio, visual, N, L, D, A, Vd, num_out, aux_out, flag, cmax_part
  const float* ptab;   // [V][kNFLdq]: E | P rows
  const int32_t* hot_slot1;  // [V]
  const int32_t* hot_ids;    // [n_hot]
  int n_hot;
  const _Float16* img;       // piece-ordered weight image (mmb_mm2_split_pieces)
  const float* col_inv;
  const float* c0;
  float* out;                // MMB2 rows [N][D]
  int cb_av;                 // first audio chunk of the image (kq(D) / 32)
  int kq_a, kq_v;            // K rows of the audio / visual pieces (multiples of 32)
  int rpw;                   // utterances per wave and batch (4; 1 or 2 for small N)
  int64_t nb;                // batches of 8 rpw rows (teams: of 4 rpw rows)
  int team_lag;              // teams: team 1 starts after team 0's first stream phase
};

// TM (teams): the workgroup's two halves (waves 0-3 and 4-7, one wave of
// each per SIMD) run batches of 4 rpw rows on their own LDS halves with
// their own (LDS counter) barriers, so that one team's batch GEMM and
// epilogue can run beside the other team's stream phase.
template <int UNR, int HU, int GA_MAX, int GV_MAX, bool TM = false>
__global__ __launch_bounds__(kNFThreads) __attribute__((amdgpu_waves_per_eu(kNFWaves / 4, kNFWaves / 4))) void utt_narrow_fused_kernel(
    NarrowFusedArgs f) {
  static_assert(!TM || kNFWaves == 8, "teams of 4 waves: 8-wave workgroups");
  extern __shared__ __attribute__((aligned(16))) float nf_lds[];
  float* hotEP = nf_lds;                                  // [kNFHot][kNFHotRow]: E | P
  float* sT = hotEP + kNFHot * kNFHotRow;                 // [rows][kNFLdp]
  _Float16* sA = reinterpret_cast<_Float16*>(sT + kNFRows * kNFLdp);  // [rows][2][kNFK] swizzled
  float* s_irs = reinterpret_cast<float*>(sA + kNFRows * 2 * kNFK);   // [rows] 1 / row scale
  float* s_cnt = s_irs + kNFRows;                         // [rows]
  float* s_ok = s_cnt + kNFRows;                          // [rows] 1 = a row of this batch
  float4* s_scr = reinterpret_cast<float4*>(s_ok + kNFRows);  // [waves][64] frame-slot sums
  unsigned* s_team = reinterpret_cast<unsigned*>(s_scr + (kNFWaves == 8 ? kWave * kNFWaves : 0));  // [2]

  const StreamArgs& a = f.s;
  // (holding these pointers in VGPRs instead -- fewer SGPR spills -- measured
  // slower: 4.21 vs 4.08 ms)
  float* const num_out = a.num_out;
  float* const aux_out = a.aux_out;
  float* const mmb_out = f.out;
  const int32_t* const ids_v = a.ids;
  int32_t* const flag_v = a.flag;
  const int V = static_cast<int>(a.V);  // <= 16384 (the text cache)
  constexpr int CT = 2;
  const int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int64_t wid = static_cast<int64_t>(blockIdx.x) * kNFWaves + wave;
  constexpr int kTW = TM ? 4 : kNFWaves;       // waves of a team (the workgroup: one team)
  constexpr int kTRT = TM ? 1 : kNFRT;         // MFMA row tiles of a team's batch
  const int team = TM ? wave >> 2 : 0;
  const int wt = TM ? wave & 3 : wave;          // wave in its team
  const int r0 = TM ? 16 * team : 0;            // the team's first LDS row
  const int L = a.L, D = a.D;
  const int UT = D >> 2, UA = a.A >> 2, UV = a.Vd >> 2;
  const int PA = kWave / UA, PV = kWave / UV;
  const int GA = (L + PA - 1) / PA, GV = (L + PV - 1) / PV;

  // the hot words' E | P rows into LDS
  const int NU = 2 * (D >> 2) + 1;  // float4 units of a cache row: E (D / 4) then P (D / 4 + 1)
  for (int e = tid; e < f.n_hot * NU; e += kNFThreads) {
    const int k = e / NU, u = e - k * NU;
    *reinterpret_cast<float4*>(hotEP + k * kNFHotRow + 4 * u) =
        ld4(f.ptab + static_cast<int64_t>(f.hot_ids[k]) * kNFLdq + 4 * u);
  }

  // one descriptor over the whole text cache: E | P rows | hot slots | hot
  // ids | the weights (mm2_kernels.hip); offset `cbytes` is past its end and
  // reads 0
  const int hbase = V * kNFLdq * 4;              // hot_slot1
  const int wbase = hbase + V * 4 + 4 * kNFHot;  // the weight copy
  const int cbytes = wbase + V * 4;
  const auto prsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(f.ptab), 0, cbytes, 0x00020000);
  // a token's E | P row: unit u = lane + 64 c of slot c (E units [0, UT),
  // P units [UT, NU)); slot 0 is all E, slot 1 E on lanes 64 + lane < UT and
  // P above, slot 2 P or nothing
  constexpr int CQ = 3;
  int vu[CQ], hu[CQ];
#pragma unroll
  for (int c = 0; c < CQ; ++c) {
    const int u = lane + kWave * c;
    vu[c] = u < NU ? 16 * u : cbytes;  // past the cache: reads 0
    hu[c] = 4 * min(u, NU - 1);
  }
  const bool e1 = kWave + lane < UT;  // slot 1 holds an E unit on this lane
  const int voa = ((lane / UA) * a.A + 4 * (lane % UA)) * 4;
  const int vov = ((lane / UV) * a.Vd + 4 * (lane % UV)) * 4;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 cmx[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c) cmx[c] = z4;

  // utterance u of this wave in batch j: row 8 rpw (blockIdx.x + gridDim.x j) + rpw wave + u
  // (teams: 4 rpw (tg + ntg j) + rpw wt + u, team tg = 2 blockIdx.x + team of ntg)
  const int rpw = f.rpw;
  const int nbr = kTW * rpw;  // rows of a batch
  const int nrt = (nbr + 15) / 16;  // MFMA row tiles holding them
  // 32-bit rows and batches (N < 2^31: the launcher checks), 64-bit offsets
  const int N = static_cast<int>(a.N), nb = static_cast<int>(f.nb);
  const int tg = TM ? 2 * static_cast<int>(blockIdx.x) + team : static_cast<int>(blockIdx.x);
  const int ntg = TM ? 2 * static_cast<int>(gridDim.x) : static_cast<int>(gridDim.x);
  auto row_of = [&](int j, int u) -> int { return nbr * (tg + ntg * j) + rpw * wt + u; };
  // the batch barrier: the workgroup's, or the team's 4 waves' (an LDS
  // arrival counter; every wave of a team runs the same batches)
  unsigned bar_target = 0;
  auto bar_batch = [&]() {
    if constexpr (!TM) {
      __syncthreads();
    } else {
      bar_target += kTW;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) {
        __hip_atomic_fetch_add(&s_team[team], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (__hip_atomic_load(&s_team[team], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < bar_target)
          __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
  };
  auto ld_id = [&](int i) -> int {
    if (NF_ABL & 32) return (i < N && lane < L) ? (lane * 131 + i) % V : -1;
    return (i < N && lane < L) ? ids_v[static_cast<int64_t>(i) * L + lane] : -1;
  };
  auto resolve = [&](int raw, int& rid, float& w, int& hs) {
    rid = -1;
    w = 0.f;
    hs = 0;
    if (NF_ABL & 32) {
      if (raw >= 0) rid = raw, w = 1.f;
    } else if (lane < L) {
      int id = raw;
      const bool in = id >= 0 && id < V;
      w = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(prsrc, in ? wbase + id * 4 : cbytes, 0, 0));
      if (id < 0) id += V;
      if (id < 0 || id >= V) {
        if (flag_v) atomicOr(flag_v, MMB_FLAG_ID_RANGE);
      } else {
        rid = id;
        hs = __builtin_amdgcn_raw_buffer_load_b32(prsrc, hbase + rid * 4, 0, 0);
      }
    }
  };

  // MFMA phase: this wave's column tiles wave, wave + 8, wave + 16 (< 20);
  // lane (q, g) holds row / column q, K group g of a 16 x 32 fragment
  const int q = lane & 15, g = lane >> 4;
  constexpr int CH = 2 * kNFLdw * 32, PL = kNFLdw * 32;  // image chunk / plane (halves)
  constexpr int kMaxT = (kNFCT + kTW - 1) / kTW;  // 3 (8 waves), 2 (12) or 5 (teams)
  const int nch = (f.kq_a + f.kq_v) / 32;
  const auto brsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(f.img), 0,
                                                       (f.cb_av + nch) * CH * 2, 0x00020000);
  int boff[kMaxT];
#pragma unroll
  for (int tt = 0; tt < kMaxT; ++tt) {
    const int col = 16 * min(wt + kTW * tt, kNFCT - 1) + q;
    boff[tt] = col * 32 + ((g ^ x3_swz(col)) << 3);
  }
  static_assert(kMaxT == 2 || kMaxT == 3 || kMaxT == 5, "column tiles per wave");
  const int ntt = wt + kTW * (kMaxT - 1) < kNFCT ? kMaxT : kMaxT - 1;  // this wave's column tiles
  float cinv[kMaxT], cc0[kMaxT];  // the tiles' column scales and c0
#pragma unroll
  for (int tt = 0; tt < kMaxT; ++tt) {
    const int col = 16 * min(wt + kTW * tt, kNFCT - 1) + q;
    const bool held = tt < ntt && col < kNFLdp;
    cinv[tt] = held ? f.col_inv[col] : 0.f;
    cc0[tt] = held ? f.c0[col] : 0.f;
  }
  auto ld_b = [&](int c, half8 (&bh)[kMaxT], half8 (&bl)[kMaxT]) {
    const int so = (f.cb_av + c) * CH * 2;
#pragma unroll
    for (int tt = 0; tt < kMaxT; ++tt) {
      if (tt < ntt) {
        bh[tt] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(brsrc, boff[tt] * 2, so, 0));
        bl[tt] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(brsrc, (boff[tt] + PL) * 2, so, 0));
      }
    }
  };

  auto frame_rsrc = [&](int i, const float* base, int W) {
    const bool live = i < N;
    const int64_t ic = live ? i : 0;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base + ic * L * W), 0, live ? L * W * 4 : 0,
                                             0x00020000);
  };
  auto take = [](uint64_t& m) -> int {  // next token of a (uniform) mask, -1 = none
    const int t = m ? __builtin_ctzll(m) : -1;
    m &= m - 1;
    return t;
  };

  // the A rows' pads (K past each piece) stay zero: zeroed once here
  for (int e = tid; e < kNFRows * 2 * kNFK / 8; e += kNFThreads)
    reinterpret_cast<float4*>(sA)[e] = z4;
  if (TM && tid < 2) s_team[tid] = 0u;
  int rid_n, hs_n, raw = -1;  // the next utterance's ids, weights, hot slots
  float w_n;
  resolve(ld_id(row_of(0, 0)), rid_n, w_n, hs_n);
  __syncthreads();  // hot rows in LDS
  if (TM && team == 1 && f.team_lag && tg < nb) {
    // team 1 starts once team 0 (which has a batch if team 1 has) is past its
    // first stream phase: the teams' phases start out of step
    if (lane == 0)
      while (__hip_atomic_load(&s_team[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < static_cast<unsigned>(kTW))
        __builtin_amdgcn_s_sleep(2);
    __builtin_amdgcn_wave_barrier();
  }
  for (int j = 0; j < nb; j += 1) {
    if (tg + ntg * j >= nb) break;
    // ------------------------------------------------------------ stream phase
    for (int u = 0; u < rpw; ++u) {
      const int i = row_of(j, u);
      const int r = r0 + rpw * wt + u;  // LDS row
      const bool live = i < N;
      const int rid = rid_n, hs = hs_n;
      const float w = w_n;
      raw = ld_id(u + 1 < rpw ? row_of(j, u + 1) : row_of(j + 1, 0));
      const auto arsrc = frame_rsrc(i, a.audio, a.A);
      const auto vrsrc = frame_rsrc(i, a.visual, a.Vd);
      float4 sa = z4, saa = z4, sv = z4, svv = z4;
      auto frames = [&](auto gmax, auto rsrc, int vo, int W, int U, int P, int g0, float4& s1, float4& s2) {
        constexpr int GM = decltype(gmax)::value;
        float4 v[GM > 0 ? GM : 1];
#pragma unroll
        for (int g = 0; g < GM; ++g)
          v[g] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo, (g0 + g) * P * W * 4, 2));
        const bool mine = lane < P * U;
        return [=, &s1, &s2]() {
#pragma unroll
          for (int g = 0; g < GM; ++g) {
            if (mine) {
              add4(s1, v[g]);
              sq4(s2, v[g]);
            }
          }
        };
      };
      using GAc = std::integral_constant<int, GA_MAX>;
      using GVc = std::integral_constant<int, GV_MAX>;
      using G0 = std::integral_constant<int, 0>;
      auto acc_a = frames(std::conditional_t<(NF_ABL & 2) != 0, G0, GAc>{}, arsrc, voa, a.A, UA, PA, 0, sa, saa);
      auto acc_v = frames(std::conditional_t<(NF_ABL & 2) != 0, G0, GVc>{}, vrsrc, vov, a.Vd, UV, PV, 0, sv, svv);

      // text: the x sums (w E) and the P rows of the text term over the
      // utterance's valid tokens -- hot words (LDS) while the first group of
      // cold words (global loads) is in flight, then the cold groups.  The
      // order (hot tokens, then cold, each by position) is not
      // utt_narrow_kernel's: x agrees with it to f32 rounding.
      float4 ac[CQ];  // slot sums: w E units, then P units (e1: slot 1 mixes them)
#pragma unroll
      for (int c = 0; c < CQ; ++c) ac[c] = z4;
      const bool tok = lane < L && rid >= 0;
      uint64_t cold = (NF_ABL & 4) ? 0 : __builtin_amdgcn_ballot_w64(tok && hs == 0);
      uint64_t hot = (NF_ABL & 4) ? 0 : __builtin_amdgcn_ballot_w64(tok && hs > 0);
      auto cold_row = [&](int t, float4 (&v)[CQ]) {
        const int rr = t >= 0 ? __builtin_amdgcn_readlane(rid, t) : -1;
        const int so = rr >= 0 ? rr * kNFLdq * 4 : cbytes;  // none: out of range, reads 0
#pragma unroll
        for (int c = 0; c < CQ; ++c)
          v[c] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(prsrc, vu[c], so, 0));
      };
      auto accum = [&](int t, const float4 (&v)[CQ]) {
        const float wt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), t));
        fma4(ac[0], wt, v[0]);
        fma4(ac[1], e1 ? wt : 1.f, v[1]);  // 1 * p + s == p + s exactly
        add4(ac[2], v[2]);
      };
      {
        float4 vc[UNR][CQ];
        int tq[UNR];
#pragma unroll
        for (int q = 0; q < UNR; ++q) {
          tq[q] = take(cold);
          cold_row(tq[q], vc[q]);
        }
        while (hot) {
          float4 vh[HU][CQ];
          int th[HU];
#pragma unroll
          for (int q = 0; q < HU; ++q) {
            th[q] = take(hot);
            const int hh = th[q] >= 0 ? __builtin_amdgcn_readlane(hs, th[q]) - 1 : 0;
            const float* pr = hotEP + hh * kNFHotRow;
#pragma unroll
            for (int c = 0; c < CQ; ++c) vh[q][c] = *reinterpret_cast<const float4*>(pr + hu[c]);
          }
#pragma unroll
          for (int q = 0; q < HU; ++q)
            if (th[q] >= 0) accum(th[q], vh[q]);
        }
        acc_a();
        acc_v();
        for (;;) {
#pragma unroll
          for (int q = 0; q < UNR; ++q)
            if (tq[q] >= 0) accum(tq[q], vc[q]);
          if (!cold) break;
#pragma unroll
          for (int q = 0; q < UNR; ++q) {
            tq[q] = take(cold);
            cold_row(tq[q], vc[q]);
          }
        }
      }
      const float cnt = static_cast<float>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(w != 0.f)));
      const float sw = wave_sum_dpp_f32(w);  // (DPP row sums: another order than wave_sum's)
      if (live && lane == 0 && cnt == 0.f && flag_v) atomicOr(flag_v, MMB_FLAG_ZERO_WEIGHTS);
      for (int g0 = GA_MAX; g0 < GA; g0 += GA_MAX) frames(GAc{}, arsrc, voa, a.A, UA, PA, g0, sa, saa)();
      for (int g0 = GV_MAX; g0 < GV; g0 += GV_MAX) frames(GVc{}, vrsrc, vov, a.Vd, UV, PV, g0, sv, svv)();
      // The A row [Sa | Saa | 0 | Sv | Svv] (K = 4 lane .. 4 lane + 3 on lane
      // `lane`): each frame sum's P row slots added up through this wave's 1
      // KB of LDS (one write, P reads by the lanes holding that piece; slot 0
      // first, as the shuffle reduction of utt_narrow_kernel); pads 0
      float4* scr = kNFWaves == 8 ? s_scr + wave * kWave : reinterpret_cast<float4*>(sT + r * kNFLdp);
      float4 av = z4;
      auto gather = [&](const float4& acc, int U, int P, int u0) {
        __builtin_amdgcn_wave_barrier();  // the previous piece's reads are issued
        scr[lane] = acc;
        __builtin_amdgcn_wave_barrier();
        const int l = lane - u0;
        if (l >= 0 && l < U) {
          av = scr[l];
          for (int q = 1; q < P; ++q) add4(av, scr[l + q * U]);
        }
      };
      gather(sa, UA, PA, 0);
      gather(saa, UA, PA, UA);
      gather(sv, UV, PV, f.kq_a >> 2);
      gather(svv, UV, PV, (f.kq_a >> 2) + UV);
      __builtin_amdgcn_wave_barrier();  // (12 waves: the T row is written below)
      const float rsc = row_scale(wave_max_dpp_f32(amax4(av)));
      resolve(raw, rid_n, w_n, hs_n);  // the next utterance's
      // x (the a2 row), column bounds, aux; the text term T into LDS
      const float rc = 1.f / cnt;
      float* trow = sT + r * kNFLdp;
      // T = sum w E + sum P: the P units into the T row first (unit UT, the
      // total weight column, plus the weight sum; pads 0), then each E unit's
      // lane adds its sum there
#pragma unroll
      for (int c = 1; c < CQ; ++c) {
        const int p = lane + kWave * c - UT;  // P unit of this slot
        if (p >= 0 && p <= UT) {
          float4 tv = ac[c];
          if (p == UT) tv.x += sw;
          *reinterpret_cast<float4*>(trow + 4 * p) = tv;
        }
      }
      if (lane > UT && lane < kNFLdp / 4) *reinterpret_cast<float4*>(trow + 4 * lane) = z4;
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int uu = lane + kWave * c;
        if (uu < UT) {
          const float4 xr = make_float4(ac[c].x * rc, ac[c].y * rc, ac[c].z * rc, ac[c].w * rc);
          if (live) {
            if (!(NF_ABL & 8)) st4(num_out + static_cast<int64_t>(i) * D + 4 * uu, xr);
            cmx[c] = bmax4(cmx[c], xr);
          }
          float4 tv = *reinterpret_cast<const float4*>(trow + 4 * uu);
          add4(tv, ac[c]);
          *reinterpret_cast<float4*>(trow + 4 * uu) = tv;
        }
      }
      // the A row as fp16 hi | lo, row-scaled, swizzled per row
      {
        _Float16* arow = sA + r * 2 * kNFK;
        const int q = r & 15;
        auto put = [&](int k, float4 v) {  // 4 consecutive K at k (k % 4 == 0)
          const int grp = k >> 3, o = ((grp ^ q) << 3) + (k & 7);
          split_store4(arow + o, arow + kNFK + o, v, rsc);
        };
        put(4 * lane, av);  // the whole row, pads included
      }
      if (lane == 0) {
        s_irs[r] = 1.f / rsc;
        s_cnt[r] = cnt;
        s_ok[r] = live ? 1.f : 0.f;
        if (live && !(NF_ABL & 8)) {
          aux_out[i] = cnt;
          aux_out[static_cast<int64_t>(N) + i] = sw;
          aux_out[2 * static_cast<int64_t>(N) + i] = rsc;
        }
      }
    }
    // the first image chunk's B fragments load across the barrier
    half8 bh[kMaxT], bl[kMaxT];
    ld_b(0, bh, bl);
    bar_batch();
    // ------------------------------------------------------------ MFMA phase
    {
      f32x4 acc[kTRT][kMaxT];
#pragma unroll
      for (int rt = 0; rt < kTRT; ++rt)
#pragma unroll
        for (int tt = 0; tt < kMaxT; ++tt) acc[rt][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int c = 0; c < ((NF_ABL & 1) ? 0 : nch); ++c) {
        half8 nh[kMaxT], nl[kMaxT];  // chunk c + 1, in flight during chunk c
        if (c + 1 < nch) ld_b(c + 1, nh, nl);
#pragma unroll
        for (int rt = 0; rt < kTRT; ++rt) {
          if (rt < nrt) {
            // (36-row batches: rows past the last are clamped, their results unused)
            const int rr = r0 + (kNFRows % 16 == 0 ? 16 * rt + q : min(16 * rt + q, kNFRows - 1));
            const int o = (((4 * c + g) ^ q) << 3);
            const half8 ah = *reinterpret_cast<const half8*>(sA + rr * 2 * kNFK + o);
            const half8 al = *reinterpret_cast<const half8*>(sA + rr * 2 * kNFK + kNFK + o);
#pragma unroll
            for (int tt = 0; tt < kMaxT; ++tt) {
              if (tt < ntt) {
                acc[rt][tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[tt], acc[rt][tt], 0, 0, 0);
                acc[rt][tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[tt], acc[rt][tt], 0, 0, 0);
                acc[rt][tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[tt], acc[rt][tt], 0, 0, 0);
              }
            }
          }
        }
#pragma unroll
        for (int tt = 0; tt < kMaxT; ++tt) {
          bh[tt] = nh[tt];
          bl[tt] = nl[tt];
        }
      }
      // y = acc * (col scale * row scale) + T + c0, in place in the T rows
      // (lane value (rt, tt, jj): row 16 rt + 4 g + jj, column 16 ct + q).
      // Every T value and row scale is read before any update is written: in
      // place, each read-modify-write waited for the previous one's store
      // (the compiler cannot tell the rows apart)
      static_assert(kNFCT * 16 <= kNFLdp, "the column tiles lie inside the T rows");
      float irs[kTRT][4], tv[kMaxT][kTRT][4];
#pragma unroll
      for (int rt = 0; rt < kTRT; ++rt)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) irs[rt][jj] = s_irs[r0 + min(16 * rt + 4 * g + jj, kNFRows - 1)];
#pragma unroll
      for (int tt = 0; tt < kMaxT; ++tt) {
        const int col = 16 * min(wt + kTW * tt, kNFCT - 1) + q;
#pragma unroll
        for (int rt = 0; rt < kTRT; ++rt)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            tv[tt][rt][jj] = sT[(r0 + min(16 * rt + 4 * g + jj, kNFRows - 1)) * kNFLdp + col];
      }
#pragma unroll
      for (int tt = 0; tt < kMaxT; ++tt) {
        if (tt < ntt) {
          const int col = 16 * (wt + kTW * tt) + q;
          const float ci = cinv[tt], cc = cc0[tt];
#pragma unroll
          for (int rt = 0; rt < kTRT; ++rt)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              const int rr = 16 * rt + 4 * g + jj;
              if (kNFRows % 16 == 0 ? rt < nrt : rr < nbr)
                sT[(r0 + rr) * kNFLdp + col] = acc[rt][tt][jj] * (ci * irs[rt][jj]) + tv[tt][rt][jj] + cc;
            }
        }
      }
    }
    bar_batch();
    // ------------------------------------------------------------ epilogue
    // wave w finishes rows rpw w .. rpw w + rpw - 1: / total (column D), L2 norm, store
    for (int u = 0; u < rpw; ++u) {
      const int r = r0 + rpw * wt + u;
      const int i = row_of(j, u);
      const float* trow = sT + r * kNFLdp;
      const float rt = __builtin_amdgcn_rcpf(trow[D]);  // v_rcp_f32 (1 ulp): the MMB2 bar is 2e-6
      float4 y[CT];
      float ss = 0.f;
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        const int uu = lane + kWave * c;
        y[c] = *reinterpret_cast<const float4*>(trow + 4 * min(uu, UT - 1));
        y[c] = make_float4(y[c].x * rt, y[c].y * rt, y[c].z * rt, y[c].w * rt);
        if (uu < UT) ss += y[c].x * y[c].x + y[c].y * y[c].y + y[c].z * y[c].z + y[c].w * y[c].w;
      }
      const float inv = __builtin_amdgcn_rsqf(wave_sum_dpp_f32(ss));  // v_rsq_f32 (1 ulp)
      if (s_ok[r] != 0.f && !(NF_ABL & 16)) {
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          const int uu = lane + kWave * c;
          if (uu < UT) st4(mmb_out + static_cast<int64_t>(i) * D + 4 * uu, make_float4(y[c].x * inv, y[c].y * inv, y[c].z * inv, y[c].w * inv));
        }
      }
    }
    bar_batch();  // the T / A rows are rewritten by the next batch
  }
  if (a.cmax_part) {
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const int uu = lane + kWave * c;
      if (uu < UT) st4(a.cmax_part + wid * D + 4 * uu, cmx[c]);
    }
  }
}

// the narrow fused kernel's shapes: gathered ids, a weight table, 256 < d <
// 304 (d % 4), frame rows of 4..128 floats (two or more per instruction,
// A % 4 == Vd % 4 == 0), kq(A) + kq(Vd) <= 256, t <= 64, V <= 16384 (the
// text cache)
}  // namespace mmb

extern "C" int mmb_mm2_stream_project_narrow_supported(int t, int d, int a_, int vd, int64_t v) {
  const int kq = (2 * a_ + 31) / 32 * 32 + (2 * vd + 31) / 32 * 32;
  return t > 0 && t <= kWave && d > 256 && d < kNFLdp && d % 4 == 0 && a_ >= 4 && vd >= 4 &&
         a_ <= 128 && vd <= 128 && a_ % 4 == 0 && vd % 4 == 0 && kq <= kNFK && v > 0 && v <= 16384 &&
         v * (kNFLdq + 2) * 4 + 4 * kNFHot < (int64_t{1} << 31) && static_cast<int64_t>(t) * (a_ > vd ? a_ : vd) * 4 < (int64_t{1} << 31);
}

extern "C" int mmb_mm2_stream_project_narrow(const int32_t* ids, const float* table, int64_t v,
                                             const float* wtab32, const void* text_cache,
                                             const float* audio, const float* visual, int64_t n,
                                             int t, int d, int a_, int vd, const void* wpieces,
                                             const float* c0, float* num_out, float* aux_out,
                                             float* mmb2_out, int32_t* flag, uint32_t* colmax,
                                             void* colmax_ws, hipStream_t stream) {
  MMB_REQUIRE(n >= 0 && n < (int64_t{1} << 31) - kNFRows && mmb_mm2_stream_project_narrow_supported(t, d, a_, vd, v));
  MMB_REQUIRE(ids && table && wtab32 && text_cache && audio && visual && num_out && aux_out &&
              mmb2_out && wpieces && c0);
  MMB_REQUIRE(colmax == nullptr || colmax_ws != nullptr);
  MMB_REQUIRE(aligned16(table) && aligned16(text_cache) && aligned16(audio) && aligned16(visual) &&
              aligned16(num_out) && aligned16(mmb2_out) && aligned16(wpieces));
  if (n == 0) {
    if (colmax) {
      const hipError_t e = static_cast<hipError_t>(zero_words_async(colmax, static_cast<int64_t>(sizeof(uint32_t) * d) / 4, stream));
      if (e != hipSuccess) return static_cast<int>(e);
    }
    return MMB_OK;
  }
  NarrowFusedArgs f{};
  StreamArgs& s = f.s;
  s.ids = ids; s.table = table; s.V = v; s.wtab = wtab32; s.audio = audio; s.visual = visual;
  s.N = n; s.L = t; s.D = d; s.A = a_; s.Vd = vd; s.Kp = mmb_mm2_k(d, a_, vd);
  s.num_out = num_out; s.aux_out = aux_out; s.flag = flag; s.s_half = 1;
  s.cmax_part = colmax ? static_cast<float*>(colmax_ws) : nullptr;
  f.ptab = static_cast<const float*>(text_cache);
  f.hot_slot1 = reinterpret_cast<const int32_t*>(f.ptab + static_cast<size_t>(v) * kNFLdq);
  f.hot_ids = f.hot_slot1 + v;
  f.n_hot = static_cast<int>(v < kNFHot ? v : kNFHot);
  const int kq_t = (2 * d + 31) / 32 * 32;
  f.kq_a = (2 * a_ + 31) / 32 * 32;
  f.kq_v = (2 * vd + 31) / 32 * 32;
  f.cb_av = kq_t / 32;
  f.img = static_cast<const _Float16*>(wpieces);
  f.col_inv = reinterpret_cast<const float*>(f.img + 2 * static_cast<size_t>(kNFLdw) * (kq_t + f.kq_a + f.kq_v));
  f.c0 = c0;
  f.out = mmb2_out;
  // 4 utterances per wave (32-row batches) once that fills every CU; small N
  // (dataset splits) fewer per wave: more workgroups, a shorter chain each
  const int64_t cus = stream_cu_count(stream);
  f.rpw = kNFRpw;
  while (f.rpw > 1 && ceil_div(n, static_cast<int64_t>(kNFWaves) * f.rpw) < cus) --f.rpw;
#ifndef MMB_HOOK_NF_TEAMS  // (tools/diag: MMB_NF_TEAMS)
#define MMB_HOOK_NF_TEAMS 0
#endif
  int teams = MMB_HOOK_NF_TEAMS;  // 1: two teams of 4 waves per workgroup, 2: the same, team 1 starting a phase later
  if (kNFWaves != 8) teams = 0;
  f.team_lag = teams == 2 ? 1 : 0;
  // batches: of 8 rpw rows, or of 4 rpw rows per team (two per workgroup)
  f.nb = ceil_div(n, static_cast<int64_t>(teams ? kNFWaves / 2 : kNFWaves) * f.rpw);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&utt_narrow_fused_kernel<NF_UNR, NF_HU, NF_GA, NF_GV>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kNFLds));
#ifdef MMB_HOOK_NF_TEAMS_ATTR
    MMB_HOOK_NF_TEAMS_ATTR;
#endif
    attr = true;
  }
  int64_t grid = stream_cu_count(stream);
  if (colmax && grid > kCmaxRows / kNFWaves) grid = kCmaxRows / kNFWaves;
  if (grid > (teams ? ceil_div(f.nb, int64_t{2}) : f.nb)) grid = teams ? ceil_div(f.nb, int64_t{2}) : f.nb;
#ifndef MMB_HOOK_NF_TEAMS_LAUNCH
#define MMB_HOOK_NF_TEAMS_LAUNCH false
#endif
  if (!(MMB_HOOK_NF_TEAMS_LAUNCH))
    utt_narrow_fused_kernel<NF_UNR, NF_HU, NF_GA, NF_GV><<<static_cast<unsigned>(grid), kNFThreads, kNFLds, stream>>>(f);
  MMB_LAUNCH_CHECK();
  if (!colmax) return MMB_OK;
  colmax_reduce_kernel<<<static_cast<unsigned>(ceil_div(d, 64)), 1024, 0, stream>>>(
      static_cast<const float*>(colmax_ws), static_cast<int>(grid) * kNFWaves, d, colmax);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

// the tools build's variant launches, knobs and probes (tools/diag/); the
// product library includes an empty header here
#ifndef MMB_TOOLS_TAIL_SIF
#define MMB_TOOLS_TAIL_SIF "mmb_no_tools.h"
#endif
#include MMB_TOOLS_TAIL_SIF
