// First-principal-component removal (a3/a4) for MI355X.
//
// The reference computes the PC with scikit-learn's randomized SVD
// (TruncatedSVD(npc, n_iter=7, random_state=0), sif_functions.py:58-67), which
// makes ~15 passes over X.  Here X is read ONCE for its 300x300 Gram
// G = X^T X (fp64 MFMA: products of f32 values are exact in f64), the Gram is
// the only thing that crosses GPUs (RCCL all-reduce, 720 KB), and the
// randomized SVD is replayed on G in one workgroup:
//   * direct branch (n >= d): Z0 = Omega [d,k] (RandomState(0).normal);
//     span(G^n_iter Z0) is the span the reference's LU-normalised iterations
//     build (LU/QR only right-multiply the block); the final SVD of Q^T X with
//     Q = orth(X Z) reduces to the k x k generalised symmetric eigenproblem
//     (Z^T G^2 Z) y = s^2 (Z^T G Z) y, v = G Z y;
//   * transposed branch (n < d, extmath.py:562-566): Z0 = X^T Omega_n, the same
//     iterations, then v = Z u with u the top eigenvector of Z^T G Z;
//   * svd_flip(u_based_decision=False): largest-|.| entry of each component > 0.
// The removal pass x - (x.pc) pc runs in f64 like the reference (:77-80).
#include <algorithm>
#include <vector>

#include "mmb_common.h"

namespace mmb {

using f64x4 = __attribute__((ext_vector_type(4))) double;

constexpr int kGB = 64;  // Gram block edge per workgroup (4 waves x 32x32)

__host__ __device__ inline int gram_pair_index(int bp, int bq, int nb) {
  return bp * nb - bp * (bp - 1) / 2 + (bq - bp);
}

__device__ __forceinline__ float load_x(const float* __restrict__ num, const float* __restrict__ cnt,
                                        int64_t row, int col, int D) {
  if (col >= D) return 0.f;
  const float v = num[row * D + col];
  return cnt ? v / cnt[row] : v;  // x = num / count_nonzero(w), f32 (sif_functions.py:55)
}
// float64 rows (the numpy drop-in's general f64 X, sif_functions.py:58-81): no count
__device__ __forceinline__ double load_x(const double* __restrict__ num, const float* __restrict__,
                                         int64_t row, int col, int D) {
  return col < D ? num[row * D + col] : 0.0;
}

// One workgroup: a 64x64 block (bp,bq), bp<=bq, of G over one chunk of rows.
// fp64 MFMA 16x16x4: lane l holds A[l&15][l>>4] and B[l>>4][l&15]; with
// A = X^T and B = X both fragments are 16 consecutive columns of 4 rows of X.
template <typename TX>
__global__ __launch_bounds__(256) void gram_partial_kernel(const TX* __restrict__ num,
                                                           const float* __restrict__ cnt,
                                                           int64_t N, int D, int nb, int npairs,
                                                           int S, int64_t chunk, int xcd_map,
                                                           double* __restrict__ part) {
  int pair, s;
  if (xcd_map) {
    // blocks b and b+8 share an XCD (round-robin dispatch; speed only): give
    // every pair of one row chunk to one XCD so the chunk is fetched once per L2.
    const int b = blockIdx.x, x = b & 7, local = b >> 3;
    s = x + 8 * (local / npairs);
    pair = local % npairs;
  } else {
    pair = blockIdx.x % npairs;
    s = blockIdx.x / npairs;
  }
  int bp = 0, rem = pair;
  while (rem >= nb - bp) {
    rem -= nb - bp;
    ++bp;
  }
  const int bq = bp + rem;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wp = wave >> 1, wq = wave & 1;
  const int ca0 = bp * kGB + wp * 32 + (lane & 15), ca1 = ca0 + 16;
  const int cb0 = bq * kGB + wq * 32 + (lane & 15), cb1 = cb0 + 16;
  const int kr = lane >> 4;
  const int64_t n0 = s * chunk;
  const int64_t n1 = min(N, n0 + chunk);
  f64x4 acc00 = {0, 0, 0, 0}, acc01 = acc00, acc10 = acc00, acc11 = acc00;
#pragma unroll 4
  for (int64_t n = n0; n < n1; n += 4) {
    const int64_t row = n + kr;
    double a0 = 0, a1 = 0, b0 = 0, b1 = 0;
    if (row < n1) {
      a0 = load_x(num, cnt, row, ca0, D);
      a1 = load_x(num, cnt, row, ca1, D);
      b0 = load_x(num, cnt, row, cb0, D);
      b1 = load_x(num, cnt, row, cb1, D);
    }
    acc00 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc00, 0, 0, 0);
    acc01 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc01, 0, 0, 0);
    acc10 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc10, 0, 0, 0);
    acc11 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc11, 0, 0, 0);
  }
  // f64 C/D layout: col = lane&15, row = (lane>>4) + 4*reg
  double* out = part + (static_cast<int64_t>(s) * npairs + pair) * (kGB * kGB);
  const int c = lane & 15, r0 = lane >> 4;
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) {
    const int i0 = wp * 32 + r0 + 4 * reg, j0 = wq * 32 + c;
    out[i0 * kGB + j0] = acc00[reg];
    out[i0 * kGB + j0 + 16] = acc01[reg];
    out[(i0 + 16) * kGB + j0] = acc10[reg];
    out[(i0 + 16) * kGB + j0 + 16] = acc11[reg];
  }
}

// ------------------------------------------------------------------ Gram v2
// Upper triangle of G in 16x16 tiles (D <= 320: 20 tile rows, 210 tiles).  A
// PAIR of 16-wave workgroups owns one contiguous row range: each stages the
// range's rows once in LDS as f64 (16 rows per chunk, double-buffered, the
// next chunk's global loads in flight during the current chunk's MFMAs) and
// computes half of the tiles (~7 per wave, fp64 MFMA 16x16x4 — one k-step is
// 4 rows).  The pair sits on one XCD (blocks b and b+8) so the second read of
// the rows hits L2.  Per-range partials are summed in a fixed order.
constexpr int kG2NT = 1024;
constexpr int kG2Rows = 16;            // rows per LDS chunk (4 MFMA k-steps)
constexpr int kG2Stride = 336;         // doubles per LDS row: 320 + 16 (rows alternate bank halves)
constexpr int kG2MaxTiles = 8;         // tiles per wave

__device__ __forceinline__ void tri_tile(int tau, int nt, int& ti, int& tj) {
  int r = 0, rem = tau;
  while (rem >= nt - r) {
    rem -= nt - r;
    ++r;
  }
  ti = r;
  tj = r + rem;
}

// ------------------------------------------------------------------ Gram, small n (r05)
// Dataset splits (MOSI 229-1284 rows, POM 100-203) take the exact f64 Gram.
// The row-range kernel below spends its time there on fixed costs: 16 ranges
// of 80 rows, every workgroup writing 95 tiles of partials that a second
// launch reduces (37 us per split, r04 dataset_splits).  For n <= 4096 this
// kernel is tile-parallel instead: one workgroup per 16 x 16 tile of the
// upper triangle over ALL rows, its 16 waves taking strided 4-row k-steps
// (fp64 MFMA 16x16x4: f32 x f32 products exact in f64), the 16 partial tiles
// summed in a fixed order through LDS and written straight into G (and its
// mirror): one launch, no partials.
constexpr int kGsNT = 1024;
constexpr int64_t kGsMaxN = 4096;

template <int G = 8>
__global__ __launch_bounds__(kGsNT) void gram_small_kernel(const float* __restrict__ num,
                                                           const float* __restrict__ cnt,
                                                           int64_t N, int D, int nt, int accumulate,
                                                           double* __restrict__ g) {
  __shared__ double s_acc[kGsNT / kWave][256];
  int bi, bj;
  tri_tile(blockIdx.x, nt, bi, bj);
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  constexpr int NW = kGsNT / kWave;
  const int ca = 16 * bi + (lane & 15), cb = 16 * bj + (lane & 15), kr = lane >> 4;
  f64x4 acc = {0, 0, 0, 0};
  // wave w: k-steps w, w + 16, ... (4 rows each), loads issued ahead in
  // groups of G k-steps (one round trip per group)
  const int64_t nks = (N + 3) / 4;
  for (int64_t s0 = wave; s0 < nks; s0 += NW * G) {
    double av[G], bv[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int64_t row = (s0 + NW * u) * 4 + kr;
      const bool ok = s0 + NW * u < nks && row < N;
      av[u] = ok ? static_cast<double>(load_x(num, cnt, row, ca, D)) : 0.0;
      bv[u] = ok ? static_cast<double>(load_x(num, cnt, row, cb, D)) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < G; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc, 0, 0, 0);
  }
  // C/D layout: col = lane & 15, row = (lane >> 4) + 4 reg
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) s_acc[wave][((lane >> 4) + 4 * reg) * 16 + (lane & 15)] = acc[reg];
  __syncthreads();
  if (threadIdx.x >= 256) return;
  const int e = threadIdx.x, r = e >> 4, c = e & 15;
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < NW; ++w) s += s_acc[w][e];
  const int p = 16 * bi + r, q = 16 * bj + c;
  if (p >= D || q >= D) return;
  const int64_t e1 = static_cast<int64_t>(p) * D + q;
  g[e1] = accumulate ? g[e1] + s : s;
  if (bi != bj) {
    const int64_t e2 = static_cast<int64_t>(q) * D + p;
    g[e2] = accumulate ? g[e2] + s : s;
  }
}


__global__ __launch_bounds__(kG2NT) void gram_tri_kernel(const float* __restrict__ num,
                                                         const float* __restrict__ cnt, int64_t N,
                                                         int D, int nt, int R, int64_t chunk,
                                                         int xcd_map, int acc_part,
                                                         double* __restrict__ part) {
  extern __shared__ double s_x[];  // [2][kG2Rows][kG2Stride]
  const int T = nt * (nt + 1) / 2;
  int half, range;
  if (xcd_map) {
    const int b = blockIdx.x;
    half = (b >> 3) & 1;
    range = (b & 7) + 8 * (b >> 4);
  } else {
    half = blockIdx.x & 1;
    range = blockIdx.x >> 1;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t0 = half * ((T + 1) / 2), t1 = half ? T : (T + 1) / 2;
  // this wave's tiles: wave, wave+16, ... within [t0, t1)
  int ti[kG2MaxTiles], tj[kG2MaxTiles];
  int ntl = 0;
#pragma unroll
  for (int q = 0; q < kG2MaxTiles; ++q) {
    const int tau = t0 + wave + (kG2NT / kWave) * q;
    ti[q] = tj[q] = 0;
    if (tau < t1) {
      tri_tile(tau, nt, ti[q], tj[q]);
      ntl = q + 1;
    }
  }
  f64x4 acc[kG2MaxTiles];
#pragma unroll
  for (int q = 0; q < kG2MaxTiles; ++q) acc[q] = f64x4{0, 0, 0, 0};

  const int64_t r0 = range * chunk;
  const int64_t r1 = min(N, r0 + chunk);
  const int nchunks = static_cast<int>(r1 > r0 ? (r1 - r0 + kG2Rows - 1) / kG2Rows : 0);
  const int U = D >> 2;  // float4 units per row (D % 4 == 0)
  // staging map: thread -> (row, float4 unit); 16 rows x 80 units (padded to 320 cols)
  const int srow = tid / 80, sunit = tid % 80;  // tid < 1280 covers 16 x 80; 1024 threads: 2 passes
  auto load_regs = [&](int c, float4 (&v)[2], float (&sc)[2]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + kG2NT * q;
      const int rr = idx / 80, uu = idx % 80;
      const int64_t row = r0 + static_cast<int64_t>(c) * kG2Rows + rr;
      v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      sc[q] = 1.f;
      if (idx < kG2Rows * 80 && row < r1 && uu < U) {
        v[q] = *reinterpret_cast<const float4*>(num + row * D + 4 * uu);
        if (cnt) sc[q] = cnt[row];
      }
    }
  };
  auto store_lds = [&](int buf, const float4 (&v)[2], const float (&sc)[2]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = tid + kG2NT * q;
      if (idx < kG2Rows * 80) {
        const int rr = idx / 80, uu = idx % 80;
        double* dst = s_x + (buf * kG2Rows + rr) * kG2Stride + 4 * uu;
        // x = num / count in f32 (sif_functions.py:55), then exact f64
        // widening; two 16-byte writes (ds_write_b128: the 8 lanes of a
        // write phase hit disjoint banks at this 32-byte lane stride, where
        // four 8-byte writes conflicted 2-way)
        using d2 = double __attribute__((ext_vector_type(2)));
        const d2 lo = {static_cast<double>(cnt ? v[q].x / sc[q] : v[q].x),
                       static_cast<double>(cnt ? v[q].y / sc[q] : v[q].y)};
        const d2 hi = {static_cast<double>(cnt ? v[q].z / sc[q] : v[q].z),
                       static_cast<double>(cnt ? v[q].w / sc[q] : v[q].w)};
        *reinterpret_cast<d2*>(dst) = lo;
        *reinterpret_cast<d2*>(dst + 2) = hi;
      }
    }
  };
  (void)srow;
  (void)sunit;
  float4 pv[2];
  float psc[2];
  if (nchunks > 0) {
    load_regs(0, pv, psc);
    store_lds(0, pv, psc);
  }
  __syncthreads();
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    if (c + 1 < nchunks) load_regs(c + 1, pv, psc);
    const double* xb = s_x + buf * kG2Rows * kG2Stride;
#pragma unroll
    for (int s = 0; s < kG2Rows / 4; ++s) {
      const double* xr = xb + (4 * s + (lane >> 4)) * kG2Stride + (lane & 15);
#pragma unroll
      for (int q = 0; q < kG2MaxTiles; ++q) {
        if (q < ntl) {
          const double a = xr[16 * ti[q]];
          const double b = xr[16 * tj[q]];
          acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
        }
      }
    }
    if (c + 1 < nchunks) store_lds(buf ^ 1, pv, psc);
    __syncthreads();
  }
  // partial tiles: part[range][tau][16*16], C/D f64 layout col = lane&15, row = (lane>>4)+4*reg
  double* pr = part + static_cast<int64_t>(range) * T * 256;
#pragma unroll
  for (int q = 0; q < kG2MaxTiles; ++q) {
    if (q < ntl) {
      const int tau = t0 + wave + (kG2NT / kWave) * q;
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        // acc_part: add to this range's partial of the previous row chunk (each
        // element has one owner wave: no race; chunks run in stream order)
        double* dst = pr + static_cast<int64_t>(tau) * 256 + ((lane >> 4) + 4 * reg) * 16 + (lane & 15);
        *dst = acc_part ? *dst + acc[q][reg] : acc[q][reg];
      }
    }
  }
}


// ------------------------------------------------------------------ Gram i8
// G = X^T X on the int8 matrix pipe (v_mfma_i32_16x16x64_i8: 64x the fp64
// MFMA rate per operation), for the fused step's x rows.  Each value becomes
// a 30-bit fixed-point integer of its column's power-of-two bound 2^e_j
// (colmax: max |x| of the column):  v = rint(x 2^(30 - e_j)), |v| < 2^30,
// cut into four balanced base-256 digits (the low three sign-extended bytes
// in [-128, 127], the top one in [-64, 64]):  v = sum_a d_a 2^(8 (3 - a)).
// G_ij = 2^(e_i + e_j - 60) sum_rows v_i v_j, keeping the digit pairs of
// level a + b <= 4 (13 of 16; the dropped (2,3), (3,2), (3,3) weigh 2^8 and
// 1 against the top pair's 2^48).  Per 64-row k-step the levels are summed
// EXACTLY in three int32 accumulators, H = acc_0 2^8 + acc_1 (< 2^27),
// M = acc_2 2^8 + acc_3 (< 2^30), L = acc_4, then added in f64 as
// H 2^-20 + M 2^-36 + L 2^-44.  The only roundings are v's (2^-31 of the
// column bound per value) and the f64 accumulation: G within 1e-10 of the
// exact f64 Gram on the golden splits (7e-10 on heavy-tailed t(3) columns),
// the PC within 6e-11 of the reference's (CPU restatement:
// oracle.sif_oracle.sliced_gram; the digit format was chosen by measuring
// it: base-128 digits of 33-bit values needed 22 pairs for the same error,
// because values far below their column's bound live in the low digits).
// Structure as gram_tri_kernel: a pair of workgroups per row range (same
// XCD), each with half of the 16x16 tiles of the upper triangle; per 64-row
// chunk every thread turns its (feature, 16-row) items into digit bytes in
// LDS ([digit][feature][4 slots of 16 rows], the conflict-free slot swizzle
// of the 16x16x32 f16 fragment reads, whose lane map this read shares), then
// each wave runs 13 MFMAs per tile and the f64 update.
constexpr int kGiRows = 64;
constexpr int kGiF = 320;       // padded feature count (D <= 320)
constexpr int kGiDig = 4;       // base-256 digits per value

// 16-byte slot swizzle of a feature's 64-byte digit row: slot kq of feature
// f sits at kq ^ gi_swz(f).  (f >> 1) & 3 keeps the MFMA operand reads
// (ds_read_b128 lane groups: features 16 t + (l & 15) at slot l >> 4)
// conflict-free AND the slicing writes (ds_write_b128 groups of 8 lanes = 8
// consecutive features at one slot) -- the r04 swizzle over f >> 2 left the
// writes 2-way (checked exhaustively, r05).
__host__ __device__ constexpr int gi_swz(int f) { return (f >> 1) & 3; }

using i32x4 = __attribute__((ext_vector_type(4))) int;

__device__ __forceinline__ int gi_exp(unsigned bits) {
  const float m = __uint_as_float(bits);
  if (!(m > 0.f) || !isfinite(m)) return 0;
  int e;
  frexpf(m, &e);  // m = f 2^e, f in [0.5, 1): |x| <= m < 2^e
  return e;
}

// v' = rint(x 2^(30 - e)) + 0x808080: byte i < 3 of v' is d_i + 128 for the
// balanced digit d_i in [-128, 127] (so XOR 0x80 gives d_i's two's-complement
// byte), byte 3 is the top digit d_3 itself (|d_3| <= 64):
//   v = sum_i d_i 256^i  =>  v + 128 (1 + 256 + 65536) = sum_i (d_i + 128) 256^i
// for the low three, the top untouched.
__device__ __forceinline__ unsigned gi_vbias(float x, int e) {
  return static_cast<unsigned>(static_cast<int>(rintf(ldexpf(x, 30 - e)))) + 0x808080u;
}

// 4 values (rows r..r+3) -> the 4 digit-plane dwords, top digit first
// (a 4 x 4 byte transpose in 8 v_perm_b32, then the bias flip)
__device__ __forceinline__ void gi_planes(unsigned v0, unsigned v1, unsigned v2, unsigned v3,
                                          unsigned (&w)[4]) {
  const unsigned p0 = __builtin_amdgcn_perm(v1, v0, 0x05010400u);  // v0.b0 v1.b0 v0.b1 v1.b1
  const unsigned p1 = __builtin_amdgcn_perm(v1, v0, 0x07030602u);  // v0.b2 v1.b2 v0.b3 v1.b3
  const unsigned q0 = __builtin_amdgcn_perm(v3, v2, 0x05010400u);
  const unsigned q1 = __builtin_amdgcn_perm(v3, v2, 0x07030602u);
  w[0] = __builtin_amdgcn_perm(q1, p1, 0x07060302u);                // byte 3: top digit
  w[1] = __builtin_amdgcn_perm(q1, p1, 0x05040100u) ^ 0x80808080u;  // byte 2
  w[2] = __builtin_amdgcn_perm(q0, p0, 0x07060302u) ^ 0x80808080u;  // byte 1
  w[3] = __builtin_amdgcn_perm(q0, p0, 0x05040100u) ^ 0x80808080u;  // byte 0
}

// ------------------------------------------------------------------ Gram i8, range level sums (r05)
// The same digits and the same 13 digit-pair products as gram_i8_kernel, but
// each of the five levels l = a + b is summed in its OWN int32 accumulator
// over the workgroup's whole row range, and the range's f64 partial is formed
// once at the end:  S = (((L0 2^8 + L1) 2^8 + L2) 2^8 + L3) 2^8 + L4 (exact in
// f64 up to the last step, which rounds once), G_part = S 2^(e_i + e_j - 44).
// gram_i8_kernel shifted and combined the levels into three words per 64-row
// k-step and added them to f64 accumulators: per tile and k-step 8 shifts,
// 12 conversions and 12 f64 FMAs beside the 13 MFMAs -- with the digit
// slicing, ~700 vector instructions per wave and chunk against 156 MFMAs, a
// kernel bound by vector issue (0.76 ms at 1M x 300), not by the matrix pipe
// (~0.3 ms of MFMA work).  Here the k-step loop issues the MFMAs, their
// operand reads and the slicing only.
// Exactness: per 64-row k-step |L0| <= 64 * 64 * 64 = 2^18, |L1| <= 2^20,
// |L2| <= 2^21, |L3|, |L4| <= 2^21.6, so int32 level sums are exact for 512
// k-steps: a range holds at most kGlMaxRows = 32768 rows (gram_i8l_plan).
// Registers: 5 levels x 4 words per 16x16 tile, so a workgroup holds fewer
// tiles than gram_i8_kernel's pairs: THREE workgroups per row range (on one
// XCD: the range's x is read from HBM once), each a contiguous run of the
// row-major triangle (<= 64 tiles, <= 8 per wave), split on the host so that
// the vector work -- a part slices only the features its tiles touch, from
// its first tile row on -- and the MFMA work balance (gram_i8l_split).
constexpr int kGlLev = 5;
constexpr int64_t kGlMaxRows = 512 * kGiRows;        // int32 level sums exact
constexpr int kGlMaxParts = 4;
constexpr int kGlMaxPartTiles = 64;

// One workgroup's share of a range's work: its tiles (ti | tj << 8, grouped
// by tile row for A reuse) and the features it slices, [f0, f0 + n0) and
// [f1, f1 + n1) -- every feature its tiles touch (gram_i8l_parts).
struct GlPart {
  int n, f0, n0, f1, n1;
  uint16_t tile[kGlMaxPartTiles];
};
struct GlParts {
  GlPart p[kGlMaxParts];
};

// Shape of a level-sum kernel: P workgroups per row range, NW waves each, at
// most MT tiles per wave (P * NW * MT >= 190 tiles at d = 300); IT slicing
// items (16 rows of one feature) per thread.
// SB: the mask of the scheduling barrier between tiles (0: nothing crosses;
// 0x100: LDS reads may move up into the previous tile); PF: the next tile's
// first B digit is read during the current tile's MFMAs (4 VGPRs).
// ST: staggered slicing -- waves 0 .. NW/2-1 slice each item BEFORE their
// run of tiles, waves NW/2 .. NW-1 (their SIMD partners) AFTER it, so one
// wave of a SIMD slices while the other issues MFMAs; each item's x for the
// chunk after next is loaded as soon as it is sliced.
template <int P, int NW, int MT, int IT, int SB = 0, bool PF = false, bool ST = false>
struct GlShape {
  static constexpr int kP = P, kNW = NW, kMT = MT, kNT = NW * kWave, kSB = SB;
  static constexpr bool kPF = PF, kST = ST;
  // staggered: the slice point of item u (before tile p; p = MT: after the last)
  static constexpr int slice_before(int u, bool second) { return ((u + (second ? 1 : 0)) * MT) / IT; }
  static constexpr int kPartMax = NW * MT < kGlMaxPartTiles ? NW * MT : kGlMaxPartTiles;
  static constexpr int kIt = IT;
  // item u is sliced after tile slice_at(u): spread over the tile loop
  static constexpr int slice_at(int u) { return (u * MT) / kIt + MT / kIt - 1; }
};

// DIAG (timing-only builds, wrong results; MMB_GRAM_DIAG with the level-sum
// kernel): bit 0 no MFMAs (operands kept live), bit 2 no slicing, bit 3 no x loads
template <int DIAG, class S>
__global__ __launch_bounds__(S::kNT) void gram_i8l_kernel(const float* __restrict__ x,
                                                         const unsigned* __restrict__ colmax,
                                                         int64_t N, int D, int nt, int64_t chunk,
                                                         int xcd_map, GlParts parts,
                                                         double* __restrict__ part) {
  constexpr int MT = S::kMT, NT = S::kNT, kIt = S::kIt;
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dig[];  // [2][4][kGiF][64]
  int range, p;
  if (xcd_map) {  // the P parts of a range on one XCD (round-robin dispatch: b % 8)
    const int b = blockIdx.x, s = b >> 3;
    range = (b & 7) + 8 * (s / S::kP);
    p = s % S::kP;
  } else {
    range = blockIdx.x / S::kP;
    p = blockIdx.x % S::kP;
  }
  const GlPart& pt = parts.p[p];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int npt = pt.n;
  if (npt <= 0) return;  // an empty part (tiny d)
  const int per = (npt + S::kNW - 1) / S::kNW;
  const int q0 = wave * per;
  int ti[MT], tj[MT];
  int ntl = 0;
#pragma unroll
  for (int q = 0; q < MT; ++q) {
    ti[q] = tj[q] = 0;
    if (q < per && q0 + q < npt) {
      const int t = pt.tile[q0 + q];
      ti[q] = t & 255;
      tj[q] = t >> 8;
      ntl = q + 1;
    }
  }
  i32x4 lev[MT][kGlLev];
#pragma unroll
  for (int q = 0; q < MT; ++q)
#pragma unroll
    for (int l = 0; l < kGlLev; ++l) lev[q][l] = i32x4{0, 0, 0, 0};

  const int64_t r0 = range * chunk;
  const int64_t r1 = min(N, r0 + chunk);
  const int nchunks = static_cast<int>(r1 > r0 ? (r1 - r0 + kGiRows - 1) / kGiRows : 0);
  // the features this part slices: two ranges (every feature its tiles touch)
  const int f0 = pt.f0, n0 = pt.n0, f1 = pt.f1;
  const int nf = n0 + pt.n1;
  const int nitems = nf * 4;
  // item it = k + nf * kq: the k-th sliced feature f, rows 16 kq .. 16 kq + 15
  // of the chunk; packed (f | kq << 9 | (e + 256) << 11) with its row offset
  int it_pk[kIt], it_off[kIt];
#pragma unroll
  for (int u = 0; u < kIt; ++u) {
    const int it = tid + NT * u;
    const int k = it < nitems ? it % nf : 0;
    const int f = it < nitems ? (k < n0 ? f0 + k : f1 + k - n0) : 0;
    const int kq = it < nitems ? it / nf : 0;
    const int e = (it < nitems && f < D) ? gi_exp(colmax[f]) : 0;
    it_pk[u] = f | (kq << 9) | ((e + 256) << 11);
    // padding features / missing items read past the record count: 0
    it_off[u] = (it < nitems && f < D) ? (kq * 16 * D + f) * 4 : 0x7ffffff0;
  }
  const int nrec = __builtin_amdgcn_readfirstlane(static_cast<int>((r1 > r0 ? r1 - r0 : 0) * D * 4));
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x + r0 * D), 0, nrec, 0x00020000);
  float xv[kIt][16];
  auto load = [&](int c) {
    if constexpr ((DIAG & 8) != 0) {
#pragma unroll
      for (int u = 0; u < kIt; ++u)
#pragma unroll
        for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(xv[u][j]));
      return;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int so = __builtin_amdgcn_readfirstlane((c * kGiRows + j) * D * 4);
#pragma unroll
      for (int u = 0; u < kIt; ++u)
        xv[u][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, it_off[u], so, 0));
    }
  };
  auto load_item = [&](int u, int c) {
    if constexpr ((DIAG & 8) != 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(xv[u][j]));
      return;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int so = __builtin_amdgcn_readfirstlane((c * kGiRows + j) * D * 4);
      xv[u][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, it_off[u], so, 0));
    }
  };
  auto slice_item = [&](int u, unsigned char* buf) {
    if constexpr ((DIAG & 4) != 0) return;
    const int it = tid + NT * u;
    if (it < nitems) {
      const int f = it_pk[u] & 511, kq = (it_pk[u] >> 9) & 3, e = (it_pk[u] >> 11) - 256;
      unsigned w[4][kGiDig];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        gi_planes(gi_vbias(xv[u][4 * g + 0], e), gi_vbias(xv[u][4 * g + 1], e),
                  gi_vbias(xv[u][4 * g + 2], e), gi_vbias(xv[u][4 * g + 3], e), w[g]);
      const int slot = kq ^ gi_swz(f);
#pragma unroll
      for (int a = 0; a < kGiDig; ++a)
        *reinterpret_cast<uint4*>(buf + ((a * kGiF + f) * 4 + slot) * 16) =
            make_uint4(w[0][a], w[1][a], w[2][a], w[3][a]);
    }
  };
  constexpr int kBuf = kGiDig * kGiF * kGiRows;

  // double-buffered digits, one barrier per 64-row chunk (as gram_i8_kernel)
  if (nchunks > 0) {
    load(0);
#pragma unroll
    for (int u = 0; u < kIt; ++u) slice_item(u, s_dig);
    if (nchunks > 1) load(1);
  }
  __syncthreads();
  const int lf = lane & 15, lsl = lane >> 4;
  for (int c = 0; c < nchunks; ++c) {
    const unsigned char* cur = s_dig + (c & 1) * kBuf;
    unsigned char* nxt = s_dig + ((c + 1) & 1) * kBuf;
    const bool more = c + 1 < nchunks;
    i32x4 A[kGiDig];
    auto ld_b = [&](const unsigned char* buf, int fb, int b) {
      return *reinterpret_cast<const i32x4*>(buf + ((b * kGiF + fb) * 4 + (lsl ^ gi_swz(fb))) * 16);
    };
    i32x4 Bn0 = {0, 0, 0, 0};
    if constexpr (S::kPF) {
      if (ntl > 0) Bn0 = ld_b(cur, tj[0] * 16 + lf, 0);
    }
    const bool second = wave >= S::kNW / 2;
    // staggered slicing: the items whose slice point is before tile p
    auto slice_point = [&](int p) {
      if constexpr (S::kST) {
#pragma unroll
        for (int u = 0; u < kIt; ++u) {
          if (S::slice_before(u, second) == p && more) {
            slice_item(u, nxt);
            if (c + 2 < nchunks) load_item(u, c + 2);
          }
        }
      }
    };
#pragma unroll
    for (int q = 0; q < MT; ++q) {
      slice_point(q);
      if (q < ntl) {
        if (q == 0 || ti[q] != ti[q - 1]) {  // the row block changes (wave-uniform)
          const int fa = ti[q] * 16 + lf;
#pragma unroll
          for (int a = 0; a < kGiDig; ++a)
            A[a] = *reinterpret_cast<const i32x4*>(cur + ((a * kGiF + fa) * 4 + (lsl ^ gi_swz(fa))) * 16);
        }
        const int fb = tj[q] * 16 + lf;
        i32x4 Bd[kGiDig];
#pragma unroll
        for (int b = 0; b < kGiDig; ++b)
          Bd[b] = (S::kPF && b == 0) ? Bn0 : ld_b(cur, fb, b);
        if constexpr (S::kPF) {
          if (q + 1 < ntl) Bn0 = ld_b(cur, tj[q + 1] * 16 + lf, 0);
        }
        // B digit by digit: digit b meets A digits a <= 4 - b (levels a + b <= 4)
#pragma unroll
        for (int b = 0; b < kGiDig; ++b) {
          const i32x4 B = Bd[b];
          if constexpr ((DIAG & 1) != 0) {
            asm volatile("" ::"v"(B));
          } else {
#pragma unroll
            for (int a = 0; a < kGiDig; ++a)
              if (a + b < kGlLev)
                lev[q][a + b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[a], B, lev[q][a + b], 0, 0, 0);
          }
        }
        if constexpr ((DIAG & 1) != 0) {
#pragma unroll
          for (int a = 0; a < kGiDig; ++a) asm volatile("" ::"v"(A[a]));
        }
      }
      // the next chunk's slicing spread between the tiles: VALU work beside
      // the MFMAs in flight
      if constexpr (!S::kST) {
#pragma unroll
        for (int u = 0; u < kIt; ++u)
          if (S::slice_at(u) == q && more) slice_item(u, nxt);
      }
      __builtin_amdgcn_sched_barrier(S::kSB);
    }
    slice_point(MT);
    if (!S::kST && c + 2 < nchunks) load(c + 2);
    __syncthreads();
  }
  // the range's partials: S exact to the last step, one rounding, then the
  // exact power-of-two scale; a non-finite bound gives NaN rows / columns
  const int T = nt * (nt + 1) / 2;
  double* pr = part + static_cast<int64_t>(range) * T * 256;
  const int lc = lane & 15, lr = 4 * (lane >> 4);
#pragma unroll
  for (int q = 0; q < MT; ++q) {
    if (q < ntl) {
      const int tau = ti[q] * nt - ti[q] * (ti[q] - 1) / 2 + (tj[q] - ti[q]);  // row-major triangle
      const int fj = tj[q] * 16 + lc;
      const int ej = fj < D ? gi_exp(colmax[fj]) : 0;
      const bool okj = fj >= D || isfinite(__uint_as_float(colmax[fj]));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int fi = ti[q] * 16 + lr + e;
        const int ei = fi < D ? gi_exp(colmax[fi]) : 0;
        const bool bad = (fi < D && !isfinite(__uint_as_float(colmax[fi]))) || !okj;
        double sum = static_cast<double>(lev[q][0][e]);
#pragma unroll
        for (int l = 1; l < kGlLev; ++l) sum = fma(sum, 256.0, static_cast<double>(lev[q][l][e]));
        pr[static_cast<int64_t>(tau) * 256 + (lr + e) * 16 + lc] =
            bad ? __builtin_nan("") : ldexp(sum, ei + ej - 44);
      }
    }
  }
}

// product shape: three workgroups per range (80 ranges), 8 waves, <= 8 tiles
// per wave, each slicing two of three feature groups (<= 2 items per
// thread), staggered slicing between SIMD partners (r05, tools/gram_ab.py at
// 1M x 300: 0.62-0.63 ms vs 0.65-0.66 unstaggered, 0.77-0.80 for r04's
// kernel; 125k: 0.095 vs 0.099 / 0.122)
using GlProduct = GlShape<3, 8, 8, 2, 0, false, true>;

// colmax[j] = max_i |x[i, j]| as float bits (atomicMax on the bits of a
// non-negative float orders like the float); a NaN bound wins (non-finite x
// then reaches G through mmb_gram_i8).
__global__ void colmax_kernel(const float* __restrict__ x, int64_t N, int D, int64_t rows_per_block,
                              unsigned* __restrict__ colmax) {
  const int64_t r0 = blockIdx.x * rows_per_block;
  const int64_t r1 = min(N, r0 + rows_per_block);
  for (int j = threadIdx.x; j < D; j += blockDim.x) {
    unsigned m = 0u;  // bits of max |x|: NaN (0x7fc00000..) ranks above inf, so it propagates
    for (int64_t r = r0; r < r1; ++r) m = max(m, __float_as_uint(fabsf(x[r * D + j])));
    if (m > 0u) atomicMax(colmax + j, m);
  }
}

// Fixed-order sum of the R range partials of every upper-triangle tile
// element (consecutive threads read consecutive partial elements: coalesced;
// the former element-of-G order read the lower half transposed, 8x the bytes),
// written to G[p][q] and mirrored to G[q][p] for off-diagonal tiles (diagonal
// tiles hold both halves themselves).  Same sums in the same order as before.
// r03: 8 threads per element (thread group u sums the ranges r = u (mod 8) in
// increasing r, all of its <= 16 loads in flight at once; the 8 sums are
// combined in LDS) -- the same eight partial sums and the same combine order
// as the one-thread-per-element kernel, so G is bit-identical, but 8x the
// loads in flight: the reduction of 128 ranges (49.8 MB of partials at
// D = 300) was latency-bound at ~57 us.
constexpr int kRedEl = 32;      // elements per block
constexpr int kRedMaxPer = 16;  // ranges per thread (R <= 128)
__global__ __launch_bounds__(256) void gram_tri_reduce_kernel(const double* __restrict__ part, int D,
                                                              int nt, int R, int accumulate,
                                                              double* __restrict__ g) {
  __shared__ double s_p[8][kRedEl];
  const int T = nt * (nt + 1) / 2;
  const int64_t total = static_cast<int64_t>(T) * 256;
  const int el = threadIdx.x % kRedEl, u = threadIdx.x / kRedEl;
  const int64_t e = static_cast<int64_t>(blockIdx.x) * kRedEl + el;
  double s = 0.0;
  if (e < total) {
    if (R >= 8) {  // thread group u sums ranges u, u + 8, .. (< R)
      double v[kRedMaxPer];
      const int per = (R + 7) / 8;
#pragma unroll
      for (int j = 0; j < kRedMaxPer; ++j)
        v[j] = (j < per && u + 8 * j < R) ? part[static_cast<int64_t>(u + 8 * j) * total + e] : 0.0;
#pragma unroll
      for (int j = 0; j < kRedMaxPer; ++j)
        if (j < per && u + 8 * j < R) s += v[j];
    } else if (u == 0) {
      for (int r = 0; r < R; ++r) s += part[static_cast<int64_t>(r) * total + e];
    }
  }
  s_p[u][el] = s;
  __syncthreads();
  if (u != 0 || e >= total) return;
  const int tau = static_cast<int>(e >> 8), w = static_cast<int>(e & 255);
  int bi, bj;
  tri_tile(tau, nt, bi, bj);
  const int p = 16 * bi + (w >> 4), q = 16 * bj + (w & 15);
  if (p >= D || q >= D) return;
  const double sum = ((s_p[0][el] + s_p[1][el]) + (s_p[2][el] + s_p[3][el])) +
                     ((s_p[4][el] + s_p[5][el]) + (s_p[6][el] + s_p[7][el]));
  const int64_t e1 = static_cast<int64_t>(p) * D + q;
  g[e1] = accumulate ? g[e1] + sum : sum;
  if (bi != bj) {
    const int64_t e2 = static_cast<int64_t>(q) * D + p;
    g[e2] = accumulate ? g[e2] + sum : sum;
  }
}

static int launch_tri_reduce(const double* part, int d, int nt, int R, int accumulate, double* g,
                             hipStream_t stream) {
  // the kernel sums ranges u + 8 j < R (at most kRedMaxPer per thread) for
  // R >= 8: a plan outside that would silently drop ranges
  MMB_REQUIRE(R >= 1 && R <= 8 * kRedMaxPer);
  const int64_t total = static_cast<int64_t>(nt) * (nt + 1) / 2 * 256;
  gram_tri_reduce_kernel<<<static_cast<int>(ceil_div(total, kRedEl)), 256, 0, stream>>>(
      part, d, nt, R, accumulate, g);
  return MMB_OK;
}

// Fixed-order sum over the S row chunks (deterministic), mirrored to both halves.
__global__ void gram_reduce_kernel(const double* __restrict__ part, int D, int nb, int npairs,
                                   int S, int accumulate, double* __restrict__ g) {
  const int64_t total = static_cast<int64_t>(D) * D;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int p = static_cast<int>(e / D), q = static_cast<int>(e % D);
    int bp = p / kGB, bq = q / kGB, i = p % kGB, j = q % kGB;
    if (bp > bq) {
      int t = bp; bp = bq; bq = t;
      t = i; i = j; j = t;
    }
    const int pair = gram_pair_index(bp, bq, nb);
    double sum = 0.0;
    for (int s = 0; s < S; ++s) sum += part[(static_cast<int64_t>(s) * npairs + pair) * (kGB * kGB) + i * kGB + j];
    g[e] = accumulate ? g[e] + sum : sum;
  }
}

template <typename TX>
__global__ void xt_omega_kernel(const TX* __restrict__ num, const float* __restrict__ cnt,
                                int64_t N, int D, const double* __restrict__ om, int k,
                                double* __restrict__ z0) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= D * k) return;
  const int p = e / k, j = e % k;
  double acc = 0.0;
  for (int64_t n = 0; n < N; ++n) acc += static_cast<double>(load_x(num, cnt, n, p, D)) * om[n * k + j];
  z0[e] = acc;
}

// X^T Omega for the transposed branch's small splits (N < d rows, k <= 16):
// one wave per feature p, lane l summing rows l, l + 64, ... for all k
// columns (every load of a lane independent), then a fixed-order DPP wave sum
// per column.  The thread-per-output kernel above walked all N rows as one
// dependent chain of loads: 59 us for a 229-row split (r04 dataset_splits).
// X^T Omega for the transposed branch's small splits (N < d rows, k <= 16)
// on the f64 matrix pipe: workgroup `blk` owns the 16-feature tile blk of z0
// (all k <= 16 columns: one 16x16 output tile), its 4 waves split the N / 4
// MFMA k-steps (v_mfma_f64_16x16x4f64, A = X^T rows, B = Omega rows; every
// k-step's operands loaded before the first MFMA) and their sums are added in
// wave order.  (r05's wave per feature read 64 rows per load instruction and
// chained its iterations: 5 / 11 us at 100 / 203 rows, r06 kernel trace; a
// lane-per-feature loop over the rows with Omega in LDS measured 31 us.)
constexpr int kXtK = 16;
constexpr int kXtMaxN = 320;  // rows (the branch has N < d <= 320)
template <typename TX, bool CNT>
__device__ __forceinline__ void xt_omega_wave_body(const TX* __restrict__ num, const float* __restrict__ cnt,
                                                   int64_t N, int D, const double* __restrict__ om, int k,
                                                   double* __restrict__ z0, int blk) {
  __shared__ double s_part[4][256];
  constexpr int kS = (kXtMaxN / 4 + 3) / 4;  // k-steps per wave (20)
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int n_ = static_cast<int>(N);
  const int p = blk * 16 + (lane & 15), j = lane & 15;
  double xa[kS], ob[kS];
#pragma unroll
  for (int u = 0; u < kS; ++u) {
    const int n = 4 * (wave + 4 * u) + (lane >> 4);
    const bool ok = n < n_;
    xa[u] = (ok && p < D) ? static_cast<double>(CNT ? load_x(num, cnt, n, p, D)
                                                    : num[static_cast<int64_t>(n) * D + p])
                          : 0.0;
    ob[u] = (ok && j < k) ? om[static_cast<int64_t>(n) * k + j] : 0.0;
  }
  f64x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < kS; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[u], ob[u], acc, 0, 0, 0);
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) s_part[wave][((lane >> 4) + 4 * reg) * 16 + (lane & 15)] = acc[reg];
  __syncthreads();
  const int e = threadIdx.x;
  if (e < 256) {
    const double v = s_part[0][e] + s_part[1][e] + s_part[2][e] + s_part[3][e];
    const int pr = blk * 16 + (e >> 4), jc = e & 15;
    if (pr < D && jc < k) z0[pr * k + jc] = v;
  }
}
template <typename TX, bool CNT = false>
__global__ __launch_bounds__(256) void xt_omega_wave_kernel(const TX* __restrict__ num,
                                                            const float* __restrict__ cnt,
                                                            int64_t N, int D,
                                                            const double* __restrict__ om, int k,
                                                            double* __restrict__ z0) {
  xt_omega_wave_body<TX, CNT>(num, cnt, N, D, om, k, z0, blockIdx.x);
}

// ------------------------------------------------------------------ pc_solve
#ifdef MMB_PC_PROBE  // phase timestamps for tools/pc_probe.hip (never in libmmb)
__device__ unsigned long long g_pc_probe[64];
// The marks go to LDS and are copied out at the end of the kernel
// (PC_PROBE_FLUSH): a global store per mark put its completion wait into the
// next barrier's phase (r05: ~4 us of a round's update phase was the mark).
__device__ __forceinline__ unsigned long long* pc_probe_lds() {
  __shared__ unsigned long long s[64];
  return s;
}
#define PC_MARK(i)                                                               \
  do {                                                                           \
    __syncthreads();                                                             \
    if (threadIdx.x == 0 && blockIdx.x == 0) pc_probe_lds()[i] = wall_clock64(); \
  } while (0)
// one wave's own mark (no barrier): lane 0 of the calling wave, workgroup 0
#define PC_WMARK(i)                                                                     \
  do {                                                                                  \
    if ((threadIdx.x & 63) == 0 && blockIdx.x == 0) pc_probe_lds()[i] = wall_clock64(); \
  } while (0)
#define PC_PROBE_FLUSH()                                                                    \
  do {                                                                                      \
    __syncthreads();                                                                        \
    if (blockIdx.x == 0 && threadIdx.x < 64) g_pc_probe[threadIdx.x] = pc_probe_lds()[threadIdx.x]; \
  } while (0)
#else
#define PC_MARK(i) \
  do {             \
  } while (0)
#define PC_WMARK(i) \
  do {              \
  } while (0)
#define PC_PROBE_FLUSH() \
  do {                   \
  } while (0)
#endif
constexpr int kMaxD = 512;
constexpr int kMaxK = 16;
constexpr int kSolveNT = 1024;

// Modified Gram-Schmidt, twice ("twice is enough"), on the columns of Z [D][k]
// by one wave.  Lane l owns rows p = l (mod 64), so LDS needs no cross-lane
// ordering; dot products travel through shuffles.
__device__ void orth_wave(double* Z, int D, int k, int lane) {
  for (int j = 0; j < k; ++j) {
    for (int pass = 0; pass < 2; ++pass) {
      for (int i = 0; i < j; ++i) {
        double d = 0.0;
        for (int p = lane; p < D; p += kWave) d += Z[p * k + i] * Z[p * k + j];
        d = wave_sum(d);
        for (int p = lane; p < D; p += kWave) Z[p * k + j] -= d * Z[p * k + i];
      }
    }
    double nn = 0.0;
    for (int p = lane; p < D; p += kWave) nn += Z[p * k + j] * Z[p * k + j];
    nn = wave_sum(nn);
    const double inv = 1.0 / sqrt(nn);
    for (int p = lane; p < D; p += kWave) Z[p * k + j] *= inv;
  }
}

// GZ = G Z.  Thread (g, p) owns row p and column group g (MC columns), so
// every thread of the workgroup works (D=300: 3 groups of 4 of the 11
// columns).  G symmetric: read column p (coalesced across p; the groups
// re-read it from L1).  Z is read from LDS as a broadcast.
template <int MC>
__device__ void gz_product_mc(const double* __restrict__ G, const double* Z, double* GZ, int D,
                              int k, int groups) {
  const int t = threadIdx.x;
  const int g = t / D, p = t - g * D;
  if (g >= groups) return;
  const int j0 = g * MC;
  double acc[MC];
#pragma unroll
  for (int j = 0; j < MC; ++j) acc[j] = 0.0;
  const double* gcol = G + p;
  const double* zr = Z + j0;
#pragma unroll 16
  for (int q = 0; q < D; ++q) {
    const double gq = gcol[static_cast<int64_t>(q) * D];
#pragma unroll
    for (int j = 0; j < MC; ++j)
      if (j0 + j < k) acc[j] = fma(gq, zr[q * k + j], acc[j]);
  }
#pragma unroll
  for (int j = 0; j < MC; ++j)
    if (j0 + j < k) GZ[p * k + j0 + j] = acc[j];
}

__device__ void gz_product(const double* __restrict__ G, const double* Z, double* GZ, int D, int k) {
  const int maxg = kSolveNT / D;  // >= 2 for D <= 512
  if (maxg >= 3 && k <= 12) {
    gz_product_mc<4>(G, Z, GZ, D, k, (k + 3) / 4);
  } else {
    gz_product_mc<8>(G, Z, GZ, D, k, (k + 7) / 8);
  }
}

// M[i][j] = sum_p X[p][i] Y[p][j] for the k x k block, all waves.
__device__ void small_gram(const double* X, const double* Y, double* M, int D, int k) {
  const int wave = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  for (int e = wave; e < k * k; e += kSolveNT / kWave) {
    const int i = e / k, j = e % k;
    double d = 0.0;
    for (int p = lane; p < D; p += kWave) d += X[p * k + i] * Y[p * k + j];
    d = wave_sum(d);
    if (lane == 0) M[e] = d;
  }
}

// Cyclic Jacobi on symmetric A [k][k] (LDS) by one wave; V <- eigenvectors (columns).
__device__ void jacobi_wave(double* A, double* V, int k, int lane) {
  for (int r = lane; r < k * k; r += kWave) V[r] = (r / k == r % k) ? 1.0 : 0.0;
  wave_lds_sync();
  for (int sweep = 0; sweep < 40; ++sweep) {
    double off = 0.0, dia = 0.0;
    for (int r = lane; r < k * k; r += kWave) {
      const int i = r / k, j = r % k;
      const double a = A[r];
      if (i < j) off += a * a;
      else if (i == j) dia += a * a;
    }
    off = wave_sum(off);
    dia = wave_sum(dia);
    // converged when the off-diagonal mass is ~1e-14 of the diagonal's: the
    // rotations' own rounding (~1e-16 |lambda_max|) keeps regenerating
    // off-diagonal entries, so a bar at the rounding level itself is never met
    if (off <= 1e-28 * dia) break;
    bool rotated = false;
    for (int p = 0; p < k - 1; ++p) {
      for (int q = p + 1; q < k; ++q) {
        const double apq = A[p * k + q];
        const double app = A[p * k + p], aqq = A[q * k + q];
        // at rounding level next to both diagonal entries: rotating changes nothing
        if (fabs(apq) <= 2e-16 * (fabs(app) + fabs(aqq))) continue;
        rotated = true;
        const double theta = (aqq - app) / (2.0 * apq);
        double t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
        if (theta < 0.0) t = -t;
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        double arp = 0.0, arq = 0.0, vrp = 0.0, vrq = 0.0;
        if (lane < k) {
          arp = A[lane * k + p];
          arq = A[lane * k + q];
          vrp = V[lane * k + p];
          vrq = V[lane * k + q];
        }
        wave_lds_sync();
        if (lane < k) {
          if (lane != p && lane != q) {
            const double np_ = c * arp - s * arq, nq = s * arp + c * arq;
            A[lane * k + p] = np_;
            A[p * k + lane] = np_;
            A[lane * k + q] = nq;
            A[q * k + lane] = nq;
          }
          V[lane * k + p] = c * vrp - s * vrq;
          V[lane * k + q] = s * vrp + c * vrq;
        }
        if (lane == 0) {
          A[p * k + p] = app - t * apq;
          A[q * k + q] = aqq + t * apq;
          A[p * k + q] = 0.0;
          A[q * k + p] = 0.0;
        }
        wave_lds_sync();
      }
    }
    if (!rotated) break;
  }
}

// Orthonormalise the columns of Z [D][k] with the whole workgroup:
// column equilibration, then CholeskyQR twice (W = Z^T Z by all waves,
// Cholesky + triangular inverse by one wave, Z <- Z L^{-T} row-parallel).
// Falls back to wave-0 MGS^2 if a Cholesky pivot is not positive (only for
// extreme ill-conditioning, kappa >~ 1e8).
__device__ void orth_block(double* Z, int D, int k, double* sW, double* sL, double* sLi,
                           int* s_fail) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  for (int pass = 0; pass < 3; ++pass) {
    small_gram(Z, Z, sW, D, k);
    if (tid == 0) *s_fail = 0;
    __syncthreads();
    if (pass == 0) {  // equilibrate: unit column norms
      if (tid < D) {
        for (int j = 0; j < k; ++j) Z[tid * k + j] *= 1.0 / sqrt(sW[j * k + j]);
      }
      __syncthreads();
      continue;
    }
    if (wave == 0) {
      for (int e = lane; e < k * k; e += kWave) sL[e] = 0.0;
      wave_lds_sync();
      for (int j = 0; j < k; ++j) {
        if (lane == 0) {
          double s = sW[j * k + j];
          for (int m = 0; m < j; ++m) s -= sL[j * k + m] * sL[j * k + m];
          if (!(s > 0.0)) *s_fail = 1;
          sL[j * k + j] = sqrt(s > 0.0 ? s : 1.0);
        }
        wave_lds_sync();
        if (lane > j && lane < k) {
          double s = sW[lane * k + j];
          for (int m = 0; m < j; ++m) s -= sL[lane * k + m] * sL[j * k + m];
          sL[lane * k + j] = s / sL[j * k + j];
        }
        wave_lds_sync();
      }
      if (lane < k) {  // Linv column `lane`
        const int c = lane;
        for (int i = 0; i < k; ++i) {
          double s = (i == c) ? 1.0 : 0.0;
          for (int m = c; m < i; ++m) s -= sL[i * k + m] * sLi[m * k + c];
          sLi[i * k + c] = (i < c) ? 0.0 : s / sL[i * k + i];
        }
      }
    }
    __syncthreads();
    if (*s_fail) {
      if (wave == 0) orth_wave(Z, D, k, lane);
      __syncthreads();
      return;
    }
    if (tid < D) {  // row p: z <- z L^{-T}, i.e. z_new[j] = sum_{m<=j} z[m] Linv[j][m]
      double z[kMaxK];
#pragma unroll
      for (int m = 0; m < kMaxK; ++m) z[m] = (m < k) ? Z[tid * k + m] : 0.0;
      for (int j = 0; j < k; ++j) {
        double s = 0.0;
#pragma unroll
        for (int m = 0; m < kMaxK; ++m)
          if (m <= j) s += z[m] * sLi[j * k + m];
        Z[tid * k + j] = s;
      }
    }
    __syncthreads();
  }
}

__device__ void symmetrize(double* M, int k) {
  for (int e = threadIdx.x; e < k * k; e += blockDim.x) {
    const int i = e / k, j = e % k;
    if (i < j) {
      const double m = 0.5 * (M[i * k + j] + M[j * k + i]);
      M[i * k + j] = m;
      M[j * k + i] = m;
    }
  }
}

__global__ __launch_bounds__(kSolveNT) void pc_solve_kernel(const double* __restrict__ G, int D,
                                                            const double* __restrict__ z0, int k,
                                                            int npc, int n_iter, int transposed,
                                                            double* __restrict__ pc_out) {
  __shared__ double sZ[kMaxD * kMaxK];
  __shared__ double sGZ[kMaxD * kMaxK];
  __shared__ double sA[kMaxK * kMaxK], sV[kMaxK * kMaxK], sW[kMaxK * kMaxK];
  __shared__ double sL[kMaxK * kMaxK], sLi[kMaxK * kMaxK], sT[kMaxK * kMaxK];
  __shared__ double sy[kMaxK], sv[kMaxD];
  __shared__ double s_rd[kSolveNT / kWave];
  __shared__ double s_rv[kSolveNT / kWave];
  __shared__ int s_ri[kSolveNT / kWave];
  __shared__ int s_order[kMaxK];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;

  __shared__ int s_fail;
  PC_MARK(0);
  for (int e = tid; e < D * k; e += kSolveNT) sZ[e] = z0[e];
  __syncthreads();
  orth_block(sZ, D, k, sW, sL, sLi, &s_fail);
  PC_MARK(1);
  for (int it = 0; it < n_iter; ++it) {
    gz_product(G, sZ, sGZ, D, k);
    __syncthreads();
    PC_MARK(2 + 2 * it);
    for (int e = tid; e < D * k; e += kSolveNT) sZ[e] = sGZ[e];
    __syncthreads();
    orth_block(sZ, D, k, sW, sL, sLi, &s_fail);
    PC_MARK(3 + 2 * it);
  }
  gz_product(G, sZ, sGZ, D, k);
  __syncthreads();
  PC_MARK(40);

  if (transposed) {
    small_gram(sZ, sGZ, sA, D, k);  // Q^T G Q
    __syncthreads();
    symmetrize(sA, k);
    __syncthreads();
  } else {
    small_gram(sZ, sGZ, sW, D, k);   // W = Z^T G Z
    small_gram(sGZ, sGZ, sT, D, k);  // H = (GZ)^T (GZ)
    __syncthreads();
    symmetrize(sW, k);
    symmetrize(sT, k);
    __syncthreads();
    if (wave == 0) {
      // Cholesky W = L L^T
      for (int e = lane; e < k * k; e += kWave) sL[e] = 0.0;
      wave_lds_sync();
      for (int j = 0; j < k; ++j) {
        if (lane == 0) {
          double s = sW[j * k + j];
          for (int m = 0; m < j; ++m) s -= sL[j * k + m] * sL[j * k + m];
          sL[j * k + j] = sqrt(s);
        }
        wave_lds_sync();
        if (lane > j && lane < k) {
          double s = sW[lane * k + j];
          for (int m = 0; m < j; ++m) s -= sL[lane * k + m] * sL[j * k + m];
          sL[lane * k + j] = s / sL[j * k + j];
        }
        wave_lds_sync();
      }
      // Linv: lane c solves L x = e_c (column c)
      if (lane < k) {
        const int c = lane;
        for (int i = 0; i < k; ++i) {
          double s = (i == c) ? 1.0 : 0.0;
          for (int m = c; m < i; ++m) s -= sL[i * k + m] * sLi[m * k + c];
          sLi[i * k + c] = (i < c) ? 0.0 : s / sL[i * k + i];
        }
      }
      wave_lds_sync();
      // A = Linv H Linv^T
      for (int e = lane; e < k * k; e += kWave) {
        const int i = e / k, j = e % k;
        double s = 0.0;
        for (int m = 0; m < k; ++m) s += sLi[i * k + m] * sT[m * k + j];
        sV[e] = s;  // scratch: Linv H
      }
      wave_lds_sync();
      for (int e = lane; e < k * k; e += kWave) {
        const int i = e / k, j = e % k;
        double s = 0.0;
        for (int m = 0; m < k; ++m) s += sV[i * k + m] * sLi[j * k + m];
        sA[e] = s;
      }
      wave_lds_sync();
      for (int e = lane; e < k * k; e += kWave) {
        const int i = e / k, j = e % k;
        if (i < j) {
          const double m = 0.5 * (sA[i * k + j] + sA[j * k + i]);
          sA[i * k + j] = m;
          sA[j * k + i] = m;
        }
      }
      wave_lds_sync();
    }
    __syncthreads();
  }

  PC_MARK(41);
  if (wave == 0) {
    jacobi_wave(sA, sV, k, lane);
    if (lane == 0) {  // eigenvalues descending (selection; first max wins ties)
      bool used[kMaxK];
      for (int j = 0; j < k; ++j) used[j] = false;
      for (int c = 0; c < k; ++c) {
        int best = -1;
        for (int j = 0; j < k; ++j)
          if (!used[j] && (best < 0 || sA[j * k + j] > sA[best * k + best])) best = j;
        used[best] = true;
        s_order[c] = best;
      }
    }
  }
  __syncthreads();
  PC_MARK(42);

  for (int c = 0; c < npc; ++c) {
    const int col = s_order[c];
    if (!transposed) {
      if (tid < k) {  // y = Linv^T u
        double s = 0.0;
        for (int m = 0; m < k; ++m) s += sLi[m * k + tid] * sV[m * k + col];
        sy[tid] = s;
      }
      __syncthreads();
    }
    double v = 0.0;
    if (tid < D) {
      if (transposed) {
        for (int j = 0; j < k; ++j) v += sZ[tid * k + j] * sV[j * k + col];
      } else {
        for (int j = 0; j < k; ++j) v += sGZ[tid * k + j] * sy[j];
      }
      sv[tid] = v;
    }
    // norm and first argmax |v|
    double nn = wave_sum(v * v);
    double best = (tid < D) ? fabs(v) : -1.0;
    int bidx = (tid < D) ? tid : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double ob = __shfl_xor(best, o, kWave);
      const int oi = __shfl_xor(bidx, o, kWave);
      if (ob > best || (ob == best && oi < bidx)) {
        best = ob;
        bidx = oi;
      }
    }
    if (lane == 0) {
      s_rd[wave] = nn;
      s_rv[wave] = best;
      s_ri[wave] = bidx;
    }
    __syncthreads();
    double tot = 0.0, bb = -1.0;
    int bi = 0x7fffffff;
    for (int w = 0; w < kSolveNT / kWave; ++w) {
      tot += s_rd[w];
      if (s_rv[w] > bb || (s_rv[w] == bb && s_ri[w] < bi)) {
        bb = s_rv[w];
        bi = s_ri[w];
      }
    }
    const double scale = (sv[bi] < 0.0 ? -1.0 : 1.0) / sqrt(tot);
    if (tid < D) pc_out[c * D + tid] = v * scale;
    __syncthreads();
  }
  PC_MARK(43);
}

// ------------------------------------------------------------------ pc_solve (D <= 320)
// The same solve with every D-long contraction on the fp64 matrix pipe
// (MFMA 16x16x4): the block is kept 16 columns wide in LDS (columns >= k and
// rows >= D zero), so
//   G Z      = 16-row tiles of G (A operand, read straight from L2: G is
//              symmetric, so a fragment is 16 consecutive doubles of 4 rows)
//              times Z (B operand from LDS);
//   X^T Y    = one 16x16 MFMA accumulator per wave over a quarter-strided
//              share of the rows, the 16 partials summed in a fixed order.
// Everything k x k (Cholesky, triangular inverse, Jacobi) stays on one wave.
constexpr int kP16MaxD = 320;
// 16 waves.  (8 waves with a software-pipelined G.Z product -- two 16-deep
// batches of G per lane in flight, which 128 VGPRs cannot hold -- measured
// slower: 0.340 vs 0.310 ms per solve; the products are not what bounds it.)
constexpr int kP16NT = 1024;
constexpr int kP16W = 16;  // block width (k <= 16)

struct P16Lds {
  double* Z;     // [Dp][16]
  double* GZ;    // [Dp][16]
  double* part;  // [16 waves][256]
};

// M (k x k, compact) = X^T Y over the Dp rows of two [Dp][16] blocks (NW
// waves: every thread of the workgroup).
template <int NW = kP16NT / kWave>
__device__ __forceinline__ void p16_gram(const double* X, const double* Y, int Dp, int k, double* part, double* M) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  f64x4 acc = {0, 0, 0, 0};
  for (int p = 4 * wave; p < Dp; p += 4 * NW) {
    const int o = (p + (lane >> 4)) * kP16W + (lane & 15);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(X[o], Y[o], acc, 0, 0, 0);
  }
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) part[wave * 256 + ((lane >> 4) + 4 * reg) * 16 + (lane & 15)] = acc[reg];
  __syncthreads();
  if (tid < 256) {
    const int i = tid >> 4, j = tid & 15;
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += part[w * 256 + tid];
    if (i < k && j < k) M[i * k + j] = s;
  }
  __syncthreads();
}

// M1 = X1^T Y1 and M2 = X2^T Y2 (k x k, compact) in one pass over the Dp rows
// (the two sums as p16_gram's, one barrier pair instead of two).
template <int NW>
__device__ __forceinline__ void p16_gram2(const double* X1, const double* Y1, double* M1, const double* X2,
                                          const double* Y2, double* M2, int Dp, int k, double* part) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  f64x4 a1 = {0, 0, 0, 0}, a2 = {0, 0, 0, 0};
  for (int p = 4 * wave; p < Dp; p += 4 * NW) {
    const int o = (p + (lane >> 4)) * kP16W + (lane & 15);
    a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(X1[o], Y1[o], a1, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(X2[o], Y2[o], a2, 0, 0, 0);
  }
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) {
    part[wave * 256 + ((lane >> 4) + 4 * reg) * 16 + (lane & 15)] = a1[reg];
    part[(NW + wave) * 256 + ((lane >> 4) + 4 * reg) * 16 + (lane & 15)] = a2[reg];
  }
  __syncthreads();
  if (tid < 512) {
    const int e = tid & 255, i = e >> 4, j = e & 15, h = tid >> 8;
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += part[(h * NW + w) * 256 + e];
    if (i < k && j < k) (h ? M2 : M1)[i * k + j] = s;
  }
  __syncthreads();
}

// GZ = G Z (G symmetric [D][D] in global memory / L2).  16 k-steps of loads
// are issued before their MFMAs (one L2 latency per batch, not per step);
// two accumulators alternate so consecutive MFMAs are independent.  (32-step
// batches measured slower on MI355X: 24.3 vs 19.5 us per product.)  The p16
// helpers are force-inlined: as called functions they were compiled with
// flat loads and spilled their operands to scratch around every call
// (pc_solve 0.316 -> 0.310 ms).
constexpr int kGzBatch = 16;
__device__ __forceinline__ void p16_gz(const double* __restrict__ G, int D, int Dp, const double* Z, double* GZ) {
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int mt = Dp / 16;
  const int nbat = (Dp + 4 * kGzBatch - 1) / (4 * kGzBatch);
  for (int t = wave; t < mt; t += kP16NT / kWave) {
    const int p = t * 16 + (lane & 15);
    const int pc = min(p, D - 1);
    f64x4 acc0 = {0, 0, 0, 0}, acc1 = acc0;
    // clamped addresses, unconditional loads, selected after (keeps loads in
    // flight; a batch index past the last re-reads it, an L2 hit)
    auto load = [&](int bt, double (&g)[kGzBatch]) {
      const int q0 = 4 * kGzBatch * min(bt, nbat - 1);
#pragma unroll
      for (int s = 0; s < kGzBatch; ++s) {
        const int q = q0 + 4 * s + (lane >> 4);
        g[s] = G[static_cast<int64_t>(min(q, D - 1)) * D + pc];
      }
    };
    auto comp = [&](int bt, const double (&g)[kGzBatch]) {
      const int q0 = 4 * kGzBatch * bt;
#pragma unroll
      for (int s = 0; s < kGzBatch; ++s) {
        const int q = q0 + 4 * s + (lane >> 4);
        const double a = (p < D && q < D) ? g[s] : 0.0;
        const double b = Z[min(q, Dp - 1) * kP16W + (lane & 15)];
        if (s & 1) {
          acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc1, 0, 0, 0);
        } else {
          acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
        }
      }
    };
    double g0[kGzBatch];
    for (int bt = 0; bt < nbat; ++bt) {
      load(bt, g0);
      comp(bt, g0);
    }
#pragma unroll
    for (int reg = 0; reg < 4; ++reg)
      GZ[(t * 16 + (lane >> 4) + 4 * reg) * kP16W + (lane & 15)] = acc0[reg] + acc1[reg];
  }
}

// 1 / sqrt(x) to f64 precision: the v_rsq_f64 estimate + two Newton steps
// (r03: replaces sqrt + an f64 division per Cholesky pivot)
__device__ __forceinline__ double rsqrt_f64(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  y = y * fma(-h * y, y, 1.5);
  y = y * fma(-h * y, y, 1.5);
  return y;
}

// Cholesky of the k x k SPD matrix whose row `lane` (lane < k) is w[]
// (registers; zero elsewhere) by one wave, pivots inverted once (rsqrt_f64).
// Writes L^{-1} (compact, sLi) and returns, in x[], lane c's column of
// L^{-1}; L itself goes to sL column by column (sL[j * 16 + i], internal).
// *fail is set if a pivot is not positive (the pivot is then replaced by 1).
//
// r06b: both loops run over the pivots at run time -- one copy of a step,
// where r05 unrolled all 16 (~6 KB of code per instance, five instances in
// the multi-workgroup solve: after other kernels the solve's first pass
// through each missed in the instruction cache, +16 us over a warm solve,
// tools/pc_probe "cold").  Lane i keeps row i of the trailing matrix
// SHIFTED, so pivot j is always w[0]: d_jj = lane j's w[0], l_ij = w[0] /
// sqrt(d_jj), and w[m - 1] <- w[m] - l_ij l_(j+m)j (a readlane of lane j + m).  The substitution is right-looking in the same
// shifted form: lane c's t = e_c, step i: x_i = t_0 / L_ii to LDS, t_(m-1) <-
// t_m - L_(i+m)i x_i (column i of L as LDS broadcasts).
__device__ __forceinline__ void p16_chol_regs(double (&w)[kMaxK], double* sL, double* sLi, int k,
                                              int lane, int* fail, double (&x)[kMaxK], int mark = 31) {
  double* rl = sLi + kMaxK * kMaxK - kMaxK;  // the reciprocal pivots: sLi's last row until the end
  bool bad = false;
  PC_WMARK(mark);
#pragma unroll 1
  for (int j = 0; j < k; ++j) {
    const double djj = readlane_f64(w[0], j);
    bad = bad || !(djj > 0.0);
    const double p = djj > 0.0 ? djj : 1.0;
    const double r = rsqrt_f64(p);
    const double lij = (lane == j) ? p * r : (lane > j ? w[0] * r : 0.0);
    if (lane < kMaxK) sL[j * kMaxK + lane] = lij;
    if (lane == 0) rl[j] = r;
    // every lane's l_(j+m)j first (lanes past k hold zero rows: l = 0
    // there), then the updates -- no per-column branches, so the broadcasts
    // issue back to back
    double lm[kMaxK];
#pragma unroll
    for (int m = 1; m < kMaxK; ++m) lm[m] = readlane_f64(lij, j + m);
#pragma unroll
    for (int m = 1; m < kMaxK; ++m) w[m - 1] = w[m] - lij * lm[m];
    w[kMaxK - 1] = 0.0;
  }
  if (bad && lane == 0) *fail = 1;
  wave_lds_sync();
  PC_WMARK(mark + 1);
  double t[kMaxK];
#pragma unroll
  for (int m = 0; m < kMaxK; ++m) t[m] = (m == lane) ? 1.0 : 0.0;
  // in order within the wave: step i reads rl[i] before any lane's store of
  // row i can reach it (k = 16: row 15 is rl's storage)
#pragma unroll 1
  for (int i = 0; i < k; ++i) {
    // column i of L below the diagonal (rows past 15 clamped: they only
    // reach t's rows past k, which never become t[0] before the loop ends)
    double li[kMaxK];
#pragma unroll
    for (int m = 1; m < kMaxK; ++m) li[m] = sL[i * kMaxK + min(i + m, kMaxK - 1)];
    const double xi = t[0] * rl[i];
    if (lane < k) sLi[i * k + lane] = (i < lane) ? 0.0 : xi;
#pragma unroll
    for (int m = 1; m < kMaxK; ++m) t[m - 1] = t[m] - li[m] * xi;
    t[kMaxK - 1] = 0.0;
  }
  PC_WMARK(mark + 2);
  wave_lds_sync();
#pragma unroll
  for (int i = 0; i < kMaxK; ++i) x[i] = (i < k && lane < k) ? sLi[i * k + lane] : 0.0;
}

// Cholesky W = L L^T (k x k, compact, LDS) and Linv = L^{-1} by one wave.
__device__ __forceinline__ void p16_chol(const double* sW, double* sL, double* sLi, int k, int lane, int* fail) {
  double w[kMaxK], x[kMaxK];
#pragma unroll
  for (int m = 0; m < kMaxK; ++m) w[m] = (lane < k && m < k) ? sW[lane * k + m] : 0.0;
  p16_chol_regs(w, sL, sLi, k, lane, fail, x);
}

// Top eigenvector of the symmetric positive semi-definite A (k x k, compact,
// LDS) by one wave: B = A (16 x 16, zero padded) is squared 32 times on the
// fp64 matrix pipe, B <- B B / trace(B B), so B -> v v^T along the top
// eigenvector (any ratio lambda_2 / lambda_1 < 1 - 1e-9 is resolved); the
// f64 16x16 accumulator layout (row (l>>4) + 4 r, column l&15) IS the operand
// layout of the next squaring (B symmetric), so B never leaves the
// registers.  v = the column of B with the largest diagonal, normalised, then
// two Rayleigh steps on A.  Returns lambda = v^T A v; u[0..k) = v.
__device__ double p16_top_eig(const double* A, int k, int lane, double* u) {
  const int c = lane & 15, r0 = lane >> 4;
  f64x4 b;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = r0 + 4 * r;
    b[r] = (row < k && c < k) ? A[row * k + c] : 0.0;
  }
  for (int it = 0; it < 32; ++it) {
    f64x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(b[s], b[s], acc, 0, 0, 0);
    double tr = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r0 + 4 * r == c) tr += acc[r];
    tr = wave_sum_dpp(tr);
    const double inv = tr > 0.0 ? 1.0 / tr : 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) b[r] = acc[r] * inv;
    // from the second squaring on trace(B) = 1, and trace(B B) = 1 exactly
    // when B is rank one: B is then v v^T to rounding and more squarings
    // change nothing (r03: 32 -> ~5 squarings on separated spectra, ~8 us)
    if (it >= 1 && tr >= 1.0 - 1e-14) break;
  }
  // column with the largest diagonal entry (first index on ties)
  double dg = -1.0;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (r0 + 4 * r == c && c < k) dg = b[r];
  int jb = c;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double od = __shfl_xor(dg, o, kWave);
    const int oj = __shfl_xor(jb, o, kWave);
    if (od > dg || (od == dg && oj < jb)) {
      dg = od;
      jb = oj;
    }
  }
  if (c == jb) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r0 + 4 * r < k) u[r0 + 4 * r] = b[r];
  }
  wave_lds_sync();
  double lam = 0.0;
  for (int step = 0; step < 3; ++step) {
    // lane i < k: y_i = (A u)_i; normalise
    double y = 0.0;
    if (lane < k) {
      for (int m = 0; m < k; ++m) y += A[lane * k + m] * u[m];
    }
    const double ui = lane < k ? u[lane] : 0.0;
    const double nrm2 = wave_sum_dpp(lane < k ? ui * ui : 0.0);
    lam = wave_sum_dpp(ui * y) / nrm2;  // Rayleigh quotient of the current u
    if (step == 2) {
      if (lane < k) u[lane] = ui / sqrt(nrm2);
    } else {
      const double yn = sqrt(wave_sum_dpp(y * y));
      wave_lds_sync();
      if (lane < k) u[lane] = yn > 0.0 ? y / yn : ui;
    }
    wave_lds_sync();
  }
  return lam;
}

// Orthonormalise the k columns of Z [Dp][16]: equilibration, CholeskyQR twice;
// wave-0 MGS^2 on a compact copy if a pivot fails (extreme ill-conditioning).
// npass = 3: equilibration + CholeskyQR2 (orthonormal to rounding); npass =
// 2: equilibration + one CholeskyQR -- a well-conditioned basis of the same
// span, all the subspace iteration needs between products (the span, not the
// basis, fixes the result: span(Q) = span(G^q Omega)).
__device__ __forceinline__ void p16_orth(double* Z, int D, int Dp, int k, double* part, double* sW, double* sL,
                         double* sLi, int* s_fail, int npass = 3) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  for (int pass = 0; pass < npass; ++pass) {
    p16_gram(Z, Z, Dp, k, part, sW);
    if (pass == 0) {
      if (tid < D) {
        for (int j = 0; j < k; ++j) Z[tid * kP16W + j] *= 1.0 / sqrt(sW[j * k + j]);
      }
      __syncthreads();
      continue;
    }
    if (wave == 0) {
      if (lane == 0) *s_fail = 0;
      wave_lds_sync();
      p16_chol(sW, sL, sLi, k, lane, s_fail);
    }
    __syncthreads();
    if (*s_fail) {
      if (wave == 0) {
        // compact [D][k] copy through the partial buffer (D*k <= 16*256 doubles)
        for (int e = lane; e < D * k; e += kWave) part[e] = Z[(e / k) * kP16W + e % k];
        wave_lds_sync();
        orth_wave(part, D, k, lane);
        for (int e = lane; e < D * k; e += kWave) Z[(e / k) * kP16W + e % k] = part[e];
      }
      __syncthreads();
      return;
    }
    if (tid < D) {  // row p: z <- z L^{-T}
      double z[kP16W];
#pragma unroll
      for (int m = 0; m < kP16W; ++m) z[m] = Z[tid * kP16W + m];
      for (int j = 0; j < k; ++j) {
        double s = 0.0;
#pragma unroll
        for (int m = 0; m < kP16W; ++m)
          if (m <= j) s += z[m] * sLi[j * k + m];
        Z[tid * kP16W + j] = s;
      }
    }
    __syncthreads();
  }
}

// The k x k scratch of the solve's tail (LDS, one set per workgroup).
struct P16Small {
  double *A, *V, *W, *L, *Li, *T, *y, *U;  // [16 x 16] each (y: [16]; U: npc x 16)
  double *rd, *rv;                         // [16 waves]
  int *ri, *fail;
};

// The Rayleigh-Ritz tail of the solve (every thread of a 16-wave workgroup):
// from the final block Z and its product GZ = G Z (both [Dp][16] in LDS) to
// the npc components in pc_out -- sklearn's randomized_svd after its range
// finder: W = Z^T G Z, H = (GZ)^T (GZ), the k x k generalised eigenproblem
// H y = s^2 W y (Cholesky of W, A = L^-1 H L^-T), v = GZ L^-T u, svd_flip
// (extmath.py:537-566); the transposed branch takes A = Q^T G Q, v = Q u.
template <int NW = kP16NT / kWave>
__device__ __forceinline__ void p16_tail(const double* Z, const double* GZ, int D, int Dp, int k,
                                         int npc, int transposed, double* part, const P16Small& sm,
                                         double* __restrict__ pc_out, const double* Hpre = nullptr,
                                         bool wpre = false) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
  if (transposed) {
    p16_gram<NW>(Z, GZ, Dp, k, part, sm.A);  // Q^T G Q
    symmetrize(sm.A, k);
    __syncthreads();
  } else {
    if (!wpre) p16_gram<NW>(Z, GZ, Dp, k, part, sm.W);  // W = Z^T G Z (wpre: the caller's, in sm.W)
    if (Hpre) {                           // H = (GZ)^T (GZ), summed by the caller
      if (threadIdx.x < k * k) sm.T[threadIdx.x] = Hpre[threadIdx.x];
      __syncthreads();
    } else {
      p16_gram<NW>(GZ, GZ, Dp, k, part, sm.T);
    }
    symmetrize(sm.W, k);
    symmetrize(sm.T, k);
    __syncthreads();
    if (wave == 0) {
      p16_chol(sm.W, sm.L, sm.Li, k, lane, sm.fail);  // a failed pivot is clamped (W is SPD here)
      // A = Linv H Linv^T on the matrix pipe (r05; two k^3 LDS loops before):
      // U^T = H Linv^T lands in the accumulator layout that is the B operand
      // of A = Linv U^T (k-step st = U^T's rows 4 st .. 4 st + 3), zero padded
      // past k
      const int r = lane & 15, g = lane >> 4;
      f64x4 ut = {0, 0, 0, 0}, av = {0, 0, 0, 0};
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const int m = 4 * st + g;
        const bool in = r < k && m < k;
        ut = __builtin_amdgcn_mfma_f64_16x16x4f64(in ? sm.T[r * k + m] : 0.0, in ? sm.Li[r * k + m] : 0.0, ut, 0, 0,
                                                  0);
      }
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const int m = 4 * st + g;
        av = __builtin_amdgcn_mfma_f64_16x16x4f64((r < k && m < k) ? sm.Li[r * k + m] : 0.0, ut[st], av, 0, 0, 0);
      }
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int i = g + 4 * reg;
        if (i < k && r < k) sm.A[i * k + r] = av[reg];
      }
      wave_lds_sync();
      for (int e = lane; e < k * k; e += kWave) {
        const int i = e / k, j = e % k;
        if (i < j) {
          const double m = 0.5 * (sm.A[i * k + j] + sm.A[j * k + i]);
          sm.A[i * k + j] = m;
          sm.A[j * k + i] = m;
        }
      }
      wave_lds_sync();
    }
    __syncthreads();
  }
  PC_MARK(41);
  if (wave == 0) {  // top npc eigenvectors of A, largest first (deflation)
    for (int c = 0; c < npc; ++c) {
      double* u = sm.U + c * kMaxK;
      const double lam = p16_top_eig(sm.A, k, lane, u);
      if (c + 1 < npc) {
        for (int e = lane; e < k * k; e += kWave) sm.A[e] -= lam * u[e / k] * u[e % k];
        wave_lds_sync();
      }
    }
  }
  __syncthreads();
  PC_MARK(42);

  for (int c = 0; c < npc; ++c) {
    const double* u = sm.U + c * kMaxK;
    if (!transposed) {
      if (tid < k) {  // y = Linv^T u
        double s = 0.0;
        for (int m = 0; m < k; ++m) s += sm.Li[m * k + tid] * u[m];
        sm.y[tid] = s;
      }
      __syncthreads();
    }
    // v = row tid of Z u (transposed) or GZ y; each thread starts its row at
    // column tid mod k: rows are 128 B apart, so lanes reading one column
    // fell on 2 bank pairs (8-way conflicts)
    double v = 0.0;
    if (tid < D) {
      const double* row = (transposed ? Z : GZ) + tid * kP16W;
      const double* c = transposed ? u : sm.y;
      int j = tid % k;
      for (int q = 0; q < k; ++q) {
        v += row[j] * c[j];
        j = j + 1 == k ? 0 : j + 1;
      }
    }
    // norm and first argmax |v|
    double nn = wave_sum(v * v);
    double best = (tid < D) ? fabs(v) : -1.0;
    int bidx = (tid < D) ? tid : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double ob = __shfl_xor(best, o, kWave);
      const int oi = __shfl_xor(bidx, o, kWave);
      if (ob > best || (ob == best && oi < bidx)) {
        best = ob;
        bidx = oi;
      }
    }
    if (lane == 0) {
      sm.rd[wave] = nn;
      sm.rv[wave] = best;
      sm.ri[wave] = bidx;
    }
    __syncthreads();
    double tot = 0.0, bb = -1.0;
    int bi = 0x7fffffff;
    for (int w = 0; w < NW; ++w) {
      tot += sm.rd[w];
      if (sm.rv[w] > bb || (sm.rv[w] == bb && sm.ri[w] < bi)) {
        bb = sm.rv[w];
        bi = sm.ri[w];
      }
    }
    if (tid == bi) part[0] = v;  // sign of the largest-|.| entry (svd_flip)
    __syncthreads();
    const double vbest = part[0];
    const double scale = (vbest < 0.0 ? -1.0 : 1.0) / sqrt(tot);
    if (tid < D) pc_out[c * D + tid] = v * scale;
    __syncthreads();
  }
  PC_MARK(43);
}

#define P16_SMALL_DECL                                                                      \
  __shared__ double sA[kMaxK * kMaxK], sV[kMaxK * kMaxK], sW[kMaxK * kMaxK];                 \
  __shared__ double sL[kMaxK * kMaxK], sLi[kMaxK * kMaxK], sT[kMaxK * kMaxK];                \
  __shared__ double sy[kMaxK];                                                               \
  __shared__ double s_rd[kP16NT / kWave];                                                    \
  __shared__ double s_rv[kP16NT / kWave];                                                    \
  __shared__ int s_ri[kP16NT / kWave];                                                       \
  __shared__ double sU[kMaxK * kMaxK]; /* eigenvectors of A, largest first */               \
  __shared__ int s_fail;                                                                     \
  const P16Small sm{sA, sV, sW, sL, sLi, sT, sy, sU, s_rd, s_rv, s_ri, &s_fail};

__global__ __launch_bounds__(kP16NT) void pc_solve16_kernel(const double* __restrict__ G, int D,
                                                              const double* __restrict__ z0, int k,
                                                              int npc, int n_iter, int transposed,
                                                              double* __restrict__ pc_out) {
  extern __shared__ __attribute__((aligned(16))) double p16_lds[];
  const int Dp = (D + 15) / 16 * 16;
  double* sZ = p16_lds;
  double* sGZ = sZ + Dp * kP16W;
  double* part = sGZ + Dp * kP16W;  // max(16 x 256, Dp x 16): partials / fallback copy
  P16_SMALL_DECL
  const int tid = threadIdx.x;

  PC_MARK(0);
  for (int e = tid; e < Dp * kP16W; e += kP16NT) {
    const int p = e / kP16W, j = e % kP16W;
    sZ[e] = (p < D && j < k) ? z0[p * k + j] : 0.0;
    sGZ[e] = 0.0;
  }
  __syncthreads();
  // one CholeskyQR pass between products, CholeskyQR2 for the block the
  // final Rayleigh-Ritz step uses (orthonormal to rounding, as before)
  p16_orth(sZ, D, Dp, k, part, sW, sL, sLi, &s_fail, n_iter > 0 ? 2 : 3);
  PC_MARK(1);
  double* Z = sZ;
  double* GZ = sGZ;
  for (int it = 0; it < n_iter; ++it) {
    p16_gz(G, D, Dp, Z, GZ);
    __syncthreads();
    PC_MARK(2 + 2 * it);
    double* t = Z; Z = GZ; GZ = t;  // the product becomes the block
    p16_orth(Z, D, Dp, k, part, sW, sL, sLi, &s_fail, it == n_iter - 1 ? 3 : 2);
    PC_MARK(3 + 2 * it);
  }
  p16_gz(G, D, Dp, Z, GZ);
  __syncthreads();
  PC_MARK(40);
  p16_tail(Z, GZ, D, Dp, k, npc, transposed, part, sm, pc_out);
  PC_PROBE_FLUSH();
}

// ------------------------------------------------------------------ pc_solve, multi-workgroup (r03)
// The same randomized-SVD replay with the D-long products spread over
// T = Dp / 16 workgroups (19 at D = 300), one per 16-row tile of G.  The
// single-workgroup solve spent ~20 us per G Z product (76 dependent MFMA
// k-steps per tile, two rounds of tiles over 16 waves, G re-read from L2)
// and ~16 us per orthonormalisation; here each workgroup keeps its 16 rows of
// G in registers for the whole solve (wave w: k-steps w, w + 16, ..), so a
// product is <= 5 MFMAs per wave plus a 16-way LDS sum, and the
// orthonormalisation needs only the block's k x k Gram, which the tiles
// contribute as partials.  Per power iteration ONE exchange: every workgroup
// publishes its tile Y_t = G_t Z (16 x 16) and P_t = Y_t^T Y_t with
// write-through (sc1) stores, drains them and adds one to an arrival counter
// (agent scope, relaxed); each polls the counter for T (it + 1) arrivals
// (bounded), acquires, and gathers all tiles with sc1 loads (CDNA guide
// Guideline 16, R1).  Then EVERY workgroup runs the identical equilibrated
// CholeskyQR on the identical data (W = sum_t P_t in tile order), so the next
// block Z is the same in all of them with no second exchange.  After the
// n_iter-th block, one more exchange gives the final product, and workgroup 0
// runs the Rayleigh-Ritz tail (p16_tail).  Between products the
// equilibration scales W itself (W' = d W d) instead of recomputing the Gram
// of the scaled block; the block entering the tail still gets CholeskyQR2.
// ws: [2][T][512] doubles of tiles (double-buffered by round parity: a round
// r + 2 write needs every workgroup past round r + 1's wait, hence done
// reading round r), then the arrival counter and the abort word (zero when
// the caller first hands ws over; workgroup 0 returns the counter to zero
// once every workgroup has made its last arrival, so a launch -- eager or a
// graph replay -- leaves ws ready for the next one).
constexpr int kPmMaxT = kP16MaxD / 16;  // tiles (20)

// tools/diag: a test shortens the bounded waits (mmb_diag_pc_wait_iters) and
// names one workgroup that never arrives (mmb_diag_pc_skip_arrival), so the
// count a wait polls for cannot be reached whatever the arrival skew: the
// timeout path runs deterministically
#ifndef MMB_HOOK_PM_WAIT_ITERS
#define MMB_HOOK_PM_WAIT_ITERS (1 << 20)
#endif
#ifndef MMB_HOOK_PM_SKIP_ARRIVAL
#define MMB_HOOK_PM_SKIP_ARRIVAL false
#endif
__device__ __forceinline__ bool pm_wait(unsigned* ctr, unsigned target, unsigned* abort_w,
                                        int32_t* flag) {
  const int iters = MMB_HOOK_PM_WAIT_ITERS;
  for (int it = 0; it < iters; ++it) {
    // the abort word first: a set word (another workgroup gave up, or a
    // workspace handed over dirty) ends the wait even where the count is met
    if (__hip_atomic_load(abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    __builtin_amdgcn_s_sleep(4);
  }
  // ~0.5-1 s without the other workgroups, or an abort seen: give up, release
  // every waiter, and say so in the flag word whichever way the abort came (a
  // launch that found the word already set would otherwise leave only a NaN PC)
  __hip_atomic_store(abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (flag) atomicOr(flag, MMB_FLAG_SYNC_TIMEOUT);
  return false;
}

// An arrival of round r must find the counter in [T r, T (r + 1)): every
// workgroup arrives at round r only after seeing T r arrivals, and no
// workgroup arrives at round r + 1 before all T of round r have.  A count
// outside that range is a counter this launch did not start from zero (a
// workspace handed over dirty): abort like a timeout instead of letting the
// waits pass before the other workgroups' tiles are written.
__device__ __forceinline__ bool pm_arrive(unsigned* ctr, int T, int r, unsigned* abort_w,
                                          int32_t* flag) {
  if (MMB_HOOK_PM_SKIP_ARRIVAL) return true;  // (tools/diag) never arrives
  const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old >= static_cast<unsigned>(T * r) && old < static_cast<unsigned>(T * (r + 1))) return true;
  __hip_atomic_store(abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (flag) atomicOr(flag, MMB_FLAG_SYNC_TIMEOUT);
  return false;
}

// Out [Dp][16] = In [Dp][16] M^T for a 16 x 16 M (row-major, zero past k;
// MT: M holds M^T, whose reads are conflict-free): the 16-row tiles over the
// NW waves, 4 MFMA k-steps each.  In != Out.
template <int NW = kP16NT / kWave, bool MT = false>
__device__ __forceinline__ void p16_rmul(const double* In, const double* M, double* Out, int Dp) {
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  for (int t = wave; t < Dp / 16; t += NW) {
    f64x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const int m = 4 * st + (lane >> 4);
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(In[(t * 16 + (lane & 15)) * kP16W + m],
                                                 MT ? M[m * kP16W + (lane & 15)] : M[(lane & 15) * kP16W + m],
                                                 acc, 0, 0, 0);
    }
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) Out[(t * 16 + (lane >> 4) + 4 * reg) * kP16W + (lane & 15)] = acc[reg];
  }
}

// Wave 0: the equilibrated Cholesky factor of a block's Gram W (k x k
// compact, LDS): d_j = 1 / sqrt(W_jj), d W d = L L^T, and on return
// M = L^-1 diag(d) (16 x 16, zero past k) is the right factor that
// orthonormalises the block: Z = B M^T (one CholeskyQR pass after
// equilibration, from the Gram alone).  d[] = the scales.  All in registers
// (lane i = row i); *fail as p16_chol.  Mt (optional) receives M^T, the
// layout whose MFMA B-operand reads are conflict-free (M's own reads
// M[j][m] for lanes j = 0..15 fall 16 doubles apart: 8-way LDS conflicts).
// EQ = false (r05, pc_solve_mc_kernel): no equilibration -- M = L^-1 of W
// itself.  Cholesky's backward error is invariant to diagonal scaling (the
// factor of D W D is D times W's, to rounding), so scaling W first changes
// neither which blocks factor nor the span Z keeps; it only put ~1 us of
// broadcasts and scalings on the round's critical path.  d is then not
// written (the MGS^2 fallback forms its scales from W).
template <bool EQ = true>
__device__ __forceinline__ void p16_eq_chol(const double* W, double* L, double* Li, double* M,
                                            double* d, int k, int lane, int* fail, double* Mt = nullptr) {
  double w[kMaxK], x[kMaxK];
  PC_WMARK(30);
#pragma unroll
  for (int m = 0; m < kMaxK; ++m) w[m] = (lane < k && m < k) ? W[lane * k + m] : 0.0;
  double di = 1.0;
  if constexpr (EQ) {
    di = rsqrt_f64(lane < k ? W[lane * k + lane] : 1.0);
#pragma unroll
    for (int m = 0; m < kMaxK; ++m) w[m] *= di * readlane_f64(di, m);
    if (lane < kMaxK) d[lane] = lane < k ? di : 0.0;
  }
  if (lane == 0) *fail = 0;
  p16_chol_regs(w, L, Li, k, lane, fail, x, 37);  // probe marks 37-39
  if (lane < kP16W) {  // lane c: column c of L^-1 diag(d)
#pragma unroll
    for (int i = 0; i < kP16W; ++i) {
      const double v = (lane < k && i < k) ? (EQ ? x[i] * di : x[i]) : 0.0;
      M[i * kP16W + lane] = v;
      if (Mt) Mt[lane * kP16W + i] = v;
    }
  }
  wave_lds_sync();
  PC_WMARK(34);
}

// G2 = G G for the multi-workgroup solve's squared rounds (r06): one
// upper-triangle 16 x 16 tile (a <= b) per 4 waves, which split the MFMA
// k-steps (f64 16x16x4) and are summed in wave order; each element is written
// at (i, j) and (j, i) by ONE thread, so G2 is exactly symmetric.  190 tiles
// of ~19 k-steps each at d = 300.  Run by the solve's own extra workgroups
// (pc_solve_mc_kernel, beside its first round) or by pc_prep_kernel (the
// transposed start); the same k-steps per wave and the same sum order either
// way, so G2 is the same bit for bit.
constexpr int kSqNT = 256;
// G2 tiles per squaring workgroup of the solve's launch (two at a time): 2
// puts 95 workgroups beside the solve's 19 at d = 300, 4 puts 48 (fewer CUs
// held with the solve's LDS allocation).  Alternated A/B (r06,
// tools/ab_libs/build_sq.sh, profiles/r06/sq2/): the solve alone 75.1 vs
// 76.7 us, MOSI's three-split graph 0.215 vs 0.216 ms, POM's 0.343 vs 0.344
#ifndef MMB_SQ_PER_WG
#define MMB_SQ_PER_WG 2
#endif
constexpr int kSqPerWg = MMB_SQ_PER_WG;
static_assert(kSqPerWg % 2 == 0, "two tiles per pass");
__device__ __forceinline__ void square_tile_ab(int blk, int T, int& a, int& b) {
  int rem = blk;
  a = 0;  // blk -> (a, b), a <= b, row-major over the upper triangle
  while (rem >= T - a) {
    rem -= T - a;
    ++a;
  }
  b = a + rem;
}
// wave wv (0-3) of the tile's group: its k-steps' MFMA partial into part4[wv]
__device__ __forceinline__ void square_tile_partials(const double* __restrict__ G, int D, int blk,
                                                     int wv, int lane, double* part4) {
  const int T = (D + 15) / 16;
  int a, b;
  square_tile_ab(blk, T, a, b);
  const int Ks = (D + 3) / 4;
  const int pa = a * 16 + (lane & 15), pb = b * 16 + (lane & 15);
  // every k-step's two operands loaded before the first MFMA (<= 20 k-steps
  // per wave at D <= 320): one round trip of G reads, not one per k-step group
  constexpr int kSqKs = (kP16MaxD / 4 + kSqNT / kWave - 1) / (kSqNT / kWave);  // 20
  double x[kSqKs], y[kSqKs];
#pragma unroll
  for (int u = 0; u < kSqKs; ++u) {
    const int st = wv + (kSqNT / kWave) * u;
    const int q = 4 * st + (lane >> 4);
    const bool okq = st < Ks && q < D;
    // A[i][k] = G[a16 + i][q] = G[q][a16 + i] (symmetric), B[k][j] = G[q][b16 + j]
    x[u] = (okq && pa < D) ? G[static_cast<int64_t>(q) * D + pa] : 0.0;
    y[u] = (okq && pb < D) ? G[static_cast<int64_t>(q) * D + pb] : 0.0;
  }
  f64x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < kSqKs; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x[u], y[u], acc, 0, 0, 0);
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) part4[wv * 256 + ((lane >> 4) + 4 * reg) * 16 + (lane & 15)] = acc[reg];
}
// element e (0-255) of the tile: the four partials in wave order, stored at
// (i, j) and (j, i); WT: write-through (agent-scope) stores for readers of
// the same launch on other XCDs
template <bool WT>
__device__ __forceinline__ void square_tile_store(int D, double* __restrict__ G2, int blk, int e,
                                                  const double* part4) {
  const int T = (D + 15) / 16;
  int a, b;
  square_tile_ab(blk, T, a, b);
  const int i = e >> 4, j = e & 15;
  double v = 0.0;
#pragma unroll
  for (int w = 0; w < kSqNT / kWave; ++w) v += part4[w * 256 + e];
  const int r = a * 16 + i, c = b * 16 + j;
  if (r < D && c < D && (a != b || i <= j)) {
    if (WT) {
      const unsigned long long bits = __builtin_bit_cast(unsigned long long, v);
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(G2 + static_cast<int64_t>(r) * D + c), bits,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(G2 + static_cast<int64_t>(c) * D + r), bits,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      G2[static_cast<int64_t>(r) * D + c] = v;
      G2[static_cast<int64_t>(c) * D + r] = v;
    }
  }
}

// Since r05 an implicit round exchanges the RAW product H_t = G_t B_r, which
// needs no factor of W_r, so the equilibrated Cholesky of W_r (the last wave) runs
// beside the whole exchange -- partials, publish, the wait for the other
// workgroups and the gather of H = G B_r -- instead of before it.  After the
// join every workgroup forms B_{r+1} = H M_r^T (the tiles Y_t of r04, the
// same MFMAs on the same operands) and W_{r+1} = B_{r+1}^T B_{r+1} from its
// own copy of the rows (per-wave partial Grams summed in a fixed wave order:
// identical in all workgroups), so the exchange carries 16 x 16 per tile
// instead of 16 x 32.  The partial waves synchronise among themselves through
// an LDS arrival counter while the last wave factors (s_barrier would wait
// for it).  A round whose factor fails (a pivot <= 0) drops H and runs a
// second exchange of G_t Z for the MGS^2-orthonormalised block; the round
// entering the tail is the r04 round (the factor beside the partials,
// explicit CholeskyQR2 rows for the transposed branch).  Exchange x
// (counting the extra ones) arrives at T x .. T (x + 1) - 1 and uses tile
// buffer x & 1.
//
// 8 waves, not r04's 16: at 1024 threads a wave has 128 VGPRs, and with the
// factor's 16-entry rows, the G fragments and the gather's loads in one
// kernel the compiler spilled ~70 VGPRs -- the G fragments reloaded from
// scratch before every MFMA, the gather's addresses spilled and reloaded
// around every load (probe: the round's non-factor work 2x slower than its
// operations).  At 512 threads there are 256.
constexpr int kPnNT = 512;
constexpr int kPnNW = kPnNT / kWave;                   // 8
constexpr int kPnPw = kPnNW - 1;                       // waves holding G (the last one factors)
constexpr int kPnKs = (kP16MaxD / 4 + kPnPw - 1) / kPnPw;  // k-steps of G per wave (12)
constexpr int kPnGu = (kPmMaxT * 256 + kPnPw * kWave - 1) / (kPnPw * kWave);  // gather loads per thread (12)

// ABL (tools build only, timing ablations, results invalid): 1 skips the
// round's B_{r+1} / W_{r+1} update, 2 skips the round's factor
template <int ABL = 0>
__global__ __launch_bounds__(kPnNT) void pc_solve_mc_kernel(const double* __restrict__ G,
                                                               double* __restrict__ G2, int nsq_wg, int D,
                                                               const double* __restrict__ z0, int k,
                                                               int npc, int n_iter, int transposed,
                                                               double* __restrict__ pc_out,
                                                               double* xbuf, unsigned* ctl,
                                                               int32_t* flag) {
  extern __shared__ __attribute__((aligned(16))) double p16_lds[];
  const int Dp = (D + 15) / 16 * 16;
  int T = Dp / 16;
  double* sZ = p16_lds;          // H = G B_r (implicit rounds); the explicit block Z
  double* sY = sZ + Dp * kP16W;  // the raw block B_r (z0, then G Z_{r-1}); G Z for the tail
  double* part = sY + Dp * kP16W;  // max(16 x 256, Dp x 16)
  P16_SMALL_DECL
  __shared__ double sHt[256], sYt[256], sM[256], sM2[256], sd[kMaxK];
  __shared__ int s_abort;
  __shared__ unsigned s_bar;
  int tid = threadIdx.x, lane = tid & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int t = blockIdx.x;
  unsigned* ctr = ctl;
  unsigned* abort_w = ctl + 1;
  unsigned* sq_ctr = ctl + 2;  // the squaring workgroups' arrivals

  if (t >= T) {
    // workgroups T .. T + nsq_wg - 1 (r06b): G2 = G G, kSqPerWg tiles each,
    // two at a time (waves 0-3 and 4-7), while the solve's workgroups run
    // their first round by G.  Write-through stores, drained by every wave,
    // then one arrival; the solve waits for all nsq_wg before its first
    // squared round.  An arrival that finds the count already met is a
    // workspace handed over dirty.
    double* part4 = p16_lds + 2 * Dp * kP16W + (wave >> 2) * 4 * 256;
    const int ntiles = T * (T + 1) / 2;
#pragma unroll 1
    for (int pass = 0; pass < kSqPerWg / 2; ++pass) {
      const int blk = kSqPerWg * (t - T) + 2 * pass + (wave >> 2);
      if (blk < ntiles) square_tile_partials(G, D, blk, wave & 3, lane, part4);
      __syncthreads();
      if (blk < ntiles) square_tile_store<true>(D, G2, blk, tid & 255, part4);
      __syncthreads();  // part4 is read before the next pass writes it
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const unsigned old = __hip_atomic_fetch_add(sq_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old >= static_cast<unsigned>(nsq_wg)) {
        __hip_atomic_store(abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (flag) atomicOr(flag, MMB_FLAG_SYNC_TIMEOUT);
      }
    }
    return;
  }

  // this workgroup's 16 rows of the round's matrix as MFMA A fragments on
  // waves 0-6 (symmetric: row p of the tile = column p, 16 consecutive
  // doubles per k-row: coalesced); wave 7 is free for the k x k factor that
  // overlaps the rest.  Since r06 n_sq = (n_iter - 1) / 2 rounds multiply
  // by G2 = G G, each standing for two power iterations: span(G^7 Z0) =
  // span(G2^3 G Z0), so the PC is sklearn's to rounding, with 4 exchange
  // rounds instead of 7.  The schedule is G, then the n_sq rounds by G2, then
  // what is left (n_iter even: one more) by G, and the tail by G: the first
  // round needs no G2, so the squaring workgroups of this launch (nsq_wg > 0)
  // form it beside that round instead of a launch in front of the solve
  const int n_sq = (G2 && n_iter >= 3) ? (n_iter - 1) / 2 : 0;
  double ga[kPnKs];
  // (G2 from this launch's squaring workgroups is read after the acquire
  // that follows their arrivals, so plain loads see it)
  auto load_rows = [&](const double* M) {
    const int p = t * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < kPnKs; ++j) {
      const int q = 4 * (wave + kPnPw * j) + (lane >> 4);
      ga[j] = (wave < kPnPw && p < D && q < D) ? M[static_cast<int64_t>(q) * D + p] : 0.0;
    }
  };
  load_rows(G);
  // waves 0-6: their partial products of this tile of G with a [Dp][16] block
  auto tile_partials = [&](const double* B) {
    if (wave < kPnPw) {
      f64x4 acc = {0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < kPnKs; ++j) {
        const int q = 4 * (wave + kPnPw * j) + (lane >> 4);
        if (4 * (wave + kPnPw * j) < Dp)
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ga[j], B[q * kP16W + (lane & 15)], acc, 0, 0, 0);
      }
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) part[wave * 256 + ((lane >> 4) + 4 * reg) * 16 + (lane & 15)] = acc[reg];
    }
  };
  // ... summed over the waves in a fixed order (threads 0-255; the caller
  // synchronises before and after); tr: the tile's transpose
  auto tile_sum = [&](double* out, bool tr = false) {
    if (tid < 256) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < kPnPw; ++w) s += part[w * 256 + tid];
      out[tr ? (tid & 15) * 16 + (tid >> 4) : tid] = s;
    }
  };
  auto tile_product = [&](const double* B, double* out) {
    tile_partials(B);
    __syncthreads();
    tile_sum(out);
    __syncthreads();
  };
  // the barrier of waves 0-6 while wave 7 factors: every wave adds one
  // arrival to an LDS counter after its LDS writes, then polls for the
  // phase's 7 arrivals (the counter only grows within a launch)
  unsigned bar_target = 0;
  auto bar_pw = [&]() {
    bar_target += kPnPw;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) {
      __hip_atomic_fetch_add(&s_bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      while (__hip_atomic_load(&s_bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < bar_target)
        __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  };
  // MGS^2 of the k columns of a [Dp][16] block on wave 0 (extreme
  // ill-conditioning: a Cholesky pivot <= 0), in place
  auto mgs = [&](double* B) {
    if (wave == 0) {
      for (int e = lane; e < D * k; e += kWave) part[e] = B[(e / k) * kP16W + e % k];
      wave_lds_sync();
      orth_wave(part, D, k, lane);
      for (int e = lane; e < D * k; e += kWave) B[(e / k) * kP16W + e % k] = part[e];
    }
    __syncthreads();
  };
  // wave 0: publishes this workgroup's 16 x 16 tile for exchange x with
  // write-through 8-byte stores, drains them and adds one arrival; then waits
  // for all T (not after the final exchange, except workgroup 0, which then
  // returns the counter to zero: every workgroup has made its last arrival,
  // so the next launch -- eager or a graph replay -- finds it at 0 with no
  // memset node in front of it).  A failed arrival or wait sets s_abort.
  auto publish = [&](const double* tile, int x, bool final_x) {
    double* xb = xbuf + static_cast<int64_t>(x & 1) * T * 256;
    wave_lds_sync();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = lane + kWave * u;
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(xb + t * 256 + e),
                         __builtin_bit_cast(unsigned long long, tile[e]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
      // release: the tile stores above are visible at agent scope before
      // the arrival that announces them
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      if (!pm_arrive(ctr, T, x, abort_w, flag)) {
        s_abort = 1;
      } else if (!(final_x && t != 0)) {
        if (!pm_wait(ctr, static_cast<unsigned>(T * (x + 1)), abort_w, flag)) {
          s_abort = 1;
        } else if (final_x) {
          __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(sq_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // acquire: the gather reads the other workgroups' tiles only after
        // their arrivals were observed (the barrier that follows releases the
        // other waves of this workgroup)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
    }
  };
  // every tile of exchange x into dst by the first nthr threads (element f =
  // tid + nthr u of the T x 256 published doubles, copied to dst[f]: a
  // row-major tile lands as rows t*16.. of a [Dp][16] block, a transposed one
  // as a [T][16][16] stack of transposed tiles), all of a thread's loads (sc1,
  // 8 B) issued before any is used (a load-then-store loop waited ~1.5 us per
  // load)
  auto gather = [&](double* dst, int x, int nthr) {
    if (tid < nthr) {
      const double* xb = xbuf + static_cast<int64_t>(x & 1) * T * 256;
      double v[kPnGu];
#pragma unroll
      for (int u = 0; u < kPnGu; ++u) {
        const int f = tid + nthr * u;
        v[u] = f < T * 256 ? __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(xb + f),
                                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                           : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kPnGu; ++u) {
        const int f = tid + nthr * u;
        if (f < T * 256) dst[f] = v[u];
      }
    }
  };
  // no caller may go on with a stale PC: an aborted solve leaves NaN in
  // pc_out (every aborting workgroup writes the same NaNs; workgroup 0
  // cannot complete the tail once any workgroup has left).  After a barrier.
  auto aborted = [&]() -> bool {
    if (!s_abort) return false;
    for (int e = tid; e < npc * D; e += kPnNT) pc_out[e] = __builtin_nan("");
    return true;
  };

  for (int e = tid; e < Dp * kP16W; e += kPnNT) {
    const int p = e / kP16W, j = e % kP16W;
    sY[e] = (p < D && j < k) ? z0[p * k + j] : 0.0;
    sZ[e] = 0.0;
  }
  if (tid == 0) {
    s_abort = 0;
    s_bar = 0;
  }
  __syncthreads();
  PC_MARK(0);
  p16_gram<kPnNW>(sY, sY, Dp, k, part, sW);  // W_0 = B_0^T B_0 (every workgroup: identical)
  PC_MARK(1);

  int x = 0;  // the exchange
  const int T0 = T, k0 = k;
  const int n_rounds = n_iter - n_sq;  // 1 + n_sq + (n_iter - 1 - 2 n_sq)
  for (int r = 0; r < n_rounds; ++r) {
    if (n_sq > 0 && r == 1) {
      if (nsq_wg > 0) {  // G2 from this launch's squaring workgroups
        if (tid == 0) {
          if (!pm_wait(sq_ctr, static_cast<unsigned>(nsq_wg), abort_w, flag)) s_abort = 1;
          // the acquire's L1 invalidate completes asynchronously: wait for it
          // before the barrier releases the other waves' plain loads of G2
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (aborted()) return;
      }
      load_rows(G2);
    }
    if (n_sq > 0 && r == 1 + n_sq) load_rows(G);  // G2's rounds done
    {
      // the round's LDS addresses, bounds and per-lane indices are rebuilt
      // from an opaque zero every round: left loop-invariant, the compiler
      // hoisted all of them out of the loop (hundreds of values held across
      // the kernel) and spilled the G fragments and the gather's addresses
      int zo = 0;
      asm volatile("" : "+s"(zo));
      sZ = p16_lds + zo;
      sY = sZ + Dp * kP16W;
      part = sY + Dp * kP16W;
      T = T0 + zo;
      k = k0 + zo;
      tid = static_cast<int>(threadIdx.x) + zo;
      lane = tid & (kWave - 1);
    }
    if (wave == kPnPw) {
      if (!(ABL & 2)) p16_eq_chol<false>(sW, sL, sLi, sM, sd, k, lane, &s_fail, sM2);  // M_r, beside the exchange
    } else {
      tile_partials(sY);
      bar_pw();
      tile_sum(sHt, true);  // H_t^T, H_t = G_t B_r
      bar_pw();
      if (wave == 0) {
        publish(sHt, x, false);
        PC_WMARK(2 + 3 * r);
      }
      bar_pw();
      gather(sZ, x, kPnPw * kWave);  // H = G B_r as T transposed tiles
      if (wave == 0) PC_WMARK(3 + 3 * r);
    }
    ++x;
    __syncthreads();  // the join: M_r, s_fail and H
    PC_MARK(44 + 2 * r);
    if (aborted()) return;
    if (s_fail) {
      // the equilibrated rows of B_r orthonormalised by MGS^2 (H is dropped),
      // then a second exchange of G_t Z
      for (int e = tid; e < Dp * kP16W; e += kPnNT) {
        const int p = e / kP16W, j = e % kP16W;
        sZ[e] = (p < D && j < k) ? sY[e] * rsqrt_f64(sW[j * k + j]) : 0.0;  // the equilibrated rows
      }
      __syncthreads();
      mgs(sZ);
      tile_product(sZ, sHt);
      if (wave == 0) publish(sHt, x, false);
      __syncthreads();
      if (aborted()) return;
      gather(sY, x, kPnNT);  // B_{r+1} = G Z
      ++x;
      __syncthreads();
      p16_gram<kPnNW>(sY, sY, Dp, k, part, sW);  // W_{r+1}
    } else if (!(ABL & 1)) {
      // B_{r+1} = H M_r^T tile by tile (all 8 waves), each wave's tiles' Grams
      // accumulated in its MFMA registers; W_{r+1} = their fixed-order sum.
      // Both operands are read from transposed copies (H's tiles as
      // gathered, M^T from the factor): lane (i, k) reads element 16 k + i,
      // conflict-free, where the rows' own layout put the 16 i of a read 128 B
      // apart (8-way bank conflicts: the update took ~5 us a round, r05
      // tools/pc_probe/rmul_bench.hip).  The tile's Gram Y^T Y takes its
      // operands straight from the accumulator: its k-step st is Y's rows
      // 4 st .. 4 st + 3, which is acc[st] in both operand layouts.
      f64x4 pa = {0, 0, 0, 0};
      for (int tt = wave; tt < T; tt += kPnNW) {
        f64x4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          const int m = 4 * st + (lane >> 4);
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sZ[tt * 256 + m * 16 + (lane & 15)],
                                                     sM2[m * kP16W + (lane & 15)], acc, 0, 0, 0);
        }
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) sY[(tt * 16 + (lane >> 4) + 4 * reg) * kP16W + (lane & 15)] = acc[reg];
#pragma unroll
        for (int st = 0; st < 4; ++st) pa = __builtin_amdgcn_mfma_f64_16x16x4f64(acc[st], acc[st], pa, 0, 0, 0);
      }
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) part[wave * 256 + ((lane >> 4) + 4 * reg) * 16 + (lane & 15)] = pa[reg];
      if (wave == 0) PC_WMARK(35);
      __syncthreads();
      if (wave == 0) PC_WMARK(36);
      if (tid < 256) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kPnNW; ++w) s += part[w * 256 + tid];
        const int i = tid >> 4, j = tid & 15;
        if (i < k && j < k) sW[i * k + j] = s;
      }
      __syncthreads();
    }
    PC_MARK(45 + 2 * r);
  }

  if (n_sq > 0 && n_rounds == 1 + n_sq) load_rows(G);  // (the tail's product is by G)
  if (!transposed) {
    // The direct branch's last round (r06) as an implicit round: the RAW
    // product H_t = G_t B is exchanged beside the factor of W (as in the
    // loop), and workgroup 0 alone forms Z = B M^T and G Z = H M^T after the
    // join -- the factor no longer precedes the exchange (r05: factor 5.6 us,
    // then the Y_t exchange 4.5 us, back to back).  The other workgroups
    // arrive without waiting; workgroup 0 waits for all T and, once the
    // factor held, returns the counter to zero.  A failed factor (pivot <= 0)
    // falls through to the explicit MGS^2 block below with exchange x + 1:
    // every workgroup is still there (they return only after the join).
    if (wave == kPnPw) {
      p16_eq_chol<false>(sW, sL, sLi, sM, sd, k, lane, &s_fail, sM2);
    } else {
      tile_partials(sY);
      bar_pw();
      tile_sum(sHt, true);  // H_t^T
      bar_pw();
      if (wave == 0) {
        double* xb = xbuf + static_cast<int64_t>(x & 1) * T * 256;
        wave_lds_sync();
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = lane + kWave * u;
          __hip_atomic_store(reinterpret_cast<unsigned long long*>(xb + t * 256 + e),
                             __builtin_bit_cast(unsigned long long, sHt[e]), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          if (!pm_arrive(ctr, T, x, abort_w, flag)) {
            s_abort = 1;
          } else if (t == 0) {
            if (!pm_wait(ctr, static_cast<unsigned>(T * (x + 1)), abort_w, flag)) s_abort = 1;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          }
        }
      }
    }
    __syncthreads();  // the join: M, s_fail, the arrival
    PC_MARK(44 + 2 * n_iter);
    if (aborted()) return;
    if (!s_fail) {
      if (t != 0) return;  // the tail runs on workgroup 0 only
      if (tid == 0) {
        __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(sq_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      p16_rmul<kPnNW, true>(sY, sM2, part, Dp);  // Z = B M^T (into the scratch block)
      gather(sZ, x, kPnNT);                        // H as T transposed tiles
      __syncthreads();
      for (int tt = wave; tt < T; tt += kPnNW) {  // G Z = H M^T (sY free: B is in Z)
        f64x4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          const int m = 4 * st + (lane >> 4);
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sZ[tt * 256 + m * 16 + (lane & 15)],
                                                     sM2[m * kP16W + (lane & 15)], acc, 0, 0, 0);
        }
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) sY[(tt * 16 + (lane >> 4) + 4 * reg) * kP16W + (lane & 15)] = acc[reg];
      }
      __syncthreads();
      double* zb = part;  // Z into sZ's place, the H tiles' block becomes the scratch
      part = sZ;
      sZ = zb;
      PC_MARK(45 + 2 * n_iter);
    } else {
      // the explicit block's exchange follows: no workgroup may arrive at
      // x + 1 before all T arrived at x (pm_arrive's range check), so the
      // workgroups that did not wait above wait now
      if (t != 0 && tid == 0 && !pm_wait(ctr, static_cast<unsigned>(T * (x + 1)), abort_w, flag))
        s_abort = 1;
      __syncthreads();
      if (aborted()) return;
      ++x;
    }
  }
  // the transposed branch (an orthonormal Q: CholeskyQR2 rows) and a failed
  // pivot (MGS^2): explicit rows Z, then the final exchange of Y_t = G_t Z
  if (transposed || s_fail) {
    if (transposed) {  // (the direct branch factored above)
      if (wave == kPnPw) {
        p16_eq_chol<false>(sW, sL, sLi, sM, sd, k, lane, &s_fail, sM2);
      } else {
        tile_partials(sY);
      }
      __syncthreads();
      PC_MARK(44 + 2 * n_iter);
    }
    if (s_fail) {  // the equilibrated rows, orthonormalised by MGS^2
      for (int e = tid; e < Dp * kP16W; e += kPnNT) {
        const int p = e / kP16W, j = e % kP16W;
        sZ[e] = (p < D && j < k) ? sY[e] * rsqrt_f64(sW[j * k + j]) : 0.0;  // the equilibrated rows
      }
      __syncthreads();
      mgs(sZ);
    } else {
      p16_rmul<kPnNW>(sY, sM, sZ, Dp);  // Z1 = B M1^T
      __syncthreads();
      p16_gram<kPnNW>(sZ, sZ, Dp, k, part, sW);  // second CholeskyQR pass on the rows
      if (wave == 0) {
        if (lane == 0) s_fail = 0;
        wave_lds_sync();
        p16_chol(sW, sL, sLi, k, lane, &s_fail);
        for (int e = lane; e < 256; e += kWave) {
          const int j = e / kP16W, m = e % kP16W;
          sM2[e] = (j < k && m <= j) ? sLi[j * k + m] : 0.0;
        }
      }
      __syncthreads();
      if (s_fail) {
        mgs(sZ);
      } else {
        p16_rmul<kPnNW>(sZ, sM2, sY, Dp);  // Z = Z1 L2^-T (sY free: B is no longer needed)
        __syncthreads();
        for (int e = tid; e < Dp * kP16W; e += kPnNT) sZ[e] = sY[e];
        __syncthreads();
      }
    }
    tile_product(sZ, sYt);  // Y_t = G_t Z
    if (wave == 0) publish(sYt, x, true);
    if (t != 0) return;  // the tail runs on workgroup 0 only
    __syncthreads();
    PC_MARK(45 + 2 * n_iter);
    if (aborted()) return;
    gather(sY, x, kPnNT);  // G Z
    __syncthreads();
  }
  // the direct branch's two Grams in one pass: H = (G Z)^T (G Z), W = Z^T G Z
  // (the transposed branch forms its own Q^T G Q in the tail)
  if (!transposed) p16_gram2<kPnNW>(sY, sY, sT, sZ, sY, sW, Dp, k, part);
  PC_MARK(40);
  p16_tail<kPnNW>(sZ, sY, D, Dp, k, npc, transposed, part, sm, pc_out, sT, !transposed);
  // a workspace handed over with a stale count in (0, T) lets the final wait
  // pass early; the overshooting arrivals set the abort word.  Re-read it
  // after the tail so a PC that raced them is overwritten with NaN (the flag
  // word stays the primary signal)
  __syncthreads();
  if (__hip_atomic_load(abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    for (int e = tid; e < npc * D; e += kPnNT) pc_out[e] = __builtin_nan("");
  PC_PROBE_FLUSH();
}

__device__ __forceinline__ void gram_square_tile(const double* __restrict__ G, int D,
                                                 double* __restrict__ G2, int blk) {
  __shared__ double part[kSqNT / kWave][256];
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  square_tile_partials(G, D, blk, wave, lane, &part[0][0]);
  __syncthreads();
  square_tile_store<false>(D, G2, blk, threadIdx.x, &part[0][0]);
}

// The transposed branch's start in ONE launch (r06): workgroups [0, nsq)
// square G (gram_square_tile), the next ceil(D / 4) form z0 = X^T Omega_n
// (xt_omega_wave_kernel's body: one wave per feature).  Two launches of ~5
// and ~11 us back to back before the solve of every dataset split (POM's
// and MOSI's small ones: n < d).
__global__ __launch_bounds__(kSqNT) void pc_prep_kernel(const double* __restrict__ G, int D,
                                                        double* __restrict__ G2, int nsq,
                                                        const float* __restrict__ X, int64_t N,
                                                        const double* __restrict__ om, int k,
                                                        double* __restrict__ z0) {
  if (static_cast<int>(blockIdx.x) < nsq) {
    gram_square_tile(G, D, G2, blockIdx.x);
    return;
  }
  xt_omega_wave_body<float, false>(X, nullptr, N, D, om, k, z0, static_cast<int>(blockIdx.x) - nsq);
}

inline size_t p16_lds_bytes(int d) {
  const size_t dp = (d + 15) / 16 * 16;
  return (2 * dp * kP16W + (dp * kP16W > 16 * 256 ? dp * kP16W : 16 * 256)) * sizeof(double);
}

// ------------------------------------------------------------------ pc_remove
template <int VEC, int PER, typename TX = float>
__global__ __launch_bounds__(256) void pc_remove_kernel(const TX* __restrict__ num,
                                                        const float* __restrict__ cnt, int64_t N,
                                                        int D, const double* __restrict__ pc,
                                                        int npc, float* __restrict__ out32,
                                                        double* __restrict__ out64) {
  extern __shared__ double s_pc[];
  for (int e = threadIdx.x; e < npc * D; e += blockDim.x) s_pc[e] = pc[e];
  __syncthreads();
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int U = D / VEC;
  const int64_t wstride = static_cast<int64_t>(gridDim.x) * (blockDim.x / kWave);
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * (blockDim.x / kWave) + wave; row < N;
       row += wstride) {
    const float sc = cnt ? cnt[row] : 1.f;
    double x[PER][VEC];
#pragma unroll
    for (int m = 0; m < PER; ++m) {
      const int u = lane + kWave * m;
      TX v[VEC];
      if (u < U) {
        if constexpr (VEC == 4) {
          const float4 q = *reinterpret_cast<const float4*>(num + row * D + u * 4);
          v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
          v[0] = num[row * D + u];
        }
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e) v[e] = TX(0);
      }
#pragma unroll
      for (int e = 0; e < VEC; ++e) x[m][e] = static_cast<double>(cnt ? v[e] / sc : v[e]);
    }
    double y[PER][VEC];
#pragma unroll
    for (int m = 0; m < PER; ++m)
#pragma unroll
      for (int e = 0; e < VEC; ++e) y[m][e] = 0.0;
    for (int c = 0; c < npc; ++c) {
      const double* pcc = s_pc + c * D;
      double d = 0.0;
#pragma unroll
      for (int m = 0; m < PER; ++m) {
        const int u = lane + kWave * m;
        if (u < U) {
#pragma unroll
          for (int e = 0; e < VEC; ++e) d = fma(x[m][e], pcc[u * VEC + e], d);
        }
      }
      d = wave_sum(d);
#pragma unroll
      for (int m = 0; m < PER; ++m) {
        const int u = lane + kWave * m;
        if (u < U) {
#pragma unroll
          for (int e = 0; e < VEC; ++e) y[m][e] = fma(d, pcc[u * VEC + e], y[m][e]);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < PER; ++m) {
      const int u = lane + kWave * m;
      if (u < U) {
        if (out32) {
          if constexpr (VEC == 4) {
            float4 q;
            q.x = static_cast<float>(x[m][0] - y[m][0]);
            q.y = static_cast<float>(x[m][1] - y[m][1]);
            q.z = static_cast<float>(x[m][2] - y[m][2]);
            q.w = static_cast<float>(x[m][3] - y[m][3]);
            *reinterpret_cast<float4*>(out32 + row * D + u * 4) = q;
          } else {
            out32[row * D + u] = static_cast<float>(x[m][0] - y[m][0]);
          }
        } else {
#pragma unroll
          for (int e = 0; e < VEC; ++e) out64[row * D + u * VEC + e] = x[m][e] - y[m][e];
        }
      }
    }
  }
}

// One PC, f32 rows of 256 < D <= 512 (float4 columns l and l + 64 per lane):
// R rows per wave in flight -- all 2R row loads issued before the first dot,
// the R wave sums interleaved -- where pc_remove_kernel has one row and its
// dependent load -> dot -> sum -> store chain per wave; the PC's lane values
// stay in registers.  Arithmetic (f64 fma order, shuffle-tree wave sum, f32
// rounding) is pc_remove_kernel<4, 2>'s: bit-identical.
// NT (tools build, MMB_PC_REMOVE_NT=1): x read and the rows written
// non-temporally -- an A/B of whether the removal's 2 x N x D x 4 bytes evict
// the word rows the next step's fused kernel would find in L2 / MALL
template <int R, bool NT = false>
__global__ __launch_bounds__(256) void pc_remove1_kernel(const float* __restrict__ num,
                                                         const float* __restrict__ cnt, int64_t N,
                                                         int D, const double* __restrict__ pc,
                                                         float* __restrict__ out32) {
  const int lane = threadIdx.x & (kWave - 1);
  const int U = D / 4;
  const bool h1 = lane + kWave < U;
  double p[2][4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    p[0][e] = lane < U ? pc[4 * lane + e] : 0.0;
    p[1][e] = h1 ? pc[4 * (lane + kWave) + e] : 0.0;
  }
  const int64_t nw = static_cast<int64_t>(gridDim.x) * (blockDim.x / kWave);
  for (int64_t base = (static_cast<int64_t>(blockIdx.x) * (blockDim.x / kWave) + threadIdx.x / kWave) * R;
       base < N; base += nw * R) {
    float4 v[R][2];
    float sc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t row = min(base + r, N - 1);
      const float* src = num + row * D;
      auto ld = [](const float* q) {
        if constexpr (NT) {
          using f4 = float __attribute__((ext_vector_type(4)));
          const f4 t = __builtin_nontemporal_load(reinterpret_cast<const f4*>(q));
          return make_float4(t.x, t.y, t.z, t.w);
        } else {
          return *reinterpret_cast<const float4*>(q);
        }
      };
      v[r][0] = lane < U ? ld(src + 4 * lane) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[r][1] = h1 ? ld(src + 4 * (lane + kWave)) : make_float4(0.f, 0.f, 0.f, 0.f);
      sc[r] = cnt ? cnt[row] : 1.f;
    }
    double x[R][2][4], d[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const float e4[4] = {v[r][m].x, v[r][m].y, v[r][m].z, v[r][m].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) x[r][m][e] = static_cast<double>(cnt ? e4[e] / sc[r] : e4[e]);
      }
      double acc = 0.0;
      if (lane < U) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = fma(x[r][0][e], p[0][e], acc);
      }
      if (h1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = fma(x[r][1][e], p[1][e], acc);
      }
      d[r] = acc;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
      for (int r = 0; r < R; ++r) d[r] += __shfl_xor(d[r], o, kWave);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (base + r >= N) break;
      float* dst = out32 + (base + r) * D;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        if (m == 0 ? lane < U : h1) {
          float4 q;
          q.x = static_cast<float>(x[r][m][0] - fma(d[r], p[m][0], 0.0));
          q.y = static_cast<float>(x[r][m][1] - fma(d[r], p[m][1], 0.0));
          q.z = static_cast<float>(x[r][m][2] - fma(d[r], p[m][2], 0.0));
          q.w = static_cast<float>(x[r][m][3] - fma(d[r], p[m][3], 0.0));
          if constexpr (NT) {
            using f4 = float __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(f4{q.x, q.y, q.z, q.w}, reinterpret_cast<f4*>(dst + 4 * (lane + kWave * m)));
          } else {
            *reinterpret_cast<float4*>(dst + 4 * (lane + kWave * m)) = q;
          }
        }
      }
    }
  }
}

// pc_remove1_kernel rows per wave (2, 4, 8); 0 = pc_remove_kernel.  Measured
// (tools/remove_ab.py, 1M x 300, r02q): R = 0 / 2 / 4 / 8 = 0.529 / 0.455 /
// 0.435 / 0.444 ms, all bit-identical
#ifndef MMB_HOOK_PC_REMOVE_R  // (tools/diag: MMB_PC_REMOVE_R)
#define MMB_HOOK_PC_REMOVE_R 4
#endif
static int remove_rows() { return MMB_HOOK_PC_REMOVE_R; }

template <int VEC, int PER, typename TX = float>
static int launch_remove(const TX* num, const float* cnt, int64_t n, int d, const double* pc,
                         int npc, float* out32, double* out64, hipStream_t stream) {
  const int64_t waves = ceil_div(n, 1);
  const int grid = static_cast<int>(std::min<int64_t>(ceil_div(waves, 4), 256 * 8));
  pc_remove_kernel<VEC, PER, TX><<<grid, 256, sizeof(double) * npc * d, stream>>>(num, cnt, n, d, pc, npc, out32, out64);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

struct GramPlan {
  int nb, npairs, S, xcd;
  int64_t chunk;
};

static GramPlan gram_plan(int64_t n, int d) {
  GramPlan p;
  p.nb = static_cast<int>(ceil_div(d, kGB));
  p.npairs = p.nb * (p.nb + 1) / 2;
  int64_t S = n / 4096;
  if (S < 1) S = 1;
  if (S > 128) S = 128;
  if (S >= 8) S = S / 8 * 8;
  p.S = static_cast<int>(S);
  p.xcd = (p.S % 8 == 0) ? 1 : 0;
  p.chunk = ceil_div(ceil_div(n, p.S), 4) * 4;
  return p;
}

struct Gram2Plan {
  int nt, T, R, xcd;
  int64_t chunk;
};

// at most 128 row ranges = 256 workgroups, one per CU (measured on MI355X at
// 1M rows: 1.87 ms with 128, 1.95 with 256, 2.08 with 512, partial reduction
// included); fewer ranges also halve the partials the reduction reads
constexpr int kG2MaxR = 128;

static Gram2Plan gram2_plan(int64_t n, int d) {
  Gram2Plan p;
  p.nt = static_cast<int>(ceil_div(d, 16));
  p.T = p.nt * (p.nt + 1) / 2;
  // ranges of >= 512 rows -- but at least 16 ranges (32 workgroups) once
  // there are 64 rows per range: a dataset split (1284 rows) ran on 4
  // workgroups (0.15 ms)
  int64_t R = n / 512;
  if (R < 16) R = std::min<int64_t>(16, n / 64);
  if (R < 1) R = 1;
  if (R > kG2MaxR) R = kG2MaxR;
  if (R >= 8) R = R / 8 * 8;
  p.R = static_cast<int>(R);
  p.xcd = (p.R % 8 == 0) ? 1 : 0;
  p.chunk = ceil_div(n, p.R);
  return p;
}

// int8 Gram: ranges of >= 64 rows (one k-step) instead of gram2_plan's
// >= 512, so a 10k-row split (POM) fills every CU instead of 32 of them
static Gram2Plan gram_i8_plan(int64_t n, int d) {
  Gram2Plan q = gram2_plan(n, d);
  int64_t R = n / kGiRows;
  if (R < 1) R = 1;
  if (R > kG2MaxR) R = kG2MaxR;
  if (R >= 8) R = R / 8 * 8;
  q.R = static_cast<int>(R);
  q.xcd = (q.R % 8 == 0) ? 1 : 0;
  q.chunk = ceil_div(ceil_div(n, q.R), kGiRows) * kGiRows;
  return q;
}

static size_t gram2_lds() {
  const size_t lds = sizeof(double) * 2 * kG2Rows * kG2Stride;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gram_tri_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    attr = true;
  }
  return lds;
}

static bool gram2_ok(const float* num, int d) {
  // 16-wave tile kernel: d <= 320 (20 tile rows, <= 8 tiles per wave per half)
  return d % 4 == 0 && d <= 320 && (reinterpret_cast<uintptr_t>(num) & 15) == 0;
}



// ---- level-sum int8 Gram (gram_i8l_kernel): plan and parts
struct GramLPlan {
  int nt, T, R, xcd, P;
  GlParts parts;
  int64_t chunk;
};

static int tri_row_host(int tau, int nt) {
  int r = 0, rem = tau;
  while (rem >= nt - r) {
    rem -= nt - r;
    ++r;
  }
  return r;
}

static void gl_set_features(GlPart& g, int f0, int n0, int f1, int n1) {
  g.f0 = f0;
  g.n0 = n0;
  g.f1 = f1;
  g.n1 = n1;
}

// Three feature groups G0 | G1 | G2 of tile rows (nt split as evenly as it
// goes, the larger groups last) and three parts, one per pair of groups:
// {G0, G1}, {G0, G2}, {G1, G2}.  Each off-diagonal block Gi x Gj goes to part
// {Gi, Gj}; each diagonal block Gg x Gg is cut between the two parts holding
// Gg (row-major: the first x_g tiles to the first of them), the three cuts
// chosen to minimise the largest part (exhaustively: <= 29^3 cases, once per
// nt).  So every part slices two thirds of the features (the three together
// twice x, like a pair of workgroups) while holding a third of the tiles --
// where contiguous runs of the triangle made the first part slice every
// feature.
static GlParts gl_parts_groups3(int nt) {
  GlParts g{};
  const int c = nt / 3 + (nt % 3 > 1 ? 1 : 0), b = nt / 3 + (nt % 3 > 0 ? 1 : 0), a = nt - b - c;
  const int lo[3] = {0, a, a + b}, hi[3] = {a, a + b, nt};
  const int pg[3][2] = {{0, 1}, {0, 2}, {1, 2}};  // part -> its two groups
  const int dpart[3][2] = {{0, 1}, {0, 2}, {1, 2}};  // group -> the two parts holding it
  auto sz = [&](int k) { return hi[k] - lo[k]; };
  const int off[3] = {sz(0) * sz(1), sz(0) * sz(2), sz(1) * sz(2)};  // blocks 01, 02, 12
  int dg[3];
  for (int k = 0; k < 3; ++k) dg[k] = sz(k) * (sz(k) + 1) / 2;
  int bx[3] = {dg[0], dg[1], dg[2]}, best = 1 << 30;
  for (int x0 = 0; x0 <= dg[0]; ++x0)
    for (int x1 = 0; x1 <= dg[1]; ++x1)
      for (int x2 = 0; x2 <= dg[2]; ++x2) {
        int load[3] = {off[0], off[1], off[2]};
        const int xs[3] = {x0, x1, x2};
        for (int k = 0; k < 3; ++k) {
          load[dpart[k][0]] += xs[k];
          load[dpart[k][1]] += dg[k] - xs[k];
        }
        const int m = std::max(load[0], std::max(load[1], load[2]));
        if (m < best) {
          best = m;
          bx[0] = x0;
          bx[1] = x1;
          bx[2] = x2;
        }
      }
  auto group_of = [&](int r) { return r < hi[0] ? 0 : (r < hi[1] ? 1 : 2); };
  std::vector<std::pair<int, int>> lists[3];
  int seen[3] = {0, 0, 0};  // diagonal tiles handed out per group
  for (int ti = 0; ti < nt; ++ti) {
    for (int tj = ti; tj < nt; ++tj) {
      const int gi = group_of(ti), gj = group_of(tj);
      int q;
      if (gi != gj) {
        q = gi == 0 ? (gj == 1 ? 0 : 1) : 2;
      } else {
        q = seen[gi] < bx[gi] ? dpart[gi][0] : dpart[gi][1];
        ++seen[gi];
      }
      lists[q].push_back({ti, tj});
    }
  }
  for (int k = 0; k < 3; ++k) {
    std::sort(lists[k].begin(), lists[k].end());
    g.p[k].n = static_cast<int>(lists[k].size());
    for (int i = 0; i < g.p[k].n && i < kGlMaxPartTiles; ++i)
      g.p[k].tile[i] = static_cast<uint16_t>(lists[k][i].first | (lists[k][i].second << 8));
    const int g0 = pg[k][0], g1 = pg[k][1];
    gl_set_features(g.p[k], 16 * lo[g0], 16 * sz(g0), 16 * lo[g1], 16 * sz(g1));
  }
  return g;
}

// P contiguous runs of the row-major triangle, <= cap tiles each, minimising
// the largest part's modelled cost per 64-row chunk in SIMD cycles: the
// matrix pipe (13 MFMAs x 16 cycles per tile over 4 SIMDs) against vector
// issue (the MFMAs' 8 cycles each plus the slicing of every feature from the
// part's first tile row on: 64 values x ~6.75 vector instructions of 4
// cycles over 64 lanes and 4 SIMDs).  Dynamic program over the split points.
static GlParts gl_parts_runs(int nt, int P, int cap) {
  const int T = nt * (nt + 1) / 2;
  auto cost = [&](int t0, int t1) {
    const int n = t1 - t0;
    if (n <= 0) return 0.0;
    const int nf = 16 * (nt - tri_row_host(t0, nt));
    return std::max(52.0 * n, 26.0 * n + 6.75 * nf);
  };
  std::vector<std::vector<double>> best(P + 1, std::vector<double>(T + 1, 1e300));
  std::vector<std::vector<int>> arg(P + 1, std::vector<int>(T + 1, 0));
  best[0][0] = 0.0;
  for (int k = 1; k <= P; ++k)
    for (int t = 0; t <= T; ++t)
      for (int s = std::max(0, t - cap); s <= t; ++s) {
        const double c = std::max(best[k - 1][s], cost(s, t));
        if (c < best[k][t]) {
          best[k][t] = c;
          arg[k][t] = s;
        }
      }
  int bnd[kGlMaxParts + 1];
  bnd[P] = T;
  for (int k = P; k >= 1; --k) bnd[k - 1] = arg[k][bnd[k]];
  GlParts g{};
  for (int k = 0; k < P; ++k) {
    g.p[k].n = bnd[k + 1] - bnd[k];
    int r0 = nt;
    for (int t = bnd[k]; t < bnd[k + 1] && t - bnd[k] < kGlMaxPartTiles; ++t) {
      const int ti = tri_row_host(t, nt);
      int rem = t;
      for (int r = 0; r < ti; ++r) rem -= nt - r;
      g.p[k].tile[t - bnd[k]] = static_cast<uint16_t>(ti | ((ti + rem) << 8));
      r0 = std::min(r0, ti);
    }
    gl_set_features(g.p[k], 16 * r0, 16 * (nt - r0), 0, 0);
  }
  return g;
}

// R ranges of whole 64-row chunks: as many as keep all P R workgroups
// resident (P = 3: 80 ranges, 240 workgroups -- ten ranges' parts on each
// XCD's 32 CUs), at least one k-step each and at most kGlMaxRows rows each
// (the int32 level sums); a multiple of 8 (the XCD map and
// gram_tri_reduce_kernel) and <= 128 -- mmb_gram_i8 cuts larger calls into
// blocks of kGlBlockRows rows.  The parts depend on nt and the shape only:
// built once per (shape, nt) and cached (the dynamic program costs ~0.1 ms
// of host time, more than a small split's whole Gram).
constexpr int64_t kGlBlockRows = 128 * kGlMaxRows;

static int gram_i8l_ranges(int64_t n, int P) {
  const int64_t resident = 256 / P / 8 * 8;
  int64_t R = std::min<int64_t>(resident, std::max<int64_t>(1, n / kGiRows));
  R = std::max<int64_t>(R, ceil_div(n, kGlMaxRows));
  if (R >= 8) R = ceil_div(R, 8) * 8;
  return static_cast<int>(std::min<int64_t>(R, 128));
}

template <class S, bool GROUPS>
static GramLPlan gram_i8l_plan(int64_t n, int d) {
  GramLPlan q;
  q.nt = static_cast<int>(ceil_div(d, 16));
  q.T = q.nt * (q.nt + 1) / 2;
  q.P = S::kP;
  q.R = gram_i8l_ranges(n, S::kP);
#ifdef MMB_HOOK_GRAM_RANGES  // (tools/diag: MMB_GRAM_RANGES, A/B runs of the range count)
  MMB_HOOK_GRAM_RANGES(q.R);
#endif
  q.xcd = (q.R % 8 == 0) ? 1 : 0;
  q.chunk = ceil_div(ceil_div(std::max<int64_t>(n, 1), q.R), kGiRows) * kGiRows;
  static GlParts cache[kGiF / 16 + 1];
  static bool have[kGiF / 16 + 1] = {};
  if (!have[q.nt]) {
    cache[q.nt] = GROUPS ? gl_parts_groups3(q.nt) : gl_parts_runs(q.nt, S::kP, S::kPartMax);
    have[q.nt] = true;
  }
  q.parts = cache[q.nt];
  return q;
}

template <int DIAG, class S>
static size_t gram_i8l_lds() {
  const size_t lds = 2 * kGiDig * kGiF * kGiRows;  // 160 KB: double-buffered digits
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gram_i8l_kernel<DIAG, S>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    attr = true;
  }
  return lds;
}

// One block of <= kGlBlockRows rows: the level-sum kernel, then the range
// reduction (writing or accumulating into g).
template <int DIAG, class S, bool GROUPS>
static int gram_i8l_block(const float* x, const uint32_t* colmax, int64_t n, int d, double* g,
                          int accumulate, double* part, hipStream_t stream) {
  const GramLPlan q = gram_i8l_plan<S, GROUPS>(n, d);
  int tiles = 0;
  for (int k = 0; k < q.P; ++k) {  // every tile once, within the shape's tiles and items
    MMB_REQUIRE(q.parts.p[k].n <= S::kPartMax);
    MMB_REQUIRE((q.parts.p[k].n0 + q.parts.p[k].n1) * 4 <= S::kIt * S::kNT);
    tiles += q.parts.p[k].n;
  }
  MMB_REQUIRE(tiles == q.T);
  // the buffer-descriptor record count and row offsets are 32-bit byte counts of one range
  MMB_REQUIRE(q.chunk * d * 4 < (int64_t{1} << 31));
  gram_i8l_kernel<DIAG, S><<<S::kP * q.R, S::kNT, gram_i8l_lds<DIAG, S>(), stream>>>(
      x, colmax, n, d, q.nt, q.chunk, q.xcd, q.parts, part);
  MMB_LAUNCH_CHECK();
  const int rc = launch_tri_reduce(part, d, q.nt, q.R, accumulate, g, stream);
  if (rc != MMB_OK) return rc;
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}


}  // namespace mmb

using namespace mmb;

extern "C" size_t mmb_gram_workspace_bytes(int64_t n, int d) {
  const GramPlan p = gram_plan(n, d);
  const size_t v1 = static_cast<size_t>(p.S) * p.npairs * kGB * kGB * sizeof(double);
  const Gram2Plan q = gram2_plan(n, d);
  const size_t v2 = static_cast<size_t>(q.R) * q.T * 256 * sizeof(double);
  const Gram2Plan qi = gram_i8_plan(n, d);
  const size_t v3 = static_cast<size_t>(qi.R) * qi.T * 256 * sizeof(double);
  // the level-sum kernel: at most 128 ranges per block (every shape)
  const int64_t ntl = ceil_div(d, 16);
  const size_t v4 = static_cast<size_t>(gram_i8l_ranges(std::min(n, kGlBlockRows), 2)) *
                    (ntl * (ntl + 1) / 2) * 256 * sizeof(double);  // every shape's ranges bound
  const size_t v23 = std::max(std::max(v2, v3), v4);
  return v1 > v23 ? v1 : v23;
}

extern "C" int mmb_gram(const float* num, const float* cnt, int64_t n, int d, double* g,
                        int accumulate, void* ws, hipStream_t stream) {
  MMB_REQUIRE(num && g && ws && n >= 0 && d > 0);
  double* part = static_cast<double*>(ws);
  const int64_t total = static_cast<int64_t>(d) * d;
  if (n <= kGsMaxN && d <= 320) {  // small splits: tile-parallel, one launch, no partials
    const int nt = static_cast<int>(ceil_div(d, 16));
    // 12 k-steps a group from 512 rows on (24 and 16 spill at 1024
    // threads): MOSI's train split (1284 rows) in two round trips of loads
    // instead of three
    if (n > 512)
      gram_small_kernel<12><<<nt * (nt + 1) / 2, kGsNT, 0, stream>>>(num, cnt, n, d, nt, accumulate, g);
    else
      gram_small_kernel<8><<<nt * (nt + 1) / 2, kGsNT, 0, stream>>>(num, cnt, n, d, nt, accumulate, g);
    MMB_LAUNCH_CHECK();
    return MMB_OK;
  }
  if (gram2_ok(num, d)) {
    const Gram2Plan q = gram2_plan(n, d);
    const size_t lds = gram2_lds();
    gram_tri_kernel<<<2 * q.R, kG2NT, lds, stream>>>(num, cnt, n, d, q.nt, q.R, q.chunk, q.xcd, 0, part);
    MMB_LAUNCH_CHECK();
    {
      const int rc = launch_tri_reduce(part, d, q.nt, q.R, accumulate, g, stream);
      if (rc != MMB_OK) return rc;
    }
    MMB_LAUNCH_CHECK();
    return MMB_OK;
  }
  const GramPlan p = gram_plan(n, d);
  gram_partial_kernel<float><<<p.npairs * p.S, 256, 0, stream>>>(num, cnt, n, d, p.nb, p.npairs, p.S,
                                                         p.chunk, p.xcd, part);
  MMB_LAUNCH_CHECK();
  gram_reduce_kernel<<<static_cast<int>(ceil_div(total, 256)), 256, 0, stream>>>(part, d, p.nb, p.npairs, p.S, accumulate, g);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}


extern "C" int mmb_colmax(const float* x, int64_t n, int d, uint32_t* colmax, int accumulate,
                          hipStream_t stream) {
  MMB_REQUIRE(x && colmax && n >= 0 && d > 0);
  if (!accumulate) {
    const hipError_t e = static_cast<hipError_t>(zero_words_async(colmax, static_cast<int64_t>(sizeof(uint32_t) * d) / 4, stream));
    if (e != hipSuccess) return static_cast<int>(e);
  }
  if (n == 0) return MMB_OK;
  const int64_t rpb = 256;
  const int64_t blocks = ceil_div(n, rpb);
  colmax_kernel<<<static_cast<int>(blocks), d < 256 ? ((d + 63) / 64) * 64 : 256, 0, stream>>>(
      x, n, d, rpb, colmax);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_gram_i8(const float* x, const uint32_t* colmax, int64_t n, int d, double* g,
                           int accumulate, void* ws, hipStream_t stream) {
  MMB_REQUIRE(x && colmax && g && ws && n >= 0 && d > 0 && d <= 304 && d % 4 == 0);
  double* part = static_cast<double*>(ws);
#ifndef MMB_HOOK_GRAM_I8  // (tools/diag: MMB_GRAM_I8_V1, the r04 kernel)
#define MMB_HOOK_GRAM_I8(rc) false
#endif
  {
    int rc_ = MMB_OK;
    if (MMB_HOOK_GRAM_I8(rc_)) return rc_;
  }
  // blocks of <= kGlBlockRows rows (<= 128 ranges of <= 32768 rows: int32
  // level sums, at most 128 range partials per reduction); the first block
  // writes (or accumulates into) g, later ones accumulate
  int64_t b0 = 0;
  do {
    const int64_t nb = std::min(n - b0, kGlBlockRows);
    const float* xb = x + b0 * d;
    const int acc = accumulate || b0 > 0;
#ifndef MMB_HOOK_GRAM_I8_BLOCK  // (tools/diag: MMB_GRAM_I8_SHAPE / MMB_GRAM_DIAG)
#define MMB_HOOK_GRAM_I8_BLOCK gram_i8l_block<0, GlProduct, true>
#endif
    const int rc = MMB_HOOK_GRAM_I8_BLOCK(xb, colmax, nb, d, g, acc, part, stream);
    if (rc != MMB_OK) return rc;
    b0 += nb;
  } while (b0 < n);
  return MMB_OK;
}

extern "C" int mmb_gram_part(const float* num, const float* cnt, int64_t n, int64_t n_plan, int d,
                             int accumulate, void* ws, hipStream_t stream) {
  MMB_REQUIRE(num && ws && n >= 0 && n <= n_plan && d > 0 && gram2_ok(num, d));
  const Gram2Plan q = gram2_plan(n_plan, d);
  gram_tri_kernel<<<2 * q.R, kG2NT, gram2_lds(), stream>>>(num, cnt, n, d, q.nt, q.R, q.chunk, q.xcd,
                                                           accumulate ? 1 : 0,
                                                           static_cast<double*>(ws));
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_gram_finish(int64_t n_plan, int d, double* g, int accumulate, const void* ws,
                               hipStream_t stream) {
  MMB_REQUIRE(g && ws && n_plan >= 0 && d > 0 && d % 4 == 0 && d <= 320);
  const Gram2Plan q = gram2_plan(n_plan, d);
  {
    const int rc = launch_tri_reduce(static_cast<const double*>(ws), d, q.nt, q.R, accumulate, g, stream);
    if (rc != MMB_OK) return rc;
  }
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_xt_omega(const float* num, const float* cnt, int64_t n, int d,
                            const double* omega, int k, double* z0, hipStream_t stream) {
  MMB_REQUIRE(num && omega && z0 && n >= 0 && d > 0 && k > 0);
  // the wave kernel is for the transposed branch's small splits: at large N
  // each of its d waves would re-read all of Omega (N x k)
  if (k <= kXtK && n <= kXtMaxN && cnt)  // (the solver's k = npc + 10 <= 16)
    xt_omega_wave_kernel<float, true><<<static_cast<int>(ceil_div(d, 16)), 256, 0, stream>>>(num, cnt, n, d, omega, k, z0);
  else if (k <= kXtK && n <= kXtMaxN)
    xt_omega_wave_kernel<float><<<static_cast<int>(ceil_div(d, 16)), 256, 0, stream>>>(num, cnt, n, d, omega, k, z0);
  else
    xt_omega_kernel<float><<<static_cast<int>(ceil_div(static_cast<int64_t>(d) * k, 256)), 256, 0, stream>>>(num, cnt, n, d, omega, k, z0);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_pc_solve(const double* g, int d, const double* z0, int k, int npc, int n_iter,
                            int transposed, double* pc_out, hipStream_t stream) {
  MMB_REQUIRE(g && z0 && pc_out && d > 1 && d <= kMaxD && k >= 1 && k <= kMaxK);
  MMB_REQUIRE(npc >= 1 && npc <= k && n_iter >= 0);
  if (d <= kP16MaxD) {
    const size_t lds = p16_lds_bytes(d);
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pc_solve16_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                static_cast<int>(p16_lds_bytes(kP16MaxD)));
      attr = true;
    }
    pc_solve16_kernel<<<1, kP16NT, lds, stream>>>(g, d, z0, k, npc, n_iter, transposed, pc_out);
  } else {
    pc_solve_kernel<<<1, kSolveNT, 0, stream>>>(g, d, z0, k, npc, n_iter, transposed, pc_out);
  }
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

__global__ __launch_bounds__(256) void step_status_kernel(const int32_t* __restrict__ flag,
                                                          const double* __restrict__ pc, int n,
                                                          int32_t bit, int32_t* __restrict__ out) {
  bool bad = false;
  for (int e = threadIdx.x; e < n; e += blockDim.x) bad |= !isfinite(pc[e]);
  bad = __syncthreads_or(bad);
  if (threadIdx.x == 0) out[0] = (flag ? flag[0] : 0) | (bad ? bit : 0);
}

extern "C" int mmb_step_status(const int32_t* flag, const double* pc, int n, int32_t nonfinite_bit,
                               int32_t* out, hipStream_t stream) {
  MMB_REQUIRE(pc && out && n >= 0);
  step_status_kernel<<<1, 256, 0, stream>>>(flag, pc, n, nonfinite_bit, out);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" size_t mmb_pc_solve_mc_ws_bytes(int d) {
  const int T = (d > 0 ? d : 0) / 16 + 1;
  const size_t dd = static_cast<size_t>(d > 0 ? d : 0) * (d > 0 ? d : 0);
  // control words | tiles | G2 (r06: the squared rounds' matrix) | z0
  // (mmb_pc_solve_mc_xt: X^T Omega, d x 16)
  return 16 + static_cast<size_t>(2) * T * 512 * sizeof(double) + dd * sizeof(double) +
         static_cast<size_t>(d > 0 ? d : 0) * kP16W * sizeof(double);
}

// squared rounds for the top component only: npc = 2 lost the second
// component's last digits (3.4e-9 of the reference's g3b rows against the
// 1e-9 bar) -- G2 keeps the dominant directions to rounding, not the smaller
// ones the later components live in
static bool solve_squares(int npc, int n_iter) { return n_iter >= 3 && npc == 1; }

static int launch_solve_mc(const double* g, int d, const double* z0, int k, int npc, int n_iter,
                           int transposed, double* pc_out, void* ws, int32_t* flag, bool g2_ready,
                           hipStream_t stream);

extern "C" int mmb_pc_solve_mc(const double* g, int d, const double* z0, int k, int npc, int n_iter,
                               int transposed, double* pc_out, void* ws, int32_t* flag,
                               hipStream_t stream) {
  MMB_REQUIRE(g && z0 && pc_out && ws && d > 1 && d <= kP16MaxD && k >= 1 && k <= kP16W);
  MMB_REQUIRE(npc >= 1 && npc <= k && n_iter >= 0);
  MMB_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 15) == 0);
  return launch_solve_mc(g, d, z0, k, npc, n_iter, transposed, pc_out, ws, flag, false, stream);
}

extern "C" int mmb_pc_solve_mc_xt(const double* g, int d, const float* x, int64_t n,
                                  const double* omega, int k, int npc, int n_iter, double* pc_out,
                                  void* ws, int32_t* flag, hipStream_t stream) {
  MMB_REQUIRE(g && x && omega && pc_out && ws && d > 1 && d <= kP16MaxD && k >= 1 && k <= kP16W);
  MMB_REQUIRE(n >= 1 && n < d && n <= kXtMaxN && npc >= 1 && npc <= k && n_iter >= 0);
  MMB_REQUIRE((reinterpret_cast<uintptr_t>(ws) & 15) == 0);
  const int T = (d + 15) / 16;
  double* g2 = reinterpret_cast<double*>(static_cast<char*>(ws) + 16) + static_cast<size_t>(2) * (d / 16 + 1) * 512;
  double* z0 = g2 + static_cast<size_t>(d) * d;
  const int nsq = solve_squares(npc, n_iter) ? T * (T + 1) / 2 : 0;
  pc_prep_kernel<<<nsq + static_cast<int>(ceil_div(d, 16)), kSqNT, 0, stream>>>(
      g, d, g2, nsq, x, n, omega, k, z0);
  MMB_LAUNCH_CHECK();
  return launch_solve_mc(g, d, z0, k, npc, n_iter, 1, pc_out, ws, flag, true, stream);
}

static int launch_solve_mc(const double* g, int d, const double* z0, int k, int npc, int n_iter,
                           int transposed, double* pc_out, void* ws, int32_t* flag, bool g2_ready,
                           hipStream_t stream) {
  const int T = (d + 15) / 16;
  unsigned* ctl = static_cast<unsigned*>(ws);  // arrival counter, abort word (16-byte block)
  double* xbuf = reinterpret_cast<double*>(static_cast<char*>(ws) + 16);
  double* g2 = xbuf + static_cast<size_t>(2) * (d / 16 + 1) * 512;  // (mmb_pc_solve_mc_ws_bytes)
  // G2 ready (pc_prep_kernel) or formed by nsq_wg extra workgroups of the
  // solve's own launch, two tiles each, beside its first round (r06b: a
  // launch in front of the solve before, ~5 us on the step's critical path)
  int nsq_wg = 0;
  if (!solve_squares(npc, n_iter)) {
    g2 = nullptr;
  } else if (!g2_ready) {
    nsq_wg = (T * (T + 1) / 2 + kSqPerWg - 1) / kSqPerWg;
  }
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&pc_solve_mc_kernel<0>),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(p16_lds_bytes(kP16MaxD)));
    attr = true;
  }
  // no memset node here: the counter / abort words must be zero when the
  // caller first hands ws over, and a completed solve leaves them zero.  The
  // r04 launcher enqueued a 16-byte hipMemsetAsync of them instead; captured
  // into a HIP graph, that node wrote an address-like 64-bit value over BOTH
  // words on every replay after the first (ctl = [0x14ABxxxx, 0x7BE2]:
  // tools/dbg/replay_cause.py, r05a).  The garbage count passed every wait at
  // once, so the workgroups gathered tiles that were not yet written: a wrong
  // PC (39 of 40 replays of the solve alone) or a NaN one where the Cholesky
  // of the inconsistent block broke down (the r04e split failure), with no
  // flag.  Since r05 every arrival checks the count it finds (pm_arrive) and
  // every wait the abort word first, so a dirty workspace aborts with
  // MMB_FLAG_SYNC_TIMEOUT and a NaN PC instead
#ifndef MMB_HOOK_SOLVE_LAUNCH  // (tools/diag: MMB_PC_SOLVE_V1, the r04 kernel; MMB_PC_ABL ablations)
#define MMB_HOOK_SOLVE_LAUNCH(rc) false
#endif
  {
    int rc_ = MMB_OK;
    if (MMB_HOOK_SOLVE_LAUNCH(rc_)) return rc_;
  }
  pc_solve_mc_kernel<<<T + nsq_wg, kPnNT, p16_lds_bytes(d), stream>>>(g, g2, nsq_wg, d, z0, k, npc, n_iter,
                                                                        transposed, pc_out, xbuf, ctl, flag);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_pc_remove(const float* num, const float* cnt, int64_t n, int d,
                             const double* pc, int npc, float* out32, double* out64,
                             hipStream_t stream) {
  MMB_REQUIRE(num && pc && n >= 0 && d > 0 && npc >= 1 && ((out32 != nullptr) != (out64 != nullptr)));
  MMB_REQUIRE(static_cast<size_t>(npc) * d * sizeof(double) <= 64 * 1024);
  if (n == 0) return MMB_OK;
  const bool v4 = (d % 4 == 0) && ((reinterpret_cast<uintptr_t>(num) & 15) == 0) &&
                  (out32 == nullptr || (reinterpret_cast<uintptr_t>(out32) & 15) == 0);
  const int U = v4 ? d / 4 : d;
  const int per = static_cast<int>(ceil_div(U, kWave));
  const int rr = remove_rows();
  if (v4 && per == 2 && npc == 1 && out32 && rr > 0) {
    const int64_t waves = ceil_div(n, rr);
    const int grid = static_cast<int>(std::min<int64_t>(ceil_div(waves, 4), 256 * 8));
#ifndef MMB_HOOK_PC_REMOVE_LAUNCH  // (tools/diag: MMB_PC_REMOVE_NT / MMB_PC_REMOVE_R)
#define MMB_HOOK_PC_REMOVE_LAUNCH false
#endif
    if (!(MMB_HOOK_PC_REMOVE_LAUNCH))    {
      pc_remove1_kernel<4><<<grid, 256, 0, stream>>>(num, cnt, n, d, pc, out32);
    }
    MMB_LAUNCH_CHECK();
    return MMB_OK;
  }
  if (v4) {
    if (per <= 1) return launch_remove<4, 1>(num, cnt, n, d, pc, npc, out32, out64, stream);
    if (per <= 2) return launch_remove<4, 2>(num, cnt, n, d, pc, npc, out32, out64, stream);
    if (per <= 4) return launch_remove<4, 4>(num, cnt, n, d, pc, npc, out32, out64, stream);
    if (per <= 8) return launch_remove<4, 8>(num, cnt, n, d, pc, npc, out32, out64, stream);
  } else {
    if (per <= 2) return launch_remove<1, 2>(num, cnt, n, d, pc, npc, out32, out64, stream);
    if (per <= 4) return launch_remove<1, 4>(num, cnt, n, d, pc, npc, out32, out64, stream);
    if (per <= 8) return launch_remove<1, 8>(num, cnt, n, d, pc, npc, out32, out64, stream);
  }
  return MMB_EINVAL;
}

// ------------------------------------------------------------------ float64 X
// The numpy drop-ins (compute_pc / remove_pc) take any X; the reference runs
// randomized SVD and the removal on it in f64 (sif_functions.py:58-81).  X
// that is not f32-representable takes these entry points instead of being
// rounded: the generic 64x64-block fp64-MFMA Gram, X^T Omega, and the f64
// removal, all reading the f64 rows.
extern "C" int mmb_gram_f64(const double* x, int64_t n, int d, double* g, int accumulate, void* ws,
                            hipStream_t stream) {
  MMB_REQUIRE(x && g && ws && n >= 0 && d > 0);
  const GramPlan p = gram_plan(n, d);
  const int64_t total = static_cast<int64_t>(d) * d;
  double* part = static_cast<double*>(ws);
  gram_partial_kernel<double><<<p.npairs * p.S, 256, 0, stream>>>(x, nullptr, n, d, p.nb, p.npairs,
                                                                  p.S, p.chunk, p.xcd, part);
  MMB_LAUNCH_CHECK();
  gram_reduce_kernel<<<static_cast<int>(ceil_div(total, 256)), 256, 0, stream>>>(part, d, p.nb, p.npairs, p.S, accumulate, g);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_xt_omega_f64(const double* x, int64_t n, int d, const double* omega, int k,
                                double* z0, hipStream_t stream) {
  MMB_REQUIRE(x && omega && z0 && n >= 0 && d > 0 && k > 0);
  if (k <= kXtK && n <= kXtMaxN)
    xt_omega_wave_kernel<double><<<static_cast<int>(ceil_div(d, 16)), 256, 0, stream>>>(x, nullptr, n, d, omega, k, z0);
  else
    xt_omega_kernel<double><<<static_cast<int>(ceil_div(static_cast<int64_t>(d) * k, 256)), 256, 0, stream>>>(
        x, nullptr, n, d, omega, k, z0);
  MMB_LAUNCH_CHECK();
  return MMB_OK;
}

extern "C" int mmb_pc_remove_f64(const double* x, int64_t n, int d, const double* pc, int npc,
                                 double* out64, hipStream_t stream) {
  MMB_REQUIRE(x && pc && out64 && n >= 0 && d > 0 && npc >= 1);
  MMB_REQUIRE(static_cast<size_t>(npc) * d * sizeof(double) <= 64 * 1024);
  if (n == 0) return MMB_OK;
  const int per = static_cast<int>(ceil_div(d, kWave));
  if (per <= 2) return launch_remove<1, 2, double>(x, nullptr, n, d, pc, npc, nullptr, out64, stream);
  if (per <= 4) return launch_remove<1, 4, double>(x, nullptr, n, d, pc, npc, nullptr, out64, stream);
  if (per <= 8) return launch_remove<1, 8, double>(x, nullptr, n, d, pc, npc, nullptr, out64, stream);
  return MMB_EINVAL;
}

// the tools build's variant kernels, launches, knobs and entry points
// (tools/diag/); the product library includes an empty header here
#ifndef MMB_TOOLS_TAIL_PC
#define MMB_TOOLS_TAIL_PC "mmb_no_tools.h"
#endif
#include MMB_TOOLS_TAIL_PC
