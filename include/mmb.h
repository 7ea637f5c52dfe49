/*
 * mmb.h — C ABI of libmmb.so, the MI355X (gfx950) SIF / MMB2 / regressor hot path.
 *
 * The reference (yaochie/multimodal-baselines) has no FFI: its boundary is a set
 * of Python functions on numpy arrays / torch tensors.  Each entry point below
 * replaces the arithmetic of one of those functions; the Python mirror in
 * `multimodal-baselines_amd/` keeps the reference names and signatures and
 * calls these through ctypes.
 *
 * Conventions:
 *   - every pointer argument except host_* is DEVICE memory allocated by the
 *     caller; the library never allocates or frees caller memory;
 *   - all work is enqueued on `stream` and is asynchronous; no entry point
 *     synchronises, so the calls can be captured into a hipGraph;
 *   - row-major, contiguous layouts; ids are int32 (the caller narrows the
 *     reference's int64 ids after a range check);
 *   - return 0 on success, MMB_EINVAL (<0) on a bad argument or shape, or a
 *     positive hipError_t from the launch;
 *   - `flag` (nullable) is an int32 device word OR-ed with MMB_FLAG_* bits by
 *     kernels that meet out-of-range ids (the shim raises IndexError, like
 *     numpy would in the reference) or all-zero-weight utterances (the shim
 *     raises ValueError where the reference's PC step would).
 */
#ifndef MMB_H_
#define MMB_H_

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMB_OK 0
#define MMB_EINVAL (-1)
#define MMB_FLAG_ID_RANGE 1
/* an utterance whose SIF weights are all 0 (its a2 row is 0/0 = NaN, like
 * numpy's; the reference's TruncatedSVD then raises ValueError on the split) */
#define MMB_FLAG_ZERO_WEIGHTS 2
/* mmb_mm2_stream_project: a hand-over between its streaming and projecting
 * waves waited ~0.5 s without progress (a bug, never expected); the kernel
 * then ends at once and its MMB2 rows are invalid */
#define MMB_FLAG_SYNC_TIMEOUT 4

/* Library version (major*10000 + minor*100 + patch). */
int mmb_version(void);

/* ---------------------------------------------------------------- a1
 * seq2weight: w[i,j] = f32(wtab64[seq[i,j]]) if sel[i,j] (nullable = all) and
 * seq[i,j] >= 0, else 0.  Bit-exact with the reference.
 * replaces: sif_functions.seq2weight   /root/reference/sif_functions.py:8-15
 *           sif.get_sentence_word_weights /root/reference/sif.py:78-82      */
int mmb_seq2weight(const int32_t* seq, const uint8_t* sel, int64_t n, int64_t l,
                   const double* wtab64, int64_t v, float* w_out, int32_t* flag,
                   hipStream_t stream);

/* ---------------------------------------------------------------- a1+a2
 * Weighted average of gathered table rows per utterance:
 *   num[i] = sum_j w[i,j] * table[ids[i,j]],  cnt[i] = count_nonzero(w[i,:]),
 *   x[i]   = num[i] / cnt[i]                       (all float32)
 * Weights come from `w` [n,l] when non-null (get_weighted_average), else from
 * the f32 table `wtab32` gathered by id with id<0 -> 0 (a1 fused).
 * Negative ids wrap like numpy (table[v+id]).  Outputs x/num/cnt are each
 * nullable (at least one required).
 * replaces: sif_functions.get_weighted_average /root/reference/sif_functions.py:28-56 */
int mmb_sif_wavg(const float* table, int64_t v, int d, const int32_t* ids, int64_t n, int l,
                 const float* w, const float* wtab32, float* x_out, float* num_out,
                 float* cnt_out, int32_t* flag, hipStream_t stream);

/* ---------------------------------------------------------------- a3 (Gram)
 * g[d,d] (float64, full symmetric) = sum_i x_i x_i^T with x_i = num[i]/cnt[i]
 * (cnt nullable -> x = num).  Products of f32 values are exact in f64 (fp64
 * MFMA).  `ws` is scratch of mmb_gram_workspace_bytes(n, d) bytes.
 * If accumulate != 0 the result is added to g (multi-split use).            */
size_t mmb_gram_workspace_bytes(int64_t n, int d);
int mmb_gram(const float* num, const float* cnt, int64_t n, int d, double* g, int accumulate,
             void* ws, hipStream_t stream);

/* The same Gram in two phases, for a split streamed in row chunks (the
 * overlapped bench step): mmb_gram_part reduces one chunk of n <= n_plan rows
 * into per-range partials in ws (accumulate = 0 for the first chunk, 1 to add
 * the next ones; every chunk must use the same n_plan, and consecutive calls
 * must be stream-ordered); mmb_gram_finish sums the partials in a fixed order
 * into g (accumulate: add to g).  ws as for mmb_gram(n_plan, d); d % 4 == 0,
 * d <= 320, num 16-byte aligned.                                             */
int mmb_gram_part(const float* num, const float* cnt, int64_t n, int64_t n_plan, int d,
                  int accumulate, void* ws, hipStream_t stream);
int mmb_gram_finish(int64_t n_plan, int d, double* g, int accumulate, const void* ws,
                    hipStream_t stream);

/* The same Gram on the int8 matrix pipe, for x rows (cnt = 1) whose column
 * bounds colmax[j] = max_i |x[i,j]| (float bits) are known: every value as a
 * 30-bit fixed-point integer of its column's power-of-two bound, cut into
 * four int8 digits; digit-pair products of level <= 4 summed exactly (int32
 * per 64-row step, then f64).  Not bit-equal to mmb_gram: ~1e-10 relative
 * (the PC within 6e-11 of the reference's on the golden splits).  d % 4 == 0,
 * d <= 304; ws as for mmb_gram_workspace_bytes(n, d).  mmb_colmax computes
 * the bounds (accumulate = 0 zeroes colmax first).
 * replaces: the X^T X inside sif_functions.compute_pc's TruncatedSVD
 *   /root/reference/sif_functions.py:58-67                                   */
int mmb_colmax(const float* x, int64_t n, int d, uint32_t* colmax, int accumulate,
               hipStream_t stream);
int mmb_gram_i8(const float* x, const uint32_t* colmax, int64_t n, int d, double* g,
                int accumulate, void* ws, hipStream_t stream);

/* z0[d,k] = X^T omega  (omega [n,k] float64) — start block of the transposed
 * randomized-SVD branch (n < d).                                             */
int mmb_xt_omega(const float* num, const float* cnt, int64_t n, int d, const double* omega,
                 int k, double* z0, hipStream_t stream);

/* ---------------------------------------------------------------- a3 (solve)
 * Top-npc right singular vectors of X exactly as scikit-learn's
 * TruncatedSVD(npc, n_iter, random_state=0) (randomized_svd, k = npc+10
 * oversampled block, LU-normalised power iterations, svd_flip on components)
 * computes them, evaluated from the Gram g alone: span(G^n_iter Z0) is the
 * subspace the reference's iterations build, and the final SVD of Q^T X is
 * solved as a k x k (generalised) symmetric eigenproblem.  One workgroup, fp64.
 *   transposed = (n_total < d): z0 = X^T Omega_n, else z0 = Omega_d [d,k].
 * pc_out [npc, d] float64.  d <= 512, k <= 16.
 * replaces: sif_functions.compute_pc /root/reference/sif_functions.py:58-67 */
int mmb_pc_solve(const double* g, int d, const double* z0, int k, int npc, int n_iter,
                 int transposed, double* pc_out, hipStream_t stream);

/* The same solve on ceil(d/16) workgroups (d <= 320, k <= 16): each keeps
 * 16 rows of G in registers, the tiles of every power-iteration product are
 * exchanged in-launch (write-through stores + an arrival counter), and every
 * workgroup runs the identical CholeskyQR; workgroup 0 runs the final
 * Rayleigh-Ritz step.  ws: mmb_pc_solve_mc_ws_bytes(d) bytes, 16-byte
 * aligned, owned by the call until it completes; its first 16 bytes (arrival
 * counter, abort word) must be ZERO when the caller first hands it over, and
 * a completed solve leaves them zero -- no memset is enqueued, so the call is
 * safe to capture into a graph and replay.  A workgroup that waits ~1 s for
 * the others gives up and sets MMB_FLAG_SYNC_TIMEOUT in *flag (nullable);
 * so does a launch that finds the words dirty (an abort word left set, or an
 * arrival count outside the round's range); pc_out is then NaN and ws must
 * be re-zeroed before the next call.
 * replaces: sif_functions.compute_pc /root/reference/sif_functions.py:58-67 */
/* The step's status word in one launch: out[0] = flag[0] | (nonfinite_bit if
 * any of the n values of pc is not finite), flag nullable (0).  What a
 * checked step (pipeline.FusedStep.status) reads back with one sync; the
 * eight elementwise torch kernels it replaced were ~40 us of every dataset
 * split's graph (r06 kernel trace).  A host-side helper of the drop-in's
 * error behaviour (sif_functions.py:65-67: TruncatedSVD rejects NaN).     */
int mmb_step_status(const int32_t* flag, const double* pc, int n, int32_t nonfinite_bit,
                    int32_t* out, hipStream_t stream);

/* (r06) the multi-workgroup solve runs (n_iter - 1) / 2 of its products by
 * G2 = G G (npc = 1, n_iter >= 3; the first product is by G, and extra
 * workgroups of the same launch form G2 beside it): ws holds G2 too, so
 * mmb_pc_solve_mc_ws_bytes grew by d * d * 8 bytes (an ABI change: size ws
 * with this call), and the third control word counts the squaring
 * workgroups (the first 16 bytes are still the block a caller re-zeroes
 * after MMB_FLAG_SYNC_TIMEOUT).                                             */
size_t mmb_pc_solve_mc_ws_bytes(int d);
/* The transposed branch (n < d) of mmb_pc_solve_mc from the rows themselves:
 * z0 = X^T omega [n, k] (x f32 [n, d], the a2 rows) and G2 formed in ONE
 * launch into ws (which holds both; mmb_pc_solve_mc_ws_bytes), then the
 * solve -- where mmb_xt_omega + mmb_pc_solve_mc took two launches before
 * it.  The same z0 (the same per-lane sums) and PC.
 * replaces: sif_functions.compute_pc for a split of n < d rows
 *   /root/reference/sif_functions.py:58-67 (sklearn extmath.py:562-566)    */
int mmb_pc_solve_mc_xt(const double* g, int d, const float* x, int64_t n, const double* omega,
                       int k, int npc, int n_iter, double* pc_out, void* ws, int32_t* flag,
                       hipStream_t stream);
int mmb_pc_solve_mc(const double* g, int d, const double* z0, int k, int npc, int n_iter,
                    int transposed, double* pc_out, void* ws, int32_t* flag, hipStream_t stream);

/* ---------------------------------------------------------------- a4
 * out[i] = x_i - sum_c (x_i . pc_c) pc_c   in float64, x_i = num[i]/cnt[i]
 * (cnt nullable).  Exactly one of out32 / out64 non-null.
 * replaces: sif_functions.remove_pc /root/reference/sif_functions.py:69-81 */
int mmb_pc_remove(const float* num, const float* cnt, int64_t n, int d, const double* pc,
                  int npc, float* out32, double* out64, hipStream_t stream);

/* float64 X (the numpy drop-ins' general input, when it is not
 * f32-representable): the same Gram (fp64 MFMA, 64x64 blocks), start block
 * X^T Omega and f64 removal reading f64 rows, so compute_pc / remove_pc do not
 * round X to f32 first.  ws as for mmb_gram_workspace_bytes(n, d).
 * replaces: sif_functions.compute_pc / remove_pc on float64 input
 *   /root/reference/sif_functions.py:58-81                                   */
int mmb_gram_f64(const double* x, int64_t n, int d, double* g, int accumulate, void* ws,
                 hipStream_t stream);
int mmb_xt_omega_f64(const double* x, int64_t n, int d, const double* omega, int k, double* z0,
                     hipStream_t stream);
int mmb_pc_remove_f64(const double* x, int64_t n, int d, const double* pc, int npc,
                      double* out64, hipStream_t stream);

/* Streams restricted to a subset of the CUs (hipExtStreamCreateWithCUMask):
 * bit i of cu_mask[i / 32] enables CU i.  Used to run the HBM-bound stream
 * kernel and the MFMA-bound projection side by side on disjoint CUs.
 * mmb_cu_count writes the device's CU count.  No reference counterpart
 * (scheduling only).                                                         */
int mmb_cu_count(int device, int* out);

/* Bandwidth probes (measurement only, no reference counterpart): the
 * same-process HBM ceilings the bench quotes beside the 8 TB/s spec (SURVEY.md
 * §8d "a measured stream-copy ceiling").  16-byte words (nt != 0: non-temporal
 * loads / stores), four loads in flight per lane, a grid of min(blocks,
 * bytes / 4 KB) 256-thread workgroups.  mmb_probe_copy: dst = src (2 * bytes moved).  mmb_probe_read:
 * reads src once and writes one word per workgroup into sink[blocks].
 * bytes and both pointers must be 16-byte aligned.                           */
int mmb_probe_copy(const void* src, void* dst, int64_t bytes, int blocks, int nt,
                   hipStream_t stream);
int mmb_probe_read(const void* src, int64_t bytes, int blocks, int nt, uint32_t* sink,
                   hipStream_t stream);
int mmb_stream_create_cu_mask(const uint32_t* cu_mask, int mask_words, hipStream_t* out);
int mmb_stream_destroy(hipStream_t stream);

/* Host helper: numpy RandomState(seed).normal(size=count) (MT19937 +
 * legacy polar Box-Muller), written to host memory.  Used for the
 * randomized-SVD start block Omega.                                          */
int mmb_host_randn(uint32_t seed, int64_t count, double* host_out);

/* ---------------------------------------------------------------- a7
 * q_mean = (x-b)/exp(2 ls), q_sigma = (x-b)^2/exp(2 ls) - 1 over [n*t, f].
 * replaces: sif2.calc_weights /root/reference/sif2.py:103-114               */
int mmb_calc_weights(const float* x, int64_t rows, int f, const float* b_mean,
                     const float* b_log_sigma, float* q_mean, float* q_sigma, hipStream_t stream);

/* ---------------------------------------------------------------- a6+a7+a8 (stream)
 * One pass over every utterance's text tokens and audio/visual frames.
 * Text rows come from the table by id (ids non-null; wtab32 gives the weights)
 * or from dense [n,t,d] tensors (ids null: text_dense for the modality sums,
 * emb_dense for the weighted sum, w_dense [n,t] the sentence weights).
 * Writes, per utterance i:
 *   num[i,:d]  = (sum_t w_t E_t) / count_nonzero(w)  (the a2 row x_i, f32
 *                division as sif_functions.py:55; NaN when every weight is 0)
 *   s[i,:]     = [Sx_e | Sxx_e | Sx_a | Sxx_a | Sx_v | Sxx_v | 0-pad]  (sum
 *                over t of x and x^2 per feature; row stride mmb_mm2_k());
 *                s_half = 0: fp32 [n][k]; s_half = 1: fp16 [n][2][k], the hi
 *                and lo (residual) planes of s[i,:] * aux[2][i] -- the A
 *                operand of mmb_mm2_project_x3 (same bytes per row)
 *   aux[0][i]  = count_nonzero(w), aux[1][i] = sum_t w_t, aux[2][i] = the
 *                power-of-2 scale putting max|s[i,:]| in [2^14, 2^15) (planar
 *                [3][n]; aux[0] is the SIF count the Gram / removal kernels take)
 * replaces the frame loops of sif2.estimate_embedding_overall_gpu2
 *   /root/reference/sif2.py:181-205 and the gathers at simplesif.py:862-871 */
int mmb_mm2_stream(const int32_t* ids, const float* table, int64_t v, const float* wtab32,
                   const float* text_dense, const float* emb_dense, const float* w_dense,
                   const float* audio, const float* visual, int64_t n, int t, int d, int a,
                   int vd, float* num_out, void* s_out, int s_half, float* aux_out,
                   int32_t* flag, uint32_t* colmax, void* colmax_ws, hipStream_t stream);

/* mmb_mm2_stream for a few long rows (POM's splits: 100 / 203 transcripts of
 * 1089 / 1357 tokens), split over workgroups: every utterance is cut into P
 * token / frame ranges (parts = 0: mmb_mm2_stream_split_parts, about one
 * workgroup per CU in all; parts > 0: that many, at most t), each range
 * summed by a text, an audio and a visual workgroup of its own whose
 * partial sums go to ws (mmb_mm2_stream_split_ws_bytes(n, t, d, a, vd, parts) bytes,
 * caller-owned scratch), and a second kernel adds an utterance's partials in
 * fixed part order and writes the same outputs as mmb_mm2_stream (x, s in
 * the s_half format asked for, aux, colmax; n <= 8192 with colmax).  Rows are
 * deterministic and equal mmb_mm2_stream's to the f32 order of the token and
 * frame sums.
 * replaces: the frame loops of sif2.estimate_embedding_overall_gpu2
 *   /root/reference/sif2.py:181-205 at the per-split call sites
 *   /root/reference/simplesif.py:308-311 (POM's long transcripts)          */
int mmb_mm2_stream_split_parts(int64_t n, int t);
size_t mmb_mm2_stream_split_ws_bytes(int64_t n, int t, int d, int a, int vd, int parts);
int mmb_mm2_stream_split(const int32_t* ids, const float* table, int64_t v, const float* wtab32,
                         const float* text_dense, const float* emb_dense, const float* w_dense,
                         const float* audio, const float* visual, int64_t n, int t, int d, int a,
                         int vd, float* num_out, void* s_out, int s_half, float* aux_out,
                         int32_t* flag, uint32_t* colmax, void* colmax_ws, int parts, void* ws,
                         size_t ws_bytes, hipStream_t stream);

/* mmb_mm2_stream and mmb_mm2_project_x3 in ONE kernel (the bench step's
 * MMB2 path): the same num (x), aux[0..1] and colmax outputs as mmb_mm2_stream
 * (aux[2] is the text piece's scale) and the MMB2 rows of mmb_mm2_project_x3
 * (same fp16 x3 products; within f32 rounding of its sum order), but the
 * per-utterance sums s never reach HBM: each workgroup's streaming waves
 * stream a batch of 48 utterances modality by modality and leave each
 * (utterance, modality) piece of sums in an LDS ring, its projecting waves
 * multiply each piece of the batch with the piece-ordered fp16 hi/lo split
 * of wm (wpieces from mmb_mm2_split_pieces; c0 from mmb_mm2_prepare).  Text
 * by ids (table, wtab32 or w_dense) or dense (text_dense with w_dense, the
 * weighted sum over the same rows).  Shapes: mmb_mm2_stream_project_supported
 * (t <= 64, 256 <= d < 320, a and vd <= 320, widths % 4); 16-byte aligned
 * rows.  MMB_EINVAL otherwise.
 * replaces: the frame loops and projections of sif2.estimate_embedding_overall_gpu2
 *   /root/reference/sif2.py:181-207 and the gathers at simplesif.py:862-871 */
int mmb_mm2_stream_project_supported(int t, int d, int a, int vd);
int mmb_mm2_stream_project(const int32_t* ids, const float* table, int64_t v,
                           const float* wtab32, const float* text_dense, const float* w_dense,
                           const float* audio, const float* visual, int64_t n, int t, int d,
                           int a, int vd, const void* wpieces, const float* c0, float* num_out,
                           float* aux_out, float* mmb2_out, int32_t* flag, uint32_t* colmax,
                           void* colmax_ws, hipStream_t stream);

/* mmb_mm2_project_x3_rmpc for a few rows (the dataset splits: 100-1,284
 * rows put one or a few workgroups through the whole K loop), split over K:
 * slices (0: mmb_mm2_project_x3_split_slices) workgroups per 128-row tile
 * each run a contiguous range of the 32-deep K chunks and write their raw
 * accumulators to ws (mmb_mm2_project_x3_split_ws_bytes(n, k, slices) bytes,
 * 16-byte aligned scratch), then one launch sums each tile's slices in slice
 * order and runs the same row-wise epilogue (ldw = 320, 256 <= d < 320;
 * other shapes, or one slice, take mmb_mm2_project_x3_rmpc unchanged).  MMB2
 * and PC-removed rows equal the one-pass kernel's to the f32 order of the K
 * sum.
 * replaces: the projections of sif2.estimate_embedding_overall_gpu2
 *   /root/reference/sif2.py:187-207 at the per-split call sites
 *   /root/reference/simplesif.py:308-311                                   */
int mmb_mm2_project_x3_split_slices(int64_t n, int k);
size_t mmb_mm2_project_x3_split_ws_bytes(int64_t n, int k, int slices);
int mmb_mm2_project_x3_split(const void* s_split, const float* num, const float* aux,
                             const void* wsplit, int ldw, const float* c0, int64_t n, int k, int d,
                             float* out, const double* pc, float* sif_out, int slices, void* ws,
                             size_t ws_bytes, hipStream_t stream);

/* The fp16 hi/lo split of wm [k, ldw] (mmb_mm2_prepare) in piece order for
 * mmb_mm2_stream_project: each modality's 2 w_m rows [Sx_m | Sxx_m] padded
 * to a multiple of 32, chunks and column scales as mmb_mm2_split_bytes'
 * image, then the per-column 1/scale [ldw] f32.                             */
size_t mmb_mm2_split_pieces_bytes(int d, int a, int vd);
int mmb_mm2_split_pieces(const float* wm, int d, int a, int vd, int ldw, void* img,
                         hipStream_t stream);

/* colmax (nullable; d <= 640): the column bounds max_i |num[i,:]| of the a2
 * rows as float bits, the input of mmb_gram_i8 -- a by-product of the stream
 * kernel (per-wave running maxima into colmax_ws, then one fixed-order reduce
 * launch) instead of a second pass over x.  colmax_ws: scratch of
 * mmb_mm2_colmax_ws_bytes(d) bytes (its last 16 bytes: the batch counter of
 * mmb_mm2_stream_project's dynamic batch order, zeroed by that call itself;
 * one launch at a time per workspace).  ABI note (r05): the size grew by those
 * 16 bytes; a workspace sized by hand from the r04 formula (8192 x d floats)
 * is too small and nothing can check it -- always size it with this call.   */
size_t mmb_mm2_colmax_ws_bytes(int d);

/* Padded width (row stride) of the per-utterance sums: roundup(2(d+a+vd), 32). */
int mmb_mm2_k(int d, int a, int vd);

/* Leading dimension of the merged projection: roundup(d+1, 64). */
int mmb_mm2_ldw(int d);

/* Merge the 6 combinations' (W_mu, b_mu, W_log_sigma, b_log_sigma) into
 * wm [k, ldw] (ldw >= d+1; column d carries the total-weight row) and
 * c0 [ldw] for frame count t.  Pointer arrays are HOST arrays of DEVICE
 * pointers in key order audio, visual, audiovisual, textaudio, textvisual,
 * textaudiovisual (sif2.py:167-174).                                         */
int mmb_mm2_prepare(const float* const* w_mu, const float* const* b_mu,
                    const float* const* w_ls, const float* const* b_ls, int d, int a, int vd,
                    int t, float* wm, int ldw, float* c0, void* wsplit, hipStream_t stream);

/* Bytes of the fp16 hi/lo split of wm written by mmb_mm2_prepare when wsplit
 * is non-null: per 32-deep K chunk, the hi and lo planes [ldw][32] of the
 * column-scaled wm (16-byte slots swizzled as mmb_mm2_project_x3 stages
 * them), then the per-column 1/scale [ldw] f32.                             */
size_t mmb_mm2_split_bytes(int d, int a, int vd);

/* cs = (t + s @ wm[:, :d] + c0) / (aux[1] + s @ wm[:, d] + c0[d]) with the
 * weighted text sum t = num * aux[0] (0 where aux[0] == 0), num as
 * mmb_mm2_stream writes it; out = cs / ||cs||_2 (fp32 MFMA GEMM + fused
 * epilogue).
 * replaces: sif2.py:186-207                                                  */
int mmb_mm2_project(const float* s, const float* num, const float* aux, const float* wm,
                    int ldw, const float* c0, int64_t n, int k, int d, float* out,
                    hipStream_t stream);

/* The same projection on the fp16 MFMA pipe: s (scaled per row by aux[2]) and
 * wm (scaled per column) split into fp16 hi + lo, a*b ~ ah*bh + ah*bl + al*bh
 * (3 f16 MFMAs, ~22-bit operands, fp32 accumulation).  s_split is the
 * s_half = 1 output of mmb_mm2_stream, wsplit from mmb_mm2_prepare; d < 320.
 * The bench path.                                                            */
int mmb_mm2_project_x3(const void* s_split, const float* num, const float* aux, const void* wsplit,
                       int ldw, const float* c0, int64_t n, int k, int d, float* out,
                       hipStream_t stream);

/* mmb_mm2_project_x3 with the first-PC removal of the a2 rows fused into its
 * epilogue (npc = 1): sif_out[i,:] = num[i,:] - (num[i,:] . pc) pc in f64,
 * rounded to f32 -- what mmb_pc_remove(num, NULL, n, d, pc, 1, sif_out, NULL)
 * writes, without re-reading num.  pc and sif_out both null = plain x3.
 * replaces: sif2.py:186-207 and sif_functions.remove_pc
 *   /root/reference/sif_functions.py:69-81 (npc = 1 branch :77-78)           */
int mmb_mm2_project_x3_rmpc(const void* s_split, const float* num, const float* aux,
                            const void* wsplit, int ldw, const float* c0, int64_t n, int k, int d,
                            float* out, const double* pc, float* sif_out, hipStream_t stream);

/* MMB2 at narrow frame widths (MOSI) in ONE kernel, a1-a8's stream and the
 * projection fused: the text rows of the merged projection are applied per
 * vocabulary row (text cache: P[v] = E_v Wm_t1 + E_v^2 Wm_t2, f64 rounded
 * once; the 32 words of smallest SIF weight kept in LDS), so only the
 * audio / visual frame sums (K = kq(A) + kq(Vd) <= 256) meet the f16 x3 MFMA,
 * inside the same launch; the frame sums never reach HBM.  Writes x (the a2
 * rows: mmb_mm2_stream's sums in another order -- hot words first -- so
 * equal to f32 rounding), aux, the MMB2 rows and (colmax non-null) the
 * column bounds of x for mmb_gram_i8.
 *   mmb_mm2_text_cache: cache of mmb_mm2_text_cache_bytes(v, d) bytes (16-B
 *   aligned) from the word table, the f32 weight table and the merged Wm
 *   (mmb_mm2_prepare); rebuild it when any of them changes (the launch reads
 *   the token weights from the cache's copy of wtab32).  v <= 16384.
 *   wpieces: the piece-ordered weight split (mmb_mm2_split_pieces).
 * replaces: sif2.calc_weights + estimate_embedding_overall_gpu2
 *   /root/reference/sif2.py:103-114,164-208 with the text gather of
 *   /root/reference/simplesif.py:862-871 and sif_functions.py:28-56      */
size_t mmb_mm2_text_cache_bytes(int64_t v, int d);
int mmb_mm2_text_cache(const float* table, int64_t v, int d, const float* wtab32, const float* wm,
                       int ldw, void* cache, hipStream_t stream);
int mmb_mm2_stream_project_narrow_supported(int t, int d, int a, int vd, int64_t v);
int mmb_mm2_stream_project_narrow(const int32_t* ids, const float* table, int64_t v,
                                  const float* wtab32, const void* text_cache, const float* audio,
                                  const float* visual, int64_t n, int t, int d, int a, int vd,
                                  const void* wpieces, const float* c0, float* num_out,
                                  float* aux_out, float* mmb2_out, int32_t* flag, uint32_t* colmax,
                                  void* colmax_ws, hipStream_t stream);

/* ---------------------------------------------------------------- a10/a11
 * SentimentModel(d -> h -> o): y = squeeze(W2 relu(W1 x + b1) + b2).
 * Forward for rows idx[0..b) (idx nullable = 0..b) of latents [*, d].
 * replaces: sentiment_model.SentimentModel.forward /root/reference/sentiment_model.py:36-41 */
int mmb_mlp_forward(const float* latents, const int64_t* idx, int64_t b, int d, int h, int o,
                    const float* w1, const float* b1, const float* w2, const float* b2,
                    float* y_out, hipStream_t stream);

/* Differentiable forward / backward of the same model, for the e2e joint
 * objective whose regressor term backpropagates into the latents
 * (simplesif.py:776-790, autograd of sentiment_model.py:36-41):
 *   forward_train: y [b,o] and the post-ReLU hidden activations hid [b,h];
 *   backward: dh_ws [b,h] scratch, dx [b,d] (nullable), dw1 [h,d], db1 [h],
 *   dw2 [o,h], db2 [o] (each nullable) for upstream gradient dy [b,o].
 * Parameter gradients reduce over the rows in a fixed order.                 */
int mmb_mlp_forward_train(const float* x, int64_t b, int d, int h, int o, const float* w1,
                          const float* b1, const float* w2, const float* b2, float* y_out,
                          float* hid_out, hipStream_t stream);
int mmb_mlp_backward(const float* x, const float* hid, int64_t b, int d, int h, int o,
                     const float* w1, const float* w2, const float* dy, float* dh_ws, float* dx,
                     float* dw1, float* db1, float* dw2, float* db2, hipStream_t stream);

/* L1 loss sum for prediction rows vs labels (per-batch means written to
 * batch_loss): the evaluation loops of sentiment_model.py:60-74,117-125.
 * Batches are consecutive slices of `perm` of size batch (last one ragged). */
int mmb_mlp_eval(const float* latents, const float* labels, const int64_t* perm, int64_t n,
                 int batch, int d, int h, int o, const float* w1, const float* b1,
                 const float* w2, const float* b2, float* batch_loss, float* pred_out,
                 hipStream_t stream);

/* SGD training of the regressor over n_epochs epochs of mini-batches drawn
 * from `perm` (the DataLoader order: epochs concatenated, batches of `batch`
 * rows, the last one ragged), with loss = L1(reduction='none').mean() and
 * p -= lr * grad, all in ONE launch of ceil(h / 32) workgroups (one 32-wide
 * hidden tile each, exchanging their output shares once per mini-batch).
 * Parameters are updated in place; per-step losses go to step_loss
 * [n_epochs * ceil(n_per_epoch / batch)].  With v_latents non-null the
 * launch also runs the validation passes: after every epoch e with
 * (epoch0 + e) % valid_every == 0 the per-batch mean L1 of the validation rows
 * v_perm[k * n_valid ...] (k = the k-th such epoch of this launch) with the
 * weights of that moment go to valid_loss[k * ceil(n_valid / batch) + j].
 * ws: scratch of mmb_mlp_workspace_bytes(d, h) bytes (16-B aligned), ZEROED
 * by the caller before its first use (a completed launch leaves it zeroed);
 * flag (nullable) gets MMB_FLAG_SYNC_TIMEOUT if the workgroups' exchange
 * stalls (~1 s) or finds ws dirty (the parameters are then invalid and ws
 * must be re-zeroed).  The P = ceil(h / 32) workgroups are launched
 * cooperatively (co-resident, or the launch fails) after an occupancy check
 * (MMB_EINVAL when the device cannot hold them at once).  d % 4 == 0, d <= 512, h <= 512,
 * n_out <= 16.
 * replaces: sentiment_model.train_sentiment loop incl. its validation passes
 *   /root/reference/sentiment_model.py:76-127                               */
size_t mmb_mlp_workspace_bytes(int d, int h);
int mmb_mlp_train(const float* latents, const float* labels, const int64_t* perm,
                  int64_t n_per_epoch, int n_epochs, int batch, int d, int h, int o, float lr,
                  float* w1, float* b1, float* w2, float* b2, float* step_loss,
                  const float* v_latents, const float* v_labels, const int64_t* v_perm,
                  int64_t n_valid, int valid_every, int epoch0, float* valid_loss, void* ws,
                  int32_t* flag, hipStream_t stream);

/* ---------------------------------------------------------------- §8f row 1
 * Latent-optimisation likelihoods (the objective simplesif.py:49-162,708-806
 * minimises).  Word term = get_word_log_prob_angular2, losses.py:68-95;
 * Gaussian term = get_normal_log_prob, losses.py:13-33, summed per modality
 * combination by get_log_prob_matrix, losses.py:216-274.
 *
 * mmb_word_normalize: wn [v, mmb_word_pad(d)] = table / max(|row|, 1e-8),
 * zero padded (torch cosine_similarity's x2 / |x2|; done once per table).   */
int mmb_word_pad(int d);
int mmb_word_normalize(const float* table, int64_t v, int d, float* wn, hipStream_t stream);

/* lp[b] = sum_t mask[b,t] log(alpha_b w[b,t] + (1-alpha_b) score_bt / Z_b),
 * Z_b = sum_{v<V} (1 - acos(cos(l_b, table_v))/pi), alpha_b = 1/(a Z_b + 1),
 * score_bt = 1 - acos(cos(l_b, e_bt))/pi, e_bt = table[ids[b,t]] (ids non-null)
 * or sent_dense[b,t,:].  d <= 320 for the MFMA Z kernel.  ws: scratch of
 * mmb_word_workspace_bytes(b, d, v).  With want_grad, state [b,4], gsum
 * [b, pad(d)] and cos_out [b, l] are written for mmb_word_logprob_backward.
 * replaces: losses.get_word_log_prob_angular2 /root/reference/losses.py:68-95
 *           (and get_word_log_prob_angular :36-66 with w = weights[data])  */
size_t mmb_word_workspace_bytes(int64_t b, int d, int64_t v);
int mmb_word_logprob_forward(const float* latents, int64_t b, int d, const float* wn, int64_t v,
                             const int32_t* ids, const float* table, const float* sent_dense,
                             int l, const float* w, const float* mask, float a, int want_grad,
                             void* ws, float* lp, float* state, float* gsum, float* cos_out,
                             hipStream_t stream);
/* dlat[b,:] = dlp[b] * d lp_b / d latents[b,:] (autograd of losses.py:68-95). */
int mmb_word_logprob_backward(const float* latents, int64_t b, int d, int64_t v,
                              const int32_t* ids, const float* table, const float* sent_dense,
                              int l, const float* w, const float* mask, float a,
                              const float* state, const float* gsum, const float* cosv,
                              const float* dlp, float* dlat, hipStream_t stream);

/* stats [n][3][f] f64 = per-utterance masked frame sums (sum_t m, sum_t m x,
 * sum_t m x^2) of x [n,t,f] (mask nullable = ones); streamed once per split. */
int mmb_gauss_stats(const float* x, const float* mask, int64_t n, int t, int f, double* stats,
                    hipStream_t stream);
/* lp[k][b] = get_normal_log_prob(mu_k[b], sigma_k[b], x, mask) for combination
 * k of modalities mods[k] (bit 0 text, 1 audio, 2 visual; features in that
 * torch.cat order), from the stats of rows idx[b] (idx nullable = b).
 * stats[3] / fm[3] / mods / mu / sigma are HOST arrays (of device pointers).
 * replaces: losses.get_normal_log_prob /root/reference/losses.py:13-33 and the
 *           per-modality loop of get_log_prob_matrix :249-256               */
int mmb_gauss_loglik(const double* const* stats, const int* fm, const int64_t* idx, int64_t b,
                     int nkeys, const int* mods, const float* const* mu,
                     const float* const* sigma, float* lp, hipStream_t stream);
/* dmu_k = dlp_k (M1 - mu M0)/s^2,  dsigma_k = dlp_k (Q/s^3 - M0/s)  (dmu/dsigma
 * entries nullable). */
int mmb_gauss_backward(const double* const* stats, const int* fm, const int64_t* idx, int64_t b,
                       int nkeys, const int* mods, const float* const* mu,
                       const float* const* sigma, const float* dlp, float* const* dmu,
                       float* const* dsigma, hipStream_t stream);
/* The same two with row strides (elements; HOST arrays, one per key): mu_k /
 * dmu_k rows ld_mu[k] apart, sigma_k / dsigma_k rows ld_sigma[k] apart -- the
 * per-key column blocks of the generator's fused output [B, 2 F] (mu) and of
 * exp() of its log-sigma half [B, F] (sigma) without copies.  ld >= F_k;
 * null arrays mean F_k (contiguous rows), as in the unstrided entry points. */
int mmb_gauss_loglik_strided(const double* const* stats, const int* fm, const int64_t* idx,
                             int64_t b, int nkeys, const int* mods, const float* const* mu,
                             const int64_t* ld_mu, const float* const* sigma,
                             const int64_t* ld_sigma, float* lp, hipStream_t stream);
int mmb_gauss_backward_strided(const double* const* stats, const int* fm, const int64_t* idx,
                               int64_t b, int nkeys, const int* mods, const float* const* mu,
                               const int64_t* ld_mu, const float* const* sigma,
                               const int64_t* ld_sigma, const float* dlp, float* const* dmu,
                               float* const* dsigma, hipStream_t stream);

/* Backward of the generator's LayerNorm (reference models.py:163-164,
 * nn.LayerNorm(embedding_dim); its backward is torch's).  dy, x, dx: [n, d]
 * row-major f32; mean, rstd: [n], the forward's saved statistics
 * (torch.native_layer_norm); gamma: [d].  Writes dx and, when non-null,
 * dgamma = sum_rows dy xhat and dbeta = sum_rows dy (fixed reduction order:
 * deterministic).  One launch. */
int mmb_layer_norm_backward(const float* dy, const float* x, const float* mean, const float* rstd,
                            const float* gamma, int64_t n, int d, float* dx, float* dgamma,
                            float* dbeta, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* MMB_H_ */
