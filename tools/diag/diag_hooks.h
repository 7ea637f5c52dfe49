// The tools build's hook definitions (tools/diag/libmmb_diag.so), force-
// included in front of every product source by `make diag` (-include).  Each
// MMB_HOOK_* point in multimodal-baselines_amd/csrc/ compiles its product
// default unless defined here; the definitions behind the hooks (variant
// kernels, sweep launches, knobs, mmb_diag_* entry points) are in
// tools/diag/{sif,pc,mm2}_tail.inc, included at the end of the product
// sources through MMB_TOOLS_TAIL_*.  The product library (`make`) sees none
// of this and reads no environment variable.  Test and timing
// infrastructure, not product code.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

namespace mmb {

// an integer knob, re-read per launch (in-process A/B sweeps flip them)
inline int diag_knob(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

// ---- sif_kernels.hip ---------------------------------------------------------
inline int diag_stream_grid_mult() {
  const int v = diag_knob("MMB_STREAM_GRID_MULT", 2);
  return v > 0 ? v : 2;
}
template <class A>
bool diag_narrow_launch(int var, const A& a, int grid, hipStream_t stream);
template <bool MM2, int CT, int CA, int CV, class A>
bool diag_wave_launch(const A& a, int grid, hipStream_t stream);
template <class F>
bool diag_fused_launch(const F& f, int grid, hipStream_t stream);
template <bool MM2, int VT, int VA, int VV, class A>
bool diag_stream_small(const A& a, int grid, hipStream_t stream);
template <class F>
void diag_fused_args(F& f) {
  f.balanced = diag_knob("MMB_FUSED_BALANCED", 1);
  if (diag_knob("MMB_FUSED_DYN", 1) == 0) f.sched = nullptr;
}
template <int I = 0>
void diag_nf_teams_attr();
template <class F>
bool diag_nf_teams_launch(int teams, const F& f, int64_t grid, hipStream_t stream);
// a test shortens the fused kernel's bounded waits (mmb_diag_fused_wait_iters)
static __device__ int g_fused_wait_iters = 1 << 23;
// per-workgroup wall-clock marks of the fused kernel (start; each streamer
// wave's and each projector wave's end), read back with mmb_diag_fused_probe
constexpr int kFProbe = 9;
static __device__ unsigned long long g_fused_probe[1024 * kFProbe];

#define MMB_HOOK_STREAM_GRID_MULT diag_stream_grid_mult()
#define MMB_HOOK_NARROW_VARIANT diag_knob("MMB_STREAM_NARROW", 10)
#define MMB_HOOK_NARROW_LAUNCH diag_narrow_launch(var, a, grid, stream)
#define MMB_HOOK_WAVE_LAUNCH diag_wave_launch<MM2, CT, CA, CV>(a, grid, stream)
#define MMB_HOOK_FUSED_WAIT_ITERS g_fused_wait_iters
#define FUSED_PROBE(slot)                                                              \
  do {                                                                                 \
    if ((threadIdx.x & (kWave - 1)) == 0 && blockIdx.x < 1024)                         \
      g_fused_probe[blockIdx.x * kFProbe + (slot)] = wall_clock64();                   \
  } while (0)
#define MMB_HOOK_FUSED_LAUNCH diag_fused_launch(f, grid, stream)
#define MMB_HOOK_STREAM_SMALL diag_stream_small<MM2, VT, VA, VV>(a, grid, stream)
#define MMB_HOOK_FUSED_ARGS(f) diag_fused_args(f)
#define MMB_HOOK_NF_TEAMS diag_knob("MMB_NF_TEAMS", 0)
#define MMB_HOOK_NF_TEAMS_ATTR diag_nf_teams_attr()
#define MMB_HOOK_NF_TEAMS_LAUNCH diag_nf_teams_launch(teams, f, grid, stream)
#define MMB_TOOLS_TAIL_SIF "../../tools/diag/sif_tail.inc"

// ---- pc_kernels.hip ----------------------------------------------------------
// a test shortens the solve's bounded waits (mmb_diag_pc_wait_iters) and names
// one workgroup that never arrives (mmb_diag_pc_skip_arrival)
static __device__ int g_pm_wait_iters = 1 << 20;
static __device__ int g_pm_skip_wg = -1;
inline void diag_gram_ranges(int& r) {
  const int v = diag_knob("MMB_GRAM_RANGES", 0);  // A/B: ranges (<= 128)
  if (v > 0) r = std::max(r, std::min(v, 128));
}
bool diag_gram_i8_v1(int& rc, const float* x, const uint32_t* colmax, int64_t n, int d, double* g,
                     int accumulate, double* part, hipStream_t stream);
int diag_gram_i8_block(const float* xb, const uint32_t* colmax, int64_t nb, int d, double* g, int acc,
                       double* part, hipStream_t stream);
bool diag_solve_launch(int& rc, const double* g, double* g2, int nsq_wg, int d, const double* z0, int k,
                       int npc, int n_iter, int transposed, double* pc_out, double* xbuf, unsigned* ctl,
                       int32_t* flag, int T, hipStream_t stream);
bool diag_pc_remove_launch(int rr, int grid, hipStream_t stream, const float* num, const float* cnt,
                           int64_t n, int d, const double* pc, float* out32);

#define MMB_HOOK_PM_WAIT_ITERS g_pm_wait_iters
#define MMB_HOOK_PM_SKIP_ARRIVAL (static_cast<int>(blockIdx.x) == g_pm_skip_wg)
#define MMB_HOOK_PC_REMOVE_R diag_knob("MMB_PC_REMOVE_R", 4)
#define MMB_HOOK_GRAM_RANGES(r) diag_gram_ranges(r)
#define MMB_HOOK_GRAM_I8(rc) diag_gram_i8_v1(rc, x, colmax, n, d, g, accumulate, part, stream)
#define MMB_HOOK_GRAM_I8_BLOCK diag_gram_i8_block
#define MMB_HOOK_SOLVE_LAUNCH(rc) \
  diag_solve_launch(rc, g, g2, nsq_wg, d, z0, k, npc, n_iter, transposed, pc_out, xbuf, ctl, flag, T, stream)
#define MMB_HOOK_PC_REMOVE_LAUNCH diag_pc_remove_launch(rr, grid, stream, num, cnt, n, d, pc, out32)
#define MMB_TOOLS_TAIL_PC "../../tools/diag/pc_tail.inc"

// ---- mm2_kernels.hip ---------------------------------------------------------
template <int CT>
bool diag_launch_project_x3(int& rc, const _Float16* s, const float* num, const float* aux,
                            const _Float16* img, const float* ci, const float* c0, int64_t n, int kp,
                            int d, float* out, const double* pc, float* sif, hipStream_t stream);
#define MMB_HOOK_PROJECT_X3(rc) \
  diag_launch_project_x3<CT>(rc, s, num, aux, img, ci, c0, n, kp, d, out, pc, sif, stream)
#define MMB_TOOLS_TAIL_MM2 "../../tools/diag/mm2_tail.inc"

}  // namespace mmb
