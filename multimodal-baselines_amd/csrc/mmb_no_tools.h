// Intentionally empty: the product library's target of the MMB_TOOLS_TAIL_*
// includes at the end of sif_kernels.hip, pc_kernels.hip and mm2_kernels.hip.
// The tools build (`make diag`, tools/diag/diag_hooks.h) points them at its
// variant kernels, sweep launches and mmb_diag_* entry points instead.
