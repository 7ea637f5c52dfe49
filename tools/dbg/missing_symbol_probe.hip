// Does hipFuncGetAttributes report a kernel whose device code is missing
// from the code object (the r05 "Cannot find Symbol" abort of
// tools/nf_ab.py), or does it abort like the launch did?  The kernel
// template's instantiation is referenced only in the host pass, so the
// device pass never emits it: the host stub is registered, the symbol is
// not in the gfx950 code object.
//   hipcc -O2 --offload-arch=gfx950 -o tools/dbg/missing_symbol_probe tools/dbg/missing_symbol_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int X>
__global__ void probe_missing_kernel(int* p) {
  p[0] = X;
}
__global__ void probe_present_kernel(int* p) { p[0] = 7; }

int main() {
  int* d = nullptr;
  if (hipMalloc(&d, sizeof(int)) != hipSuccess) return 3;
  hipFuncAttributes fa;
  hipError_t e = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&probe_present_kernel));
  std::printf("present kernel: hipFuncGetAttributes -> %d (%s)\n", static_cast<int>(e), hipGetErrorString(e));
  std::fflush(stdout);
#ifndef __HIP_DEVICE_COMPILE__
  e = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&probe_missing_kernel<3>));
  std::printf("missing kernel: hipFuncGetAttributes -> %d (%s)\n", static_cast<int>(e), hipGetErrorString(e));
  std::fflush(stdout);
#endif
  (void)hipFree(d);
  return 0;
}
