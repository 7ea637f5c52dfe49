// Diagnostic: which XCD / SE / CU does each CU-mask bit select?  One
// single-wave launch per mask bit on a stream restricted to that bit; the
// wave records its XCC_ID and HW_ID hardware registers.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

__global__ void probe(uint32_t* out) {
  if (threadIdx.x == 0) {
    out[0] = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
    out[1] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
  }
}

int main() {
  int n = 0;
  hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* d;
  hipMalloc(&d, 8);
  std::printf("bit xcc hw_id cu se\n");
  for (int b = 0; b < n; ++b) {
    std::vector<uint32_t> mask((n + 31) / 32, 0);
    mask[b / 32] = 1u << (b % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, mask.size(), mask.data()) != hipSuccess) return 1;
    probe<<<1, 64, 0, s>>>(d);
    uint32_t h[2];
    hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    hipStreamDestroy(s);
    std::printf("%d %u 0x%x %u %u\n", b, h[0] & 0xf, h[1], (h[1] >> 8) & 0xf, (h[1] >> 13) & 0x7);
  }
  return 0;
}
