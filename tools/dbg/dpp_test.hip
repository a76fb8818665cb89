#include <hip/hip_runtime.h>
#include <cstdio>
template <int PAT> __global__ void k(int* out) {
  int x = threadIdx.x * 10;
  out[threadIdx.x] = __builtin_amdgcn_mov_dpp(x, PAT, 0xF, 0xF, true);
}
template <int PAT> void run(const char* name) {
  int* d; hipMalloc(&d, 64 * 4);
  hipLaunchKernelGGL(k<PAT>, dim3(1), dim3(64), 0, 0, d);
  int h[64]; hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
  printf("%s:", name); for (int i = 0; i < 12; i++) printf(" %d", h[i]); printf("\n");
  hipFree(d);
}
int main() {
  run<0x00>("B0"); run<0x55>("B1"); run<0xAA>("B2"); run<0xFF>("B3");
  run<(1 | (0 << 2) | (2 << 4) | (3 << 6))>("SWAP01");
  run<(0 | (1 << 2) | (2 << 4) | (3 << 6))>("ID");
  return 0;
}
