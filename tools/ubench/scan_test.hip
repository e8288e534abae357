#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
  return x;
}
__global__ void k(int* o) { int l = threadIdx.x; int v = (l * 7 + 3) % 11; o[l] = wave_incl_scan(v); o[64 + l] = __builtin_amdgcn_update_dpp(0, l + 100, 0x138, 0xf, 0xf, true); }
int main() { int* d; hipMalloc(&d, 512); k<<<1, 64>>>(d); int h[128]; hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  int acc = 0, bad = 0; for (int l = 0; l < 64; l++) { acc += (l * 7 + 3) % 11; if (h[l] != acc) bad++; if (h[64 + l] != (l ? l + 99 : 0)) bad++; }
  printf("scan/shr errors: %d\n", bad); return bad != 0; }
