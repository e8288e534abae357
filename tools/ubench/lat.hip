// Single-wave latency microbenchmarks (cycles per dependent op) on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 4096
__global__ void k_salu(unsigned* out, int seed) {
  unsigned a = __builtin_amdgcn_readfirstlane(seed), b = a + 3;
  long t0 = __builtin_amdgcn_s_memtime();
  #pragma unroll 64
  for (int i = 0; i < N; i++) { a = a * 3 + b; b = a >> 1; }
  long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = (unsigned)(t1 - t0); out[1] = a + b; }
}
__global__ void k_valu(unsigned* out, int seed) {
  unsigned a = seed + threadIdx.x, b = a + 3;
  long t0 = __builtin_amdgcn_s_memtime();
  #pragma unroll 64
  for (int i = 0; i < N; i++) { a = a * 3 + b; b = a >> 1; }
  long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = (unsigned)(t1 - t0); }
  out[1 + threadIdx.x] = a + b;
}
__global__ void k_readlane(unsigned* out, int seed) {
  int v = seed + threadIdx.x;  // lane k holds seed+k
  int s = __builtin_amdgcn_readfirstlane(seed) & 63;
  long t0 = __builtin_amdgcn_s_memtime();
  #pragma unroll 64
  for (int i = 0; i < N; i++) { s = (__builtin_amdgcn_readlane(v, s) + 1) & 63; }
  long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = (unsigned)(t1 - t0); out[1] = s; }
}
__global__ void k_lds(unsigned* out, int seed) {
  __shared__ int tab[256];
  tab[threadIdx.x] = (threadIdx.x * 7 + 1) & 255; tab[threadIdx.x + 64] = (threadIdx.x * 5 + 3) & 255;
  tab[threadIdx.x + 128] = (threadIdx.x * 11 + 9) & 255; tab[threadIdx.x + 192] = (threadIdx.x * 13 + 7) & 255;
  __syncthreads();
  int s = __builtin_amdgcn_readfirstlane(seed) & 255;
  long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) { s = __builtin_amdgcn_readfirstlane(tab[s]); }
  long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = (unsigned)(t1 - t0); out[1] = s; }
}
__global__ void k_branch(unsigned* out, int seed) {
  unsigned a = __builtin_amdgcn_readfirstlane(seed);
  long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) {
    if (a & 1) { a = a * 5 + 1; } else { a = (a >> 1) ^ 0x1234; }
    asm volatile("" : "+s"(a));
  }
  long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[0] = (unsigned)(t1 - t0); out[1] = a; }
}
__global__ void k_simt_dep(unsigned* out, int seed) {
  // per-lane dependent mul/shift/select chain (a SIMT range-coder step model)
  unsigned r = 0xFF00 + threadIdx.x, l = 0, st = 100 + threadIdx.x;
  long t0 = __builtin_amdgcn_s_memtime();
  #pragma unroll 16
  for (int i = 0; i < N; i++) {
    unsigned r1 = (r * st) >> 8; unsigned bit = (st ^ i) & 1;
    l += bit ? r - r1 : 0; r = bit ? r1 : r - r1;
    if (r < 256) { r <<= 8; l = (l & 255) << 8; }
    st = (st * 13 + 7) & 255 | 1;
  }
  long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = (unsigned)(t1 - t0);
  out[1 + threadIdx.x] = r + l;
}
int main() {
  unsigned *d, h[2];
  hipMalloc(&d, 4096);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  struct { const char* n; void (*f)(unsigned*, int); int ops; } K[] = {
    {"salu_dep(mul+add,shift)", k_salu, 2 * N}, {"valu_dep(mul+add,shift)", k_valu, 2 * N},
    {"readlane_chain", k_readlane, N}, {"lds_readfirstlane_chain", k_lds, N},
    {"scalar_branch_iter", k_branch, N}, {"simt_rac_step", k_simt_dep, N}};
  for (auto& k : K) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(1), dim3(64), 0, 0, d, 5);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%-28s memtime/op=%.2f  wall_ns/op=%.2f\n", k.n, (double)h[0] / k.ops, ms * 1e6 / k.ops);
    }
  }
  return 0;
}
