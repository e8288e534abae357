// Range-pass recurrence microbenchmark (one wave per block, cycles per
// decision per lane): the current form (range32: mul, shift, sub, select,
// then the renormalisation from the leading-zero count, a 7-deep chain per
// decision) against the deferred-shift form (the renormalisation of decision
// i folded into decision i+1's product: (nr * m) << sh + a, a 4-deep chain).
// Both must end in the same range and shift count.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/range_ub tools/ubench/range_ub.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int kIters = 512;  // x 32 decisions

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

struct Masks8 { int m[8]; };
template <int G>
__device__ __forceinline__ Masks8 masks8(uint32_t bw) {
  Masks8 k;
  sfor<0, 8>([&](auto jc) { k.m[decltype(jc)::value] = __builtin_amdgcn_sbfe((int)bw, 8 * G + decltype(jc)::value, 1); });
  asm volatile("" : "+v"(k.m[0]), "+v"(k.m[1]), "+v"(k.m[2]), "+v"(k.m[3]), "+v"(k.m[4]), "+v"(k.m[5]), "+v"(k.m[6]),
               "+v"(k.m[7]));
  return k;
}

// current: range32 of ffv1_kernels.hip
__device__ __forceinline__ void range32_cur(int& range, int& shifts, const uint32_t* w, uint32_t bw) {
  sfor<0, 4>([&](auto gc) {
    constexpr int G = decltype(gc)::value;
    const Masks8 k = masks8<G>(bw);
    sfor<0, 8>([&](auto jc) {
      constexpr int J = 8 * G + decltype(jc)::value;
      const uint32_t s = (w[J >> 2] >> ((J & 3) * 8)) & 0xFFu;
      const int m = k.m[J & 7];
      const int r1 = (int)(__umul24((unsigned)range, s) >> 8);
      const int d = range - r1;
      const int nr = (m & r1) | (~m & d);
      const int sh = (int)(__builtin_clz((unsigned)nr) & 8u);
      shifts += sh;
      range = nr << sh;
    });
  });
}

// deferred shift: nr (the range before its renormalisation) and the product
// of the next decision taken as (nr * m) << sh + a, m = bit ? s : 256 - s,
// a = bit ? 0 : 255, then >> 8; the shift of nr is applied to the product
// (nr << sh) * m = (nr * m) << sh
__device__ __forceinline__ void range32_def(int& nr, int& shifts, const uint32_t* w, uint32_t bw) {
  sfor<0, 4>([&](auto gc) {
    constexpr int G = decltype(gc)::value;
    const Masks8 k = masks8<G>(bw);
    sfor<0, 8>([&](auto jc) {
      constexpr int J = 8 * G + decltype(jc)::value;
      const uint32_t s = (w[J >> 2] >> ((J & 3) * 8)) & 0xFFu;
      const int msk = k.m[J & 7];
      // off the chain: m and a
      const uint32_t mm = (uint32_t)((msk & (int)s) | (~msk & (256 - (int)s)));
      const uint32_t aa = (uint32_t)(~msk & 255);
      // on the chain
      const uint32_t sh = __builtin_clz((unsigned)nr) & 8u;
      const uint32_t x = __umul24((unsigned)nr, mm);
      shifts += (int)sh;
      nr = (int)(((x << sh) + aa) >> 8);
    });
  });
}

template <int FORM>
__global__ __launch_bounds__(64) void k_range(const uint32_t* states, const uint32_t* bits, int* out, long long* cyc) {
  const int lane = threadIdx.x + blockIdx.x * 64;
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = states[lane * 8 + i];
  uint32_t bw = bits[lane];
  int range = 0xFF00, shifts = 0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; it++) {
    if (FORM == 0) range32_cur(range, shifts, w, bw);
    else range32_def(range, shifts, w, bw);
    bw = __builtin_amdgcn_alignbit(bw, bw, 1);  // vary the bits a little
    asm volatile("" : "+v"(bw));
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (FORM == 1) {  // the final renormalisation
    const int sh = (int)(__builtin_clz((unsigned)range) & 8u);
    shifts += sh;
    range <<= sh;
  }
  out[2 * lane] = range;
  out[2 * lane + 1] = shifts;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 1;
  const int n = blocks * 64;
  uint32_t* hs = (uint32_t*)malloc(n * 32);
  uint32_t* hb = (uint32_t*)malloc(n * 4);
  srand(1);
  for (int i = 0; i < n * 8; i++) {
    uint32_t v = 0;
    for (int b = 0; b < 4; b++) v |= (uint32_t)(1 + rand() % 255) << (8 * b);
    hs[i] = v;
  }
  for (int i = 0; i < n; i++) hb[i] = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
  uint32_t *ds, *db;
  int* dout;
  long long* dc;
  hipMalloc(&ds, n * 32);
  hipMalloc(&db, n * 4);
  hipMalloc(&dout, n * 8 * 2);
  hipMalloc(&dc, blocks * 8 * 2);
  hipMemcpy(ds, hs, n * 32, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, n * 4, hipMemcpyHostToDevice);
  int* o0 = (int*)malloc(n * 8);
  int* o1 = (int*)malloc(n * 8);
  long long* c = (long long*)malloc(blocks * 8);
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k_range<0>, dim3(blocks), dim3(64), 0, 0, ds, db, dout, dc);
    hipMemcpy(o0, dout, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(c, dc, blocks * 8, hipMemcpyDeviceToHost);
    double c0 = 0;
    for (int b = 0; b < blocks; b++) c0 += c[b];
    hipLaunchKernelGGL(k_range<1>, dim3(blocks), dim3(64), 0, 0, ds, db, dout, dc);
    hipMemcpy(o1, dout, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(c, dc, blocks * 8, hipMemcpyDeviceToHost);
    double c1 = 0;
    for (int b = 0; b < blocks; b++) c1 += c[b];
    int bad = 0;
    for (int i = 0; i < 2 * n; i++) bad += o0[i] != o1[i];
    printf("blocks %d: current %.2f cycles/decision, deferred %.2f, mismatches %d\n", blocks,
           c0 / blocks / (kIters * 32.0), c1 / blocks / (kIters * 32.0), bad);
  }
  return 0;
}
