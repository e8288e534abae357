// Batch-1 floor of the range pass: cycles per decision of
// ONE range stream's serial recurrence (range only, rangecoder.h:85-102 and
// the renormalisation of :52-75), in the forms a stream could take when the
// streams are fewer than the SIMDs:
//   V64  64 streams in one wave's lanes (the ffv1_range form)
//   V1   one stream in lane 0 of a wave (the other lanes off)
//   S    one stream in scalar registers (SALU: s_mul_i32, s_flbit, s_cselect)
//   S2   two streams interleaved in one wave's scalar registers
// each with 1 wave per SIMD (grid = SIMDs) and 4 waves per SIMD.  States and
// bits come from registers (a 32-decision block is re-walked): this is the
// recurrence alone, the loads of the real pass are not in it.  Every form
// must end in the same range and shift count as V64's lane for that stream.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench/range1_ub tools/ubench/range1_ub.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

constexpr int kIters = 1024;  // x 32 decisions

template <int I, int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

// one decision: r1 = range * s >> 8; range = bit ? r1 : range - r1; then the
// renormalisation (at most one 8-bit shift: range >= 1 after either branch)
// (VALU: the 24-bit multiply, full rate, as ffv1_range; SALU: s_mul_i32)
template <bool VALU = true>
__device__ __forceinline__ void dec(int& range, int& shifts, uint32_t s, uint32_t bit) {
  const int r1 = (int)((VALU ? __umul24((uint32_t)range, s) : (uint32_t)range * s) >> 8);
  const int nr = bit ? r1 : range - r1;
  const int sh = (int)(__builtin_clz((unsigned)nr) & 8u);
  shifts += sh;
  range = nr << sh;
}

__device__ __forceinline__ void block32(int& range, int& shifts, const uint32_t (&w)[8], uint32_t bw) {
  sfor<0, 32>([&](auto jc) {
    constexpr int J = decltype(jc)::value;
    dec(range, shifts, (w[J >> 2] >> ((J & 3) * 8)) & 0xFFu, (bw >> J) & 1u);
  });
}

// FORM 0: V64 (lane = stream); 1: V1 (lane 0 only); 2: S (scalar, stream =
// the wave's); 3: S2 (two scalar streams interleaved)
template <int FORM>
__global__ __launch_bounds__(64) void k_range(const uint32_t* __restrict__ states, const uint32_t* __restrict__ bits,
                                              int* out, long long* cyc) {
  const int wave = blockIdx.x;
  long long t0 = 0, t1 = 0;
  if constexpr (FORM == 0 || FORM == 1) {
    const int lane = threadIdx.x;
    const int st = FORM == 0 ? wave * 64 + lane : wave;
    if (FORM == 1 && lane != 0) return;
    uint32_t w[8];
    for (int i = 0; i < 8; i++) w[i] = states[st * 8 + i];
    uint32_t bw = bits[st];
    int range = 0xFF00, shifts = 0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; it++) {
      block32(range, shifts, w, bw);
      bw = __builtin_amdgcn_alignbit(bw, bw, 1);
      asm volatile("" : "+v"(bw));
    }
    t1 = __builtin_amdgcn_s_memtime();
    out[2 * st] = range;
    out[2 * st + 1] = shifts;
  } else {
    constexpr int NS = FORM == 2 ? 1 : 2;
    uint32_t w[NS][8], bw[NS];
    int range[NS], shifts[NS];
    for (int q = 0; q < NS; q++) {
      const int st = wave * NS + q;
      for (int i = 0; i < 8; i++) w[q][i] = __builtin_amdgcn_readfirstlane(states[st * 8 + i]);
      bw[q] = __builtin_amdgcn_readfirstlane(bits[st]);
      range[q] = 0xFF00;
      shifts[q] = 0;
    }
    t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; it++) {
      sfor<0, 32>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        for (int q = 0; q < NS; q++)
          dec<false>(range[q], shifts[q], (w[q][J >> 2] >> ((J & 3) * 8)) & 0xFFu, (bw[q] >> J) & 1u);
      });
      for (int q = 0; q < NS; q++) bw[q] = (bw[q] >> 1) | (bw[q] << 31);
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0)
      for (int q = 0; q < NS; q++) {
        out[2 * (wave * NS + q)] = range[q];
        out[2 * (wave * NS + q) + 1] = shifts[q];
      }
  }
  if (threadIdx.x == 0) cyc[wave] = t1 - t0;
}

template <int FORM>
static double run(int waves, const uint32_t* ds, const uint32_t* db, int* dout, long long* dc, std::vector<int>& o) {
  hipLaunchKernelGGL(k_range<FORM>, dim3(waves), dim3(64), 0, 0, ds, db, dout, dc);
  hipDeviceSynchronize();
  std::vector<long long> c(waves);
  hipMemcpy(c.data(), dc, waves * 8, hipMemcpyDeviceToHost);
  const int nst = FORM == 0 ? waves * 64 : FORM == 3 ? waves * 2 : waves;
  o.resize(2 * nst);
  hipMemcpy(o.data(), dout, 8 * nst, hipMemcpyDeviceToHost);
  double s = 0;
  for (long long v : c) s += (double)v;
  return s / waves / (kIters * 32.0);
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int maxst = cus * 4 * 4 * 64;  // V64 at 4 waves per SIMD
  std::vector<uint32_t> hs(maxst * 8), hb(maxst);
  srand(1);
  for (auto& v : hs) {
    v = 0;
    for (int b = 0; b < 4; b++) v |= (uint32_t)(1 + rand() % 255) << (8 * b);
  }
  for (auto& v : hb) v = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
  uint32_t *ds, *db;
  int* dout;
  long long* dc;
  hipMalloc(&ds, hs.size() * 4);
  hipMalloc(&db, hb.size() * 4);
  hipMalloc(&dout, maxst * 8);
  hipMalloc(&dc, maxst * 8);
  hipMemcpy(ds, hs.data(), hs.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
  // the reference: V64's lanes at one wave per SIMD
  std::vector<int> ref, o;
  const int simds = cus * 4;
  printf("{\"cus\": %d, \"decisions_per_wave\": %d, \"forms\": [\n", cus, kIters * 32);
  for (int per = 1; per <= 4; per *= 4) {
    const int waves = simds * per;
    const double v64 = run<0>(waves, ds, db, dout, dc, ref);
    const double v1 = run<1>(waves, ds, db, dout, dc, o);
    int bad1 = 0;
    for (int i = 0; i < waves; i++) bad1 += o[2 * i] != ref[2 * i] || o[2 * i + 1] != ref[2 * i + 1];
    const double s1 = run<2>(waves, ds, db, dout, dc, o);
    int bad2 = 0;
    for (int i = 0; i < waves; i++) bad2 += o[2 * i] != ref[2 * i] || o[2 * i + 1] != ref[2 * i + 1];
    const double s2 = run<3>(waves, ds, db, dout, dc, o);
    int bad3 = 0;
    for (int i = 0; i < 2 * waves; i++) bad3 += o[2 * i] != ref[2 * i] || o[2 * i + 1] != ref[2 * i + 1];
    printf("  {\"waves_per_simd\": %d, \"cycles_per_decision\": {\"V64\": %.2f, \"V1\": %.2f, \"S\": %.2f, "
           "\"S2_per_stream_step\": %.2f}, \"mismatches\": {\"V1\": %d, \"S\": %d, \"S2\": %d}}%s\n",
           per, v64, v1, s1, s2, bad1, bad2, bad3, per == 1 ? "," : "");
  }
  printf("]}\n");
  return 0;
}
