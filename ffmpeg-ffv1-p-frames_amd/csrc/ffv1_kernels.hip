// ffv1_kernels.hip -- CDNA4 (gfx950) kernels of the FFV1 P-frame encoder.
//
// Hot path, three kernels per batch:
//
//   ffv1_symbols   fully parallel: one thread per sample computes median
//                  prediction, the quantised-gradient context and the folded
//                  residual (ffv1.h:148-190, ffv1enc.c:306-317), with the
//                  reference's ring-buffer edge rules (ffv1enc.c:381-388).
//                  Output: one 32-bit symbol per sample, in coding order.
//
//   ffv1_code      the range coder (rangecoder.h:52-102) + binarisation
//                  (ffv1enc.c:185-231), SIMT: ONE LANE PER (segment, slice)
//                  CHAIN.  A slice's bitstream is inherently serial, so
//                  parallelism comes from coding 64 independent slice streams
//                  per wavefront.  Each lane keeps its current context's 32
//                  adaptive states in 8 VGPRs; the binarisation is laid out as
//                  static slot positions, so every state byte is extracted and
//                  re-inserted at a compile-time offset.  Renormalisation does
//                  not emit bytes inline: it stores a 10-bit "digit" (the top
//                  byte of `low`, its carry, and the 0xFF-deferral flag) and a
//                  per-lane post-pass replays the reference's pending-byte /
//                  0xFF-run logic exactly.  The per-chain context tables (the
//                  P-frame carry, ffv1enc.c:1171-1172) live in HBM/L2 and are
//                  gathered one 32-byte row per context change, with the next
//                  symbol's row prefetched while the current one codes.
//
//   ffv1_assemble_packets  packet placement (prefix over slice sizes), the
//                  3-byte size, 0x00 and the slice CRC-32 computed chunk-
//                  parallel and combined in GF(2) (ffv1enc.c:1326-1354).
#include <hip/hip_runtime.h>
#include <cstdlib>

#include <type_traits>

#include "ffv1_internal.h"

namespace ffv1hip {

namespace {

constexpr int kWave = 64;
constexpr int kBufDword3 = 0x00020000;  // gfx9-family raw buffer (32-bit data format)

__device__ __forceinline__ int median3(int a, int b, int c) {
  return max(min(a, b), min(max(a, b), c));
}

// fold() (ffv1.h:148-159) == sign-extension of the low `bits` bits
__device__ __forceinline__ int fold_bits(int d, int bits) {
  const int sh = 32 - bits;
  return (d << sh) >> sh;
}

// ---------------------------------------------------------------------------
// Kernel 1: symbols.
#ifndef FFV1_SYM_THREADS
#define FFV1_SYM_THREADS 64
#define FFV1_SYM_SPLIT 24
#endif
constexpr int kSymThreads = FFV1_SYM_THREADS;  // one wave per block: a wave slowed by a busy SIMD holds back no other
constexpr int kSymSplit = FFV1_SYM_SPLIT;  // blocks per slice plane: the per-block loop is latency-bound

// Range-coder decisions of one residual: put_symbol_inline (ffv1enc.c:185-231)
// codes a zero flag, e+1 exponent decisions, e mantissa bits and a sign.
__device__ __forceinline__ int decisions_of(int v) {
  const unsigned mag = v < 0 ? 0u - (unsigned)v : (unsigned)v;
  return v ? 2 * (31 - __builtin_clz(mag)) + 3 : 1;
}

// The symbol's decision bits in coding order (bit d = decision d): zero flag,
// e ones and a zero, the mantissa MSB first, the sign.
__device__ __forceinline__ uint64_t decision_bits(int v) {
  if (!v) return 1;
  const unsigned mag = v < 0 ? 0u - (unsigned)v : (unsigned)v;
  const int e = 31 - __builtin_clz(mag);
  const uint64_t unary = (uint64_t)((1u << e) - 1u) << 1;
  const uint64_t mant = e ? (uint64_t)(__brev(mag) >> (32 - e)) << (e + 2) : 0;
  return unary | mant | ((uint64_t)(v < 0) << (2 * e + 2));
}

// Per-slot decisions of one symbol (put_symbol_inline, ffv1enc.c:185-231):
// slot 0 zero flag, 1..e+1 unary, 11+e sign, 22..21+e mantissa, as two slot
// masks, one bit per slot: bm the decision bit, nd "no decision" (the walk's
// code for lane k: nd ? 2 : bit; both set: several decisions, code 3, at
// e = 10, 11).  The walk reads bit k of each, so nothing is spread to 2-bit
// codes (that took ~48 VALU per record).
__device__ __forceinline__ void slot_masks(int v, uint32_t& bm, uint32_t& nd) {
  const unsigned mag = v < 0 ? 0u - (unsigned)v : (unsigned)v;
  const int e = v ? 31 - __builtin_clz(mag) : -1;
  const uint32_t neg = (uint32_t)(v < 0);
  if (e >= 10) {
    // slots 1..9 a one each, slot 10 several (3), sign in 21, mantissa bits
    // 0..8 in 22..30, bits 9..e-1 in 31 (one at e = 10, several at 11)
    const uint32_t lo9 = mag & 0x1FFu;
    const uint32_t t = 0x3FFu | (1u << 21) | (0x1FFu << 22) | (e == 10 ? 1u << 31 : 0u);  // (slot 10: several)
    bm = 0x3FEu | (1u << 10) | (neg << 21) | (lo9 << 22) | (e == 10 ? ((mag >> 9) & 1u) << 31 : 1u << 31);
    nd = ~t;
    return;
  }
  const uint32_t lo = v ? (1u << e) - 1u : 0u;  // e ones
  const uint32_t t = v ? (1u | (((2u << e) - 1u) << 1) | (1u << (11 + e)) | (lo << 22)) : 1u;
  bm = v ? ((lo << 1) | (neg << (11 + e)) | ((mag & lo) << 22)) : 1u;
  nd = ~t;
}

// The same per-slot decisions as 2-bit codes, two bits per slot (c0 slots
// 0..15, c1 16..31): 0/1 the decision bit, 2 none, 3 several (slot 10 at e
// >= 10, slot 31 at e = 11).  The walk expands the chunks with e = 10, 11
// symbols this way: one field extract gives a lane its code there, where the
// two masks need a combination of three (measured with codes in every
// chunk: c4, where such chunks are common, 7.95 -> 8.33 Gpix/s, c3 19.02 ->
// 18.87; so the plain chunks keep the masks, cheaper to expand).
__device__ __forceinline__ uint32_t spread16(uint32_t x) {
  x &= 0xFFFFu;
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return x;
}

// Per-slot codes of one symbol with e <= 9, two bits per slot (slots 0..15
// in the first word, 16..31 in the second): 0/1 the slot's decision bit,
// 2 no decision.  Slot 0 zero flag, 1..e+1 unary, 11+e sign, 22..21+e
// mantissa (put_symbol_inline, ffv1enc.c:185-231).
__device__ __forceinline__ void slot_codes(int v, uint32_t& c0, uint32_t& c1) {
  const unsigned mag = v < 0 ? 0u - (unsigned)v : (unsigned)v;
  const int e = v ? 31 - __builtin_clz(mag) : -1;
  if (e >= 10) {
    // e = 10, 11: slots 1..9 a one each, slot 10 the ones of i = 9..e-1 and
    // the terminating zero (code 3), sign in slot 21, mantissa bits 0..8 in
    // slots 22..30, bits 9..e-1 in slot 31 (one: its bit; two: code 3)
    const uint32_t pres = 0x7FFu & ~1u;  // slots 1..10
    const uint32_t lo9 = mag & 0x1FFu;
    uint32_t cc0 = spread16(pres & 0x3FEu) | (spread16(~pres & 0xFFFFu) << 1);  // 1s in 1..9, none elsewhere but 10
    cc0 = (cc0 & ~(3u << 20)) | (3u << 20);                                       // slot 10: several
    cc0 &= ~3u;                                                                   // slot 0: 0 (nonzero)
    uint32_t hi = (uint32_t)(v < 0) << 5 | (lo9 << 6);  // slot 21 (bit 5 of the high half), 22..30
    uint32_t pr = (1u << 5) | (0x1FFu << 6);
    uint32_t cc1 = spread16(hi) | (spread16(~pr & 0xFFFFu) << 1);
    const uint32_t c31 = e == 10 ? ((mag >> 9) & 1u) : 3u;
    cc1 = (cc1 & ~(3u << 30)) | (c31 << 30);
    c0 = cc0;
    c1 = cc1;
    return;
  }
  const uint32_t lo = v ? (1u << e) - 1u : 0u;  // e ones
  const uint32_t tm = v ? (1u | (((2u << e) - 1u) << 1) | (1u << (11 + e)) | (lo << 22)) : 1u;
  const uint32_t bm = v ? ((lo << 1) | ((uint32_t)(v < 0) << (11 + e)) | ((mag & lo) << 22)) : 1u;
  const uint32_t nt = ~tm;
  c0 = spread16(bm) | (spread16(nt) << 1);
  c1 = spread16(bm >> 16) | (spread16(nt >> 16) << 1);
}

// Inclusive wave scan in DPP moves (no LDS round trips): within rows of 16
// by row_shr 1, 2, 4, 8, then the row totals by row_bcast 15 / 31.
__device__ __forceinline__ int wave_incl_scan(int x, int /*lane*/) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 into rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 into rows 2, 3
  return x;
}

// the previous lane's value (lane 0: 0), a DPP wave_shr:1
__device__ __forceinline__ int wave_prev(int x) { return __builtin_amdgcn_update_dpp(0, x, 0x138, 0xf, 0xf, true); }
// the next lane's value (lane 63: 0), a DPP wave_shl:1
__device__ __forceinline__ int wave_next(int x) { return __builtin_amdgcn_update_dpp(0, x, 0x130, 0xf, 0xf, true); }

// RGB (encode_rgb_frame, ffv1enc.c:413-459): pixel (x, y) of the frame as
// coded plane p of the reversible colour transform, G' = g + (b' + r') >> 2,
// B' = b - g + off, R' = r - g + off, and A (p = 3, RGB32) as it is.  bgr0 /
// RGB32: one u32 per pixel (B, G, R, X / A bytes); gbrp: three u16 planes
// read in AVFrame data[] order as b, g, r.
template <int SB>
__device__ __forceinline__ int rct_sample(const SymbolArgs& a, const uint8_t* fr, int p, int x, int y, int2 co) {
  int b, g, r;
  if constexpr (SB == 4) {
    const uint32_t v = reinterpret_cast<const uint32_t*>(fr + a.plane_off[0] + (int64_t)y * a.plane_stride[0])[x];
    if (p == 3) return (int)(v >> 24);
    b = v & 0xFF;
    g = (v >> 8) & 0xFF;
    r = (v >> 16) & 0xFF;
  } else {
    b = reinterpret_cast<const uint16_t*>(fr + a.plane_off[0] + (int64_t)y * a.plane_stride[0])[x];
    g = reinterpret_cast<const uint16_t*>(fr + a.plane_off[1] + (int64_t)y * a.plane_stride[1])[x];
    r = reinterpret_cast<const uint16_t*>(fr + a.plane_off[2] + (int64_t)y * a.plane_stride[2])[x];
  }
  b -= g;
  r -= g;
  g += (b * co.x + r * co.y) >> 2;  // v4: the slice's coefficients (ffv1enc.c:450), else 1, 1
  return p == 0 ? g : (p == 1 ? b : r) + a.rct_offset;
}

// SB: stored sample bytes, 1 or 2; 4: bgr0.  RGB: the colour transform
// (a template argument: a run-time test inside the sample loads would keep
// them from issuing back to back)
template <int SB, bool RGB>
__global__ __launch_bounds__(kSymThreads) void ffv1_symbols(SymbolArgs a) {
  // the quant tables from global memory (2.5 KB, cached): with them in LDS
  // the kernel's blocks would take the LDS the states walk's waves need
  // beside it (~13 KB per CU is left by three walk waves)
  const int16_t* __restrict__ const qt = a.qt;
  __shared__ int red[kSymThreads / kWave];
  __shared__ uint32_t cstage[kSymThreads / kWave][kChunkWords];  // a wave's chunk bits (the largest chunk)
  // a plane of a slice is split into kSymSplit runs of whole 256-sample steps;
  // work item vb = ((plane part) * nslots + slot) * nslices + slice, strided
  // over a grid that may be smaller than the items (launch_symbols: a bounded
  // grid leaves the CUs room for the states walk's waves beside it)
  const int64_t nvb = (int64_t)a.nslices * a.nslots * a.nz;
  for (int64_t vb = blockIdx.x; vb < nvb; vb += gridDim.x) {
  const int slice = (int)(vb % a.nslices), slot = (int)(vb / a.nslices % a.nslots);
  const int z = (int)(vb / ((int64_t)a.nslices * a.nslots));
  const int p = a.p_lo + z / kSymSplit, part = z % kSymSplit;
  const int f = a.frame_of_slot[slot];
  if (f < 0 || p >= a.nplanes) continue;
  // frames mode (walk records): the outputs are indexed by batch frame (a
  // launch may cover a subset of the frames)
  const int fs = a.rec ? f : slot;
  int* const count = a.dcount ? a.dcount + ((int64_t)fs * a.nslices + slice) * 3 + p : nullptr;  // zeroed
  const SliceGeom& g = a.geom[slice];
  const int pw = g.pw[p], ph = g.ph[p], px = g.px[p], py = g.py[p];
  const uint8_t* base = a.frames + (int64_t)f * a.frame_bytes + a.plane_off[p];
  const int stride = a.plane_stride[p];
  // RGB: the slice's G', B', R' (A) rows interleave (ffv1enc.c:428-471)
  uint32_t* out = a.sym + (int64_t)slot * a.frame_samples + g.sym_off + (RGB ? 0 : g.plane_sym_off[p]);
  const int row0 = a.pset[p] * a.contexts;  // the plane context's rows follow the previous ones'
  const int step = a.pstep[p];

  // sample of the slice plane as int16 (ffv1enc.c:390-407), at in-plane
  // coordinates: every load is unconditional, so the loads of a step are
  // issued back to back and waited for once
  const int sh = a.packed_at_lsb ? 0 : a.msb_shift;
  const uint8_t* const fr = a.frames + (int64_t)f * a.frame_bytes;
  const int2 co = RGB && a.rct ? a.rct[(int64_t)f * a.nslices + slice] : make_int2(1, 1);
  // YCbCr planes through a buffer resource: a sample's address is one 24-bit
  // multiply-add on 32-bit offsets, not 64-bit arithmetic (a plane is < 2 GB)
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), 0, 0x7FFFFFFF, kBufDword3);
  auto load = [&](int x, int y) -> int {
    if constexpr (SB == 4) {
      return rct_sample<4>(a, fr, p, px + x, py + y, co);
    } else {
      if constexpr (SB == 2 && RGB) return rct_sample<2>(a, fr, p, px + x, py + y, co);
      if constexpr (SB == 1) {
        const uint32_t off = __umul24((uint32_t)(py + y), (uint32_t)stride) + (uint32_t)((px + x) * step);
        return __builtin_amdgcn_raw_buffer_load_b8(prs, off, 0, 0);
      } else {
        const uint32_t off = __umul24((uint32_t)(py + y), (uint32_t)stride) + (uint32_t)(px + x) * 2u;
        return (int16_t)(__builtin_amdgcn_raw_buffer_load_b16(prs, off, 0, 0) >> sh);
      }
    }
  };

  int ndec = 0;
  const int64_t n = (int64_t)pw * ph;
  const int64_t span = (n + kSymSplit * kSymThreads - 1) / (kSymSplit * kSymThreads) * kSymThreads;
  const int64_t b0 = part * span, b1 = min(n, b0 + span);
  const int lane = threadIdx.x & (kWave - 1);
  uint2* const rec = a.rec ? a.rec + (int64_t)fs * a.frame_samples + g.sym_off + g.plane_sym_off[p] : nullptr;
  // the plane's chunk headers (read once: a reload inside the loop would
  // wait for the record stores)
  const int cw = a.cwords;
  uint32_t* const cbase = rec ? a.cbits + ((int64_t)fs * a.frame_chunks + g.chunk_off[p]) * cw : nullptr;
  // the lane's sample, stepped along the plane without a division per step
  int cy = (int)((b0 + threadIdx.x) / pw), cx = (int)((b0 + threadIdx.x) - (int64_t)cy * pw);
  // whole waves per step: a wave's 64 consecutive samples are one walk chunk
  for (int64_t base = b0; base < b1; base += kSymThreads) {
    const int64_t idx = base + threadIdx.x;
    const bool valid = idx < n;
    const int y = valid ? cy : 0, x = valid ? cx : 0;
    cx += kSymThreads;
    while (cx >= pw) {
      cx -= pw;
      cy++;
    }
    // neighbourhood as the zeroed two/three-row ring exposes it:
    // rows above the slice read 0; L(x=0) = T; LT(x=0) = sample two rows up
    // in column 0; RT past the right edge = T; LL(x=0) = 0, LL(x=1) = T(0).
    // A wave's 64 lanes hold 64 consecutive samples of the plane, so the
    // L / LT / RT taps are the neighbouring lanes' X / T (DPP wave shifts):
    // only X and T are loaded per lane, plus two fix-up loads that touch new
    // memory on the wave's edge lanes and on the lanes at x = 0 only (every
    // other lane re-reads its own X / T address)
    const int ym1 = y ? y - 1 : 0, ym2 = y >= 2 ? y - 2 : 0;
    const bool first = lane == 0, last = lane == kWave - 1;
    const int X = load(x, y);
    const int rT = load(x, ym1);
    const bool fe = first && x, le = last && x + 1 < pw;
    const int f1 = load(fe ? x - 1 : x, x ? y : ym2);          // L on lane 0, LT at x = 0, else X again
    const int f2 = load(fe ? x - 1 : (le ? x + 1 : x), ym1);  // LT on lane 0, RT on lane 63, else T again
    const int pX = wave_prev(X), pT = wave_prev(rT), nT = wave_next(rT);
    int rLL = 0, rTT = 0, rT0 = 0;
    if (a.model1) {
      rLL = load(x >= 2 ? x - 2 : 0, y);
      rTT = load(x, ym2);
      rT0 = load(0, ym1);
    }
    const int T = y ? rT : 0;
    const int T0 = a.model1 ? (y ? rT0 : 0) : T;  // T at x = 0; model 1 also needs it at x = 1
    const int L = x ? (first ? f1 : pX) : T;
    const int LT = x ? (y ? (first ? f2 : pT) : 0) : (y >= 2 ? f1 : 0);
    const int RT = x + 1 < pw ? (y ? (last ? f2 : nT) : 0) : T;
    int ctx = qt[(L - LT) & 0xFF] + qt[256 + ((LT - T) & 0xFF)] + qt[512 + ((T - RT) & 0xFF)];
    if (a.model1) {
      const int LL = x >= 2 ? rLL : (x == 1 ? T0 : 0);
      const int TT = y >= 2 ? rTT : 0;
      ctx += qt[768 + ((LL - L) & 0xFF)] + qt[1024 + ((TT - T) & 0xFF)];
    }
    int diff = X - median3(L, L + T - LT, T);
    if (ctx < 0) {
      ctx = -ctx;
      diff = -diff;
    }
    diff = fold_bits(diff, a.coded_bits);
    const int nd = valid ? decisions_of(diff) : 0;
    ndec += nd;
    if (rec) {
      // the walk record: row inside the plane group, slot codes, the decision
      // offset inside the chunk (wave prefix sum), same-row flag
      const int raddr = (int)__umul24((uint32_t)ctx, (uint32_t)a.rowb);  // ctx >= 0 here
      const int incl = wave_incl_scan(nd, lane);
      const int d0 = incl - nd;
      const unsigned mag = diff < 0 ? 0u - (unsigned)diff : (unsigned)diff;
      const int e = diff ? 31 - __builtin_clz(mag) : 0;
      const int prev = wave_prev(raddr);
      const int prev2 = wave_prev(prev);
      // e = 10, 11: the composed N rows of slots 10 and 31 (ffv1_walk)
      const uint32_t mrows = e >= 10 && e <= 11 ? (((e == 11 ? 3u : 6u) << 12) | (((mag >> 9) & 3u) << 28)) : 0u;
      const uint32_t w = (uint32_t)d0 | ((uint32_t)(d0 + 2 * e) << 16) | (lane > 0 && prev == raddr ? kRecSame : 0u) |
                         (lane > 1 && prev2 == raddr ? kRecSame2 : 0u) | mrows;
      if (valid) rec[idx] = make_uint2((uint32_t)raddr | ((uint32_t)(uint16_t)diff << 16), w);
      // the chunk's decision bits, packed in coding order, and its header
      const int wv = threadIdx.x / kWave;
      uint32_t* const cs = cstage[wv];
      if (base + wv * kWave < n) {
        cs[lane] = 0u;
        if (lane < cw - kWave) cs[kWave + lane] = 0u;
        if (valid) {
          const uint64_t x = decision_bits(diff) << (d0 & 31);
          atomicOr(&cs[1 + (d0 >> 5)], (uint32_t)x);
          if ((uint32_t)(x >> 32)) atomicOr(&cs[2 + (d0 >> 5)], (uint32_t)(x >> 32));
        }
        const int total = __builtin_amdgcn_readlane(incl, kWave - 1);
        const bool lng = __ballot(valid && (diff >= 4096 || diff <= -4096)) != 0;
        const uint64_t mm = __ballot(valid && (diff >= 1024 || diff <= -1024) && diff < 4096 && diff > -4096);
        if (lane == 0) cs[0] = (uint32_t)total | (lng ? kChunkLong : 0u) | (mm ? kChunkMulti : 0u);
        if (lane < 2) cs[cw - 2 + lane] = (uint32_t)(mm >> (32 * lane));
        // out: the header, the words the decisions fill and the two after
        // them (ffv1_bits reads a chunk's words up to the one its last
        // decision lands in at its stream offset, which may be one more),
        // and the mask words; the rest of the 70 stay unwritten (zero words:
        // ~3 of every 4 written before, 10 GB a c3 step)
        uint32_t* const dst = cbase + ((base + wv * kWave) / kWave) * cw;
        const int last = min(cw - 3, (total >> 5) + 2);
        if (lane < cw && (lane <= last || lane >= cw - 2)) dst[lane] = cs[lane];
        const int w2 = kWave + lane;
        if (w2 < cw && (w2 <= last || w2 >= cw - 2)) dst[w2] = cs[w2];
      }
    } else if (valid) {
      out[RGB ? ((int64_t)y * a.nplanes + p) * pw + x : idx] = ((uint32_t)(row0 + ctx) << 16) | (uint16_t)diff;
    }
  }
  if (count && b0 < b1) {
    for (int o = 32; o > 0; o >>= 1) ndec += __shfl_xor(ndec, o);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = ndec;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
      for (int w = 0; w < kSymThreads / kWave; w++) t += red[w];
      atomicAdd(count, t);
    }
    __syncthreads();  // red[] is reused by the next item
  }
  }
}

// ---------------------------------------------------------------------------
// Kernel 2: SIMT range coder.
//
// Everything on the per-decision path is branch-free: a data-dependent scalar
// branch costs ~66 cycles on gfx950 (tools/ubench), more than the ~20 VALU
// ops of a whole decision, and with 64 independent streams per wave some lane
// renormalises on almost every decision anyway.
constexpr int kRing = 96;        // renorm digits per lane held in LDS before a flush
constexpr int kRingStride = kRing + 5;  // [lane][kRing + 5]: odd, so lanes at equal heads hit distinct banks
constexpr int kFlushAt = kRing - 69;    // checked every second symbol step (<= 34 digits per symbol)
constexpr int kHeaderFlushAt = kRing - 30;  // per header op (host-checked |value| < 2^14: <= 29 digits)

// Keeps a value's computation where it is written: without it the compiler
// sinks the successor-state lookups of lanes that may be idle into an
// exec-masked block behind a branch, which costs more than the lookups.
__device__ __forceinline__ void pin(uint32_t& v) { asm volatile("" : "+v"(v)); }

// Debug build: is [p, p + n) inside [base, base + bytes)?  If not, the first
// failing site is recorded and the caller drops the write (ffv1_internal.h,
// Bounds).  The release build folds every call to true.
__device__ __forceinline__ bool bounds_ok(const Bounds& b, const void* p, int64_t n, const void* base,
                                          int64_t bytes, uint32_t site) {
  if constexpr (!kBoundsCheck) return true;
  const int64_t o = (int64_t)(reinterpret_cast<const uint8_t*>(p) - reinterpret_cast<const uint8_t*>(base));
  if (o >= 0 && n >= 0 && o + n <= bytes) return true;
  if (b.err) atomicCAS(b.err, 0u, site);
  return false;
}

// LDS-typed pointer (address space 3): ring arithmetic stays 32-bit LDS
// addressing, with no generic-pointer conversions on the per-decision path
typedef __attribute__((address_space(3))) uint32_t lds_u32;

struct Lane {
  int low, range;
  uint32_t r0, r1, r2, r3, r4, r5, r6, r7;  // states of the current context row (byte k = slot k)
  lds_u32* ring;       // this lane's ring row (LDS)
  lds_u32* rp;         // ring head: the digits so far are ring[0 .. rp - ring)

  template <int D>
  __device__ __forceinline__ uint32_t& w() {
    static_assert(D >= 0 && D < 8, "row word");
    if constexpr (D == 0) return r0;
    else if constexpr (D == 1) return r1;
    else if constexpr (D == 2) return r2;
    else if constexpr (D == 3) return r3;
    else if constexpr (D == 4) return r4;
    else if constexpr (D == 5) return r5;
    else if constexpr (D == 6) return r6;
    else return r7;
  }
};

// Byte writer: renorm_encoder's outstanding-byte / 0xFF-run logic
// (rangecoder.h:52-75) replayed over the recorded values of `low`, without
// per-lane branches: every digit but the first and those of a 0xFF run
// emits the outstanding byte (+1 on a carry), a run's fill bytes follow in
// a rare wave-level loop.  Bytes gather in a dword; a full one is stored.
struct Sink {
  uint8_t* out;
  int64_t cap, opos;  // opos: bytes stored, a multiple of 4
  uint32_t ow;        // bytes not yet stored, the oldest in the low byte
  int on, pending, run;

  __device__ __forceinline__ void put(uint32_t b, bool en) {
    ow |= en ? (b & 0xFFu) << (on << 3) : 0u;
    on += en ? 1 : 0;
    if (on == 4) {
      if (opos + 4 <= cap) *reinterpret_cast<uint32_t*>(out + opos) = ow;
      opos += 4;
      ow = 0;
      on = 0;
    }
  }
  // one recorded `low` (act: this lane has it), as qv = low >> 8 and whether
  // its low byte is non-zero: low is in (0xFF00, 0x10000) iff qv is 0xFF and
  // it is
  __device__ __forceinline__ void digit(int low, bool act) { digit_q(low >> 8, (low & 0xFF) != 0, act); }
  __device__ __forceinline__ void digit_q(int qv, bool lownz, bool act) {
    const bool first = pending < 0;
    const bool isrun = !first && qv == 0xFF && lownz;
    const bool emit = act && !first && !isrun;
    const int c = qv >> 8;  // carry into the outstanding byte
    put((uint32_t)(pending + c), emit);
    if (__ballot(emit && run > 0)) {  // a run of 0xFF digits ends: its bytes, 0xFF or 0x00 after a carry
      const uint32_t fill = c ? 0x00u : 0xFFu;
      for (int r = 0; __ballot(emit && r < run); r++) put(fill, emit && r < run);
    }
    pending = act && (first || emit) ? (qv & 0xFF) : pending;
    run = act && isrun ? run + 1 : (emit ? 0 : run);
  }
  // bytes so far (ff_rac_terminate's count once the terminate digits are in)
  __device__ __forceinline__ int64_t finish() {
    for (int k = 0; k < on; k++)
      if (opos + k < cap) out[opos + k] = (uint8_t)(ow >> (k << 3));
    return opos + on;
  }
};

__device__ __forceinline__ Sink make_sink(uint8_t* out, int64_t cap) {
  Sink s;
  s.out = out;
  s.cap = cap;
  s.opos = 0;
  s.ow = 0;
  s.on = 0;
  s.pending = -1;
  s.run = 0;
  return s;
}

// Renormalisation (range < 0x100 needs at most one shift after a decision):
// the value of `low` is always written at the ring head and the head only
// advances when a byte is really shifted out.
// One byte-permute selector does both shifts: (x & 0xFF) << 8 when a byte is
// shifted out (range < 0x100, so that is range << 8 too), x as it is
// otherwise.
__device__ __forceinline__ void renorm(Lane& L) {
  const bool need = L.range < 0x100;
  *L.rp = (uint32_t)L.low;
  L.rp += need ? 1 : 0;
  const uint32_t sel = need ? 0x0c0c000cu : 0x03020100u;
  L.low = (int)__builtin_amdgcn_perm(0u, (uint32_t)L.low, sel);
  L.range = (int)__builtin_amdgcn_perm(0u, (uint32_t)L.range, sel);
}

// Every lane replays its ring, four entries read at a time (ring rows are 3
// entries longer than the ring).
__device__ __forceinline__ void flush(Lane& L, Sink& S) {
  const int n = (int)(L.rp - L.ring);
  for (int t = 0; __ballot(t < n); t += 4) {
    const uint32_t d0 = L.ring[t], d1 = L.ring[t + 1], d2 = L.ring[t + 2], d3 = L.ring[t + 3];
    S.digit((int)d0, t < n);
    S.digit((int)d1, t + 1 < n);
    S.digit((int)d2, t + 2 < n);
    S.digit((int)d3, t + 3 < n);
  }
  L.rp = L.ring;
}

template <class SinkT>
__device__ __forceinline__ void flush_if(Lane& L, SinkT& S, int above) {
  if (__ballot((int)(L.rp - L.ring) > above)) flush(L, S);
}

__device__ __forceinline__ void rac_core(Lane& L, int s, int bit) {
  const int r1 = (int)(__umul24((unsigned)L.range, (unsigned)s) >> 8);  // range < 2^16, s < 2^8
  const int r0 = L.range - r1;
  L.low += bit ? r0 : 0;
  L.range = bit ? r1 : r0;
}

// put_rac (rangecoder.h:90-102) on lanes where `act`, leaving the others.
__device__ __forceinline__ void rac_sel(Lane& L, bool act, int s, int bit) {
  const int r1 = (int)(__umul24((unsigned)L.range, (unsigned)s) >> 8);  // range < 2^16, s < 2^8
  const int r0 = L.range - r1;
  const int nl = L.low + (bit ? r0 : 0);
  const int nr = bit ? r1 : r0;
  L.low = act ? nl : L.low;
  L.range = act ? nr : L.range;
  renorm(L);
}

// One decision on the static slot K of the current row, successor inserted.
template <int K>
__device__ __forceinline__ void step(Lane& L, bool act, int bit, const uint8_t* tab) {
  constexpr int D = K >> 2, SH = (K & 3) * 8;
  const uint32_t w = L.w<D>();
  const int s = (w >> SH) & 0xFF;
  rac_sel(L, act, s, bit);
  const uint32_t ns = tab[(bit << 8) | s];
  L.w<D>() = act ? ((w & ~(0xFFu << SH)) | (ns << SH)) : w;
}

// Batched form (no slot repeats inside the symbol, e <= 9): the decision
// reads the old state and issues its successor lookup; the caller inserts
// all successors after the last decision, so no LDS latency sits between
// two decisions.
template <int K>
__device__ __forceinline__ uint32_t step_b(Lane& L, bool act, int bit, const uint8_t* tab) {
  constexpr int D = K >> 2, SH = (K & 3) * 8;
  const int s = (L.w<D>() >> SH) & 0xFF;
  rac_sel(L, act, s, bit);
  return tab[(bit << 8) | s];
}

template <int K>
__device__ __forceinline__ void insert_b(Lane& L, bool act, uint32_t ns) {
  constexpr int D = K >> 2, SH = (K & 3) * 8;
  const uint32_t w = L.w<D>();
  L.w<D>() = act ? ((w & ~(0xFFu << SH)) | (ns << SH)) : w;
}

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// The sign decision's slot 11 + min(e,10) varies per lane (dwords 2..5).
// Mask selects (not ternaries): a select between members would be folded
// into an indexed load and push the whole Lane into scratch.
struct SignSlot {
  uint32_t m2, m3, m4, m5;
  int sh;
  __device__ __forceinline__ SignSlot(int k) {
    const int d = k >> 2;
    sh = (k & 3) * 8;
    m2 = 0u - (uint32_t)(d == 2);
    m3 = 0u - (uint32_t)(d == 3);
    m4 = 0u - (uint32_t)(d == 4);
    m5 = 0u - (uint32_t)(d == 5);
  }
  __device__ __forceinline__ int get(const Lane& L) const {
    const uint32_t w = (L.r2 & m2) | (L.r3 & m3) | (L.r4 & m4) | (L.r5 & m5);
    return (w >> sh) & 0xFF;
  }
  __device__ __forceinline__ void put(Lane& L, bool act, uint32_t ns) const {
    const uint32_t msk = ~(0xFFu << sh), val = ns << sh;
    const uint32_t g2 = act ? m2 : 0u, g3 = act ? m3 : 0u, g4 = act ? m4 : 0u, g5 = act ? m5 : 0u;
    L.r2 = (((L.r2 & msk) | val) & g2) | (L.r2 & ~g2);
    L.r3 = (((L.r3 & msk) | val) & g3) | (L.r3 & ~g3);
    L.r4 = (((L.r4 & msk) | val) & g4) | (L.r4 & ~g4);
    L.r5 = (((L.r5 & msk) | val) & g5) | (L.r5 & ~g5);
  }
};

// put_symbol_inline (ffv1enc.c:185-231) for a wave whose largest exponent is
// EM <= 9: zero flag (slot 0), unary exponent (slots 1..e+1), mantissa MSB
// first (slots 22+i), sign (slot 11+e).  Fully unrolled for EM.  Activity is
// written as comparisons on e alone (e = -1 for a zero or idle lane): with a
// shared `nz &&` factor the compiler wraps the inserts in an exec-masked branch.
template <int EM>
__device__ __forceinline__ void code_symbol(Lane& L, bool act, bool nz, int v, unsigned mag, int e,
                                            const uint8_t* tab) {
  const uint32_t n0 = step_b<0>(L, act, v == 0, tab);
  if constexpr (EM >= 0) {
    uint32_t nu[EM + 1], nm[EM + 1], nsg;
    static_for<0, EM + 1>([&](auto ic) {
      constexpr int I = decltype(ic)::value;
      nu[I] = step_b<1 + I>(L, I <= e, I < e, tab);
    });
    static_for<0, EM>([&](auto ic) {
      constexpr int I = EM - 1 - decltype(ic)::value;
      nm[I] = step_b<22 + I>(L, I < e, (mag >> I) & 1, tab);
    });
    const SignSlot sg(11 + max(e, 0));
    {
      const int ss = sg.get(L);
      const int bit = v < 0;
      rac_sel(L, e >= 0, ss, bit);
      nsg = tab[(bit << 8) | ss];
    }
    insert_b<0>(L, act, n0);
    static_for<0, EM + 1>([&](auto ic) {
      constexpr int I = decltype(ic)::value;
      insert_b<1 + I>(L, I <= e, nu[I]);
    });
    static_for<0, EM>([&](auto ic) {
      constexpr int I = decltype(ic)::value;
      insert_b<22 + I>(L, I < e, nm[I]);
    });
    sg.put(L, e >= 0, nsg);
  } else {
    insert_b<0>(L, act, n0);
  }
}

// Any exponent (slots 10 and 31 repeat beyond e = 9): serial updates.
__device__ __forceinline__ void code_symbol_long(Lane& L, bool act, bool nz, int v, unsigned mag, int e,
                                              int emax, const uint8_t* tab) {
  step<0>(L, act, v == 0, tab);
  static_for<0, 10>([&](auto ic) {
    constexpr int I = decltype(ic)::value;
    step<1 + I>(L, nz && I <= e, I < e, tab);
  });
  for (int i = 10; i <= emax; i++) step<10>(L, nz && i <= e, i < e, tab);
  for (int i = emax - 1; i >= 10; i--) step<31>(L, nz && i < e, (mag >> i) & 1, tab);
  static_for<0, 10>([&](auto ic) {
    constexpr int I = 9 - decltype(ic)::value;
    step<22 + I>(L, nz && I < e, (mag >> I) & 1, tab);
  });
  const SignSlot sg(11 + min(max(e, 0), 10));
  const int ss = sg.get(L);
  const int bit = v < 0;
  rac_sel(L, nz, ss, bit);
  sg.put(L, nz, tab[(bit << 8) | ss]);
}

__device__ __forceinline__ int wave_max(int v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}

// Wave-uniform max of x in [0, 31] from five ballots (no shuffles, no branches).
__device__ __forceinline__ int wave_max5(int x) {
  int m = 0;
#pragma unroll
  for (int b = 4; b >= 0; b--) {
    const int t = m | (1 << b);
    m = __ballot(x >= t) ? t : m;
  }
  return __builtin_amdgcn_readfirstlane(m);
}

// Generic decision on a per-lane LDS state (header ops; rare).
__device__ __forceinline__ void put_lds(Lane& L, uint8_t* st, int bit, const uint8_t* tab) {
  const int s = *st;
  rac_core(L, s, bit);
  *st = tab[(bit << 8) | s];
  renorm(L);
}

__device__ __forceinline__ void symbol_lds(Lane& L, uint8_t* st, int v, bool sgn, const uint8_t* tab) {
  if (v == 0) {
    put_lds(L, st, 1, tab);
    return;
  }
  const unsigned a = v < 0 ? 0u - (unsigned)v : (unsigned)v;
  const int e = 31 - __builtin_clz(a);
  put_lds(L, st, 0, tab);
  for (int i = 0; i < e; i++) put_lds(L, st + 1 + min(i, 9), 1, tab);
  put_lds(L, st + 1 + min(e, 9), 0, tab);
  for (int i = e - 1; i >= 0; i--) put_lds(L, st + 22 + min(i, 9), (a >> i) & 1, tab);
  if (sgn) put_lds(L, st + 11 + min(e, 10), v < 0, tab);
}

__device__ __forceinline__ void store_row(const Lane& L, uint8_t* row) {
  reinterpret_cast<uint4*>(row)[0] = make_uint4(L.r0, L.r1, L.r2, L.r3);
  reinterpret_cast<uint4*>(row)[1] = make_uint4(L.r4, L.r5, L.r6, L.r7);
}

constexpr int kCodeThreads = kWave;
constexpr int kOpsetBytes = kOpSets * 32;

// Key bit / in-band v0/v1 header / v3 slice header (per-lane op program).
// os: this lane's op-set states (osb bytes); flush_at: the ring's flush
// threshold before each op (<= 29 digits per op).
// Ops [q0, q1) of the lane's program; the op states reset at q0 == 0.  pcm:
// v4's slice_coding_mode 1 (the PCM re-code): the mode ops code 1 and the RCT
// symbols are left out (ffv1enc.c:1054-1060).
template <class SinkT>
__device__ __forceinline__ void run_header_ops(const CodeArgs& a, Lane& L, SinkT& S, uint8_t* os, int key,
                                               int slice, bool live, const uint8_t* dtab,
                                               const uint8_t* ftab, int osb, int flush_at, int f,
                                               int q0 = 0, int q1 = kMaxOps, bool pcm = false) {
  // fresh op states (encode_slice_header's state[32] = 128, ffv1enc.c:1031);
  // slice 0's PCM re-run (q0 past the key bit) keeps only the key bit's set 0
  if (q0 == 0 || pcm)
    for (int i = q0 == 0 ? 0 : 32; i < osb; i++) os[i] = 128;
  const int sel = key * a.nslices + slice;
  const int n = live ? min(a.nops[sel], q1) : 0;
  const Op* ops = a.ops + (int64_t)sel * kMaxOps;
  for (int q = 0; q < a.max_ops; q++) {
    if (q >= q0 && q < n) {
      const Op op = ops[q];
      const uint8_t* t = op.tab ? ftab : dtab;
      uint8_t* st = os + op.set * 32;
      int v = op.value;
      if (op.kind == kOpSymRct) {  // v4: the frame's slice RCT coefficient
        const int2 co = a.rct[(int64_t)f * a.nslices + slice];
        v = op.value ? co.y : co.x;
      }
      if (op.kind == kOpBitMode || op.kind == kOpSymMode) v = pcm ? 1 : 0;
      if (op.kind == kOpBit || op.kind == kOpBitMode)
        put_lds(L, st, v, t);
      else if (!(pcm && op.kind == kOpSymRct))
        symbol_lds(L, st, v, op.kind == kOpSymS, t);
    }
    flush_if(L, S, flush_at);
  }
}

// A v4 PCM sample (encode_line's slice_coding_mode 1, ffv1enc.c:294-304):
// coded plane p of the slice at (x, y), untransformed: YCbCr the stored
// sample; RGB (encode_rgb_frame, :419-445) g, b, r, a from the bgr0 / RGB32
// word or the gbrp planes read in AVFrame data[] order as b, g, r.
__device__ __forceinline__ int pcm_sample(const CodeArgs& a, const SliceGeom& g, int f, int p, int x, int y) {
  const uint8_t* fr = a.frames + (int64_t)f * a.frame_bytes;
  if (a.rgb) {
    const int X = g.px[0] + x, Y = g.py[0] + y;
    if (a.sample_bytes == 4) {
      const uint32_t v = reinterpret_cast<const uint32_t*>(fr + a.plane_off[0] + (int64_t)Y * a.plane_stride[0])[X];
      return p == 0 ? (int)((v >> 8) & 0xFF) : p == 1 ? (int)(v & 0xFF) : p == 2 ? (int)((v >> 16) & 0xFF)
                                                                              : (int)(v >> 24);
    }
    const int src = p == 0 ? 1 : p == 1 ? 0 : 2;  // g from data[1], b from data[0], r from data[2]
    return reinterpret_cast<const uint16_t*>(fr + a.plane_off[src] + (int64_t)Y * a.plane_stride[src])[X];
  }
  const uint16_t v =
      reinterpret_cast<const uint16_t*>(fr + a.plane_off[p] + (int64_t)(g.py[p] + y) * a.plane_stride[p])[g.px[p] + x];
  return a.packed_at_lsb ? (int)v : (int)(v >> a.msb_shift);
}

__device__ __forceinline__ void lane_init(Lane& L, uint32_t* ring) {
  L.low = 0;
  L.range = 0xFF00;
  L.ring = (lds_u32*)ring;
  L.rp = L.ring;
  L.r0 = L.r1 = L.r2 = L.r3 = L.r4 = L.r5 = L.r6 = L.r7 = 0;
}

// slice end: a 0 decision on state 129, then ff_rac_terminate
template <class SinkT>
__device__ __forceinline__ int64_t terminate(Lane& L, SinkT& S, bool state129, int ring) {
  flush_if(L, S, ring - 4);
  if (state129) {
    rac_core(L, 129, 0);
    renorm(L);
  }
  L.range = 0xFF;
  L.low += 0xFF;
  renorm(L);
  L.range = 0xFF;
  renorm(L);
  flush(L, S);
  return S.finish();
}

// Pass 1 (ffv1enc.c:190-199, 315-321): every decision of a plane symbol
// counted by the state it is coded with and by (context, slot), from the
// row's states before the symbol (each slot codes once per symbol but slots
// 10 and 31, whose later decisions see the states their earlier ones left).
// Plain global atomics: pass 1 is a statistics run, not the timed path.
// (mask selects, as SignSlot: a ternary chain over the members with a run-time
// k became an indexed load, which put the whole Lane in scratch memory for
// every decision of the kernel, pass 1 or not)
__device__ __forceinline__ uint32_t row_byte(const Lane& L, int k) {
  const int d = k >> 2;
  auto m = [&](int i) { return 0u - (uint32_t)(d == i); };
  const uint32_t w = (L.r0 & m(0)) | (L.r1 & m(1)) | (L.r2 & m(2)) | (L.r3 & m(3)) | (L.r4 & m(4)) |
                     (L.r5 & m(5)) | (L.r6 & m(6)) | (L.r7 & m(7));
  return (w >> ((k & 3) * 8)) & 0xFFu;
}

__device__ void count_symbol(const CodeArgs& a, const Lane& L, int v, int ctx, const uint8_t* tab) {
  unsigned long long* const st2 = a.rc_stat2 + (int64_t)ctx * 64;
  auto cnt = [&](int slot, int bit, uint32_t s) {
    atomicAdd(a.rc_stat + s * 2 + bit, 1ull);
    atomicAdd(st2 + slot * 2 + bit, 1ull);
  };
  if (v == 0) {
    cnt(0, 1, row_byte(L, 0));
    return;
  }
  const unsigned mag = v < 0 ? 0u - (unsigned)v : (unsigned)v;
  const int e = 31 - __builtin_clz(mag);
  uint32_t s10 = row_byte(L, 10), s31 = row_byte(L, 31);
  cnt(0, 0, row_byte(L, 0));
  for (int i = 0; i < e; i++) {
    const int slot = 1 + min(i, 9);
    const uint32_t s = slot == 10 ? s10 : row_byte(L, slot);
    cnt(slot, 1, s);
    if (slot == 10) s10 = tab[256 | s10];
  }
  {
    const int slot = 1 + min(e, 9);
    cnt(slot, 0, slot == 10 ? s10 : row_byte(L, slot));
  }
  for (int i = e - 1; i >= 0; i--) {
    const int slot = 22 + min(i, 9), bit = (mag >> i) & 1;
    const uint32_t s = slot == 31 ? s31 : row_byte(L, slot);
    cnt(slot, bit, s);
    if (slot == 31) s31 = tab[(bit << 8) | s31];
  }
  const int sslot = 11 + min(e, 10);
  cnt(sslot, v < 0, row_byte(L, sslot));
}

// One lane per (segment, slice) chain coding frame j of every segment, the
// chain's states carried in `tables` from frame to frame.
__host__ __device__ constexpr size_t code_lds_bytes(int lanes) {
  return 1024 + (size_t)lanes * (kOpsetBytes + kRingStride * 4);
}

__global__ __launch_bounds__(kCodeThreads) void ffv1_code(CodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint8_t* const tabs = lds;
  uint8_t* const opsets = lds + 1024;                                               // [lane][kOpsetBytes]
  uint32_t* const ring = reinterpret_cast<uint32_t*>(opsets + kCodeThreads * kOpsetBytes);  // [lane][stride]
  for (int i = threadIdx.x; i < 1024; i += kCodeThreads) tabs[i] = a.tabs[i];
  __syncthreads();
  const uint8_t* dtab = tabs;        // default table (key bit, v0/v1 header)
  const uint8_t* ftab = tabs + 512;  // frame table

  const int lane = threadIdx.x;
  // a.cpw chains per wave, on lanes 0 .. cpw-1 (a symbol costs the wave its
  // chains' largest exponent, and a batch of few chains leaves SIMDs idle);
  // the other lanes run idle on a dummy table, so their row stores touch no
  // chain's.  Tables exist for the chains padded to 64.
  const bool mine = lane < a.cpw;
  const int64_t chain = (int64_t)blockIdx.x * a.cpw + (mine ? lane : 0);
  const int seg_i = (int)(chain / a.nslices);
  const int slice = (int)(chain % a.nslices);
  bool live = mine && seg_i < a.nsegs;
  Segment seg{0, 0, 0, 0};
  if (live) seg = a.segs[seg_i];
  live = live && a.j < seg.nframes;
  const int f = seg.first_frame + a.j;
  uint8_t* const table = a.tables + (mine ? chain : a.table_dummy + (blockIdx.x & 63)) * a.state_bytes;
  const int key = live ? a.keyflags[f] : 0;

  // context states: continue, or reset at a keyframe (ff_ffv1_clear_slice_state)
  if (live) {
    if (a.j == 0 && seg.load_states) {
      const uint4* src = reinterpret_cast<const uint4*>(a.persist_in + (int64_t)slice * a.state_bytes);
      for (int64_t i = 0; i < a.state_bytes / 16; i++) reinterpret_cast<uint4*>(table)[i] = src[i];
    } else if (key && a.init) {  // ff_ffv1_clear_slice_state with 2-pass initial states
      const uint4* src = reinterpret_cast<const uint4*>(a.init);
      const int64_t per = a.state_bytes / (16 * a.pcount);  // uint4s of one plane context's table
      for (int64_t i = 0; i < a.state_bytes / 16; i++) reinterpret_cast<uint4*>(table)[i] = src[i % per];
    } else if (key) {
      const uint4 v = make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);
      for (int64_t i = 0; i < a.state_bytes / 16; i++) reinterpret_cast<uint4*>(table)[i] = v;
    }
  }

  Lane L;
  lane_init(L, ring + lane * kRingStride);
  uint8_t* const out = a.slice_out + ((int64_t)(live ? f : 0) * a.nslices + slice) * a.slice_stride;
  Sink S = make_sink(out, live ? a.slice_cap : 0);  // idle lanes write nothing

  // v4: the coder as encode_slice finds it (c_bak, ffv1enc.c:1157), after
  // slice 0's key bit: the PCM re-code restarts from there
  const int split = a.v4pcm && slice == 0 ? 1 : 0;
  uint8_t* const myops = opsets + lane * kOpsetBytes;
  run_header_ops(a, L, S, myops, key, slice, live, dtab, ftab, kOpsetBytes, kHeaderFlushAt, live ? f : 0, 0,
                 a.v4pcm ? split : kMaxOps);
  Lane Lb = L;
  Sink Sb = S;
  if (a.v4pcm) {
    flush(L, S);
    Lb = L;
    Sb = S;
    run_header_ops(a, L, S, myops, key, slice, live, dtab, ftab, kOpsetBytes, kHeaderFlushAt, live ? f : 0, split);
  }

  const SliceGeom& g = a.geom[slice];
  const int64_t nsym = live ? g.nsym : 0;
  const int contexts = (int)(a.state_bytes / (32 * a.pcount));  // rows per plane context (pass-1 counts)
  // v4: encode_line's check at every line start (ffv1enc.c:282-286): fewer
  // than 35 * w bytes left in the slice's buffer (the bytes written so far,
  // renorm_encoder's outstanding byte and 0xFF run not counted) fails the
  // slice, which is then coded again as PCM.  v4 planes all have the luma
  // width (4:4:4 or RGB), so lines start every pw[0] symbols.
  const int lw = g.pw[0];
  const int64_t v4_limit = (slice == 0 ? a.v4_cap0 : a.v4_cap) - 35 * (int64_t)lw;
  bool failed = false;
  const int64_t nmax = wave_max((int)nsym);
  // g.sym_off and frame_samples are multiples of 4 (host-side padding);
  // idle lanes read group 0 of slot 0
  const uint4* sp = reinterpret_cast<const uint4*>(live ? a.sym + (int64_t)seg_i * a.frame_samples + g.sym_off
                                                        : a.sym);
  const int64_t glast = nsym > 0 ? (nsym - 1) >> 2 : 0;

  uint4 G = sp[0], GN = sp[min((int64_t)1, glast)];
  int cur = nsym > 0 ? (int)(G.x >> 16) : 0;
  {
    const uint4* r = reinterpret_cast<const uint4*>(table + (int64_t)cur * 32);
    const uint4 ra = r[0], rb = r[1];
    L.r0 = ra.x; L.r1 = ra.y; L.r2 = ra.z; L.r3 = ra.w;
    L.r4 = rb.x; L.r5 = rb.y; L.r6 = rb.z; L.r7 = rb.w;
  }
  uint4 PFa = make_uint4(0, 0, 0, 0), PFb = make_uint4(0, 0, 0, 0);
  flush_if(L, S, kFlushAt);

  auto sym_step = [&](int64_t ii, uint32_t sv, uint32_t sn) {
    if (a.v4pcm) {
      const bool ls = ii < nsym && !failed && ii % lw == 0;
      if (__ballot(ls)) flush(L, S);
      failed = failed || (ls && S.opos + S.on > v4_limit);
    }
    const bool act = ii < nsym && !failed;
    const int row = act ? (int)(sv >> 16) : cur;
    const bool sw = row != cur;  // context switch: take the prefetched row
    L.r0 = sw ? PFa.x : L.r0; L.r1 = sw ? PFa.y : L.r1; L.r2 = sw ? PFa.z : L.r2; L.r3 = sw ? PFa.w : L.r3;
    L.r4 = sw ? PFb.x : L.r4; L.r5 = sw ? PFb.y : L.r5; L.r6 = sw ? PFb.z : L.r6; L.r7 = sw ? PFb.w : L.r7;
    cur = row;
    {  // prefetch the next symbol's row (stale and unused when it is this row)
      const int nrow = ii + 1 < nsym ? (int)(sn >> 16) : cur;
      const uint4* r = reinterpret_cast<const uint4*>(table + (int64_t)nrow * 32);
      PFa = r[0];
      PFb = r[1];
    }
    const int v = (int16_t)(sv & 0xFFFF);
    if (a.rc_stat && act) count_symbol(a, L, v, row - row / contexts * contexts, ftab);
    const bool nz = act && v != 0;
    const unsigned mag = v < 0 ? 0u - (unsigned)v : (unsigned)v;
    const int e = nz ? 31 - __builtin_clz(mag) : -1;
    // (one chain per wave: lane 0's own exponent, the idle lanes' being -1)
    const int emax = (a.cpw == 1 ? __builtin_amdgcn_readfirstlane(e + 1) : wave_max5(e + 1)) - 1;
    switch (emax) {
      case -1: code_symbol<-1>(L, act, nz, v, mag, e, ftab); break;
      case 0: code_symbol<0>(L, act, nz, v, mag, e, ftab); break;
      case 1: code_symbol<1>(L, act, nz, v, mag, e, ftab); break;
      case 2: code_symbol<2>(L, act, nz, v, mag, e, ftab); break;
      case 3: code_symbol<3>(L, act, nz, v, mag, e, ftab); break;
      case 4: code_symbol<4>(L, act, nz, v, mag, e, ftab); break;
      case 5: code_symbol<5>(L, act, nz, v, mag, e, ftab); break;
      case 6: code_symbol<6>(L, act, nz, v, mag, e, ftab); break;
      case 7: code_symbol<7>(L, act, nz, v, mag, e, ftab); break;
      case 8: code_symbol<8>(L, act, nz, v, mag, e, ftab); break;
      case 9: code_symbol<9>(L, act, nz, v, mag, e, ftab); break;
      default: code_symbol_long(L, act, nz, v, mag, e, emax, ftab); break;
    }
    store_row(L, table + (int64_t)cur * 32);  // write back every step: no divergent store
  };

  for (int64_t i = 0, gi = 0; i < nmax; i += 4, gi++) {
    sym_step(i, G.x, G.y);
    sym_step(i + 1, G.y, G.z);
    flush_if(L, S, kFlushAt);
    sym_step(i + 2, G.z, G.w);
    sym_step(i + 3, G.w, GN.x);
    flush_if(L, S, kFlushAt);
    G = GN;
    GN = sp[min(gi + 2, glast)];
  }

  if (__ballot(failed)) {
    // the PCM re-code (ffv1enc.c:1207-1217): the coder as it was before the
    // slice header, the header with slice_coding_mode 1 (which clears the
    // slice's context states, :1054-1055), then every sample's bits MSB
    // first on a fresh state 128 each (:294-304), with the same per-line
    // buffer check (the reference asserts when that fails too)
    if (failed) {
      L = Lb;
      L.rp = L.ring;
      S = Sb;
    }
    run_header_ops(a, L, S, myops, key, slice, failed, dtab, ftab, kOpsetBytes, kHeaderFlushAt, live ? f : 0,
                   split, kMaxOps, true);
    if (failed) {
      const uint4 v = make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);
      const int64_t per = a.state_bytes / (16 * a.pcount);
      for (int64_t i = 0; i < a.state_bytes / 16; i++)
        reinterpret_cast<uint4*>(table)[i] = a.init ? reinterpret_cast<const uint4*>(a.init)[i % per] : v;
    }
    const int np = a.nplanes;
    const int64_t npcm = failed ? nsym : 0;
    bool again = false;
    for (int64_t ii = 0; __ballot(ii < npcm); ii++) {
      const bool act = ii < npcm;
      const bool ls = act && ii % lw == 0;
      if (__ballot(ls)) flush(L, S);
      again = again || (ls && S.opos + S.on > v4_limit);
      // symbol ii of the slice in coding order: RGB rows interleave the
      // planes (row, plane, x), YCbCr planes follow each other
      const int64_t line = ii / lw;
      const int x = (int)(ii - line * lw);
      const int p = a.rgb ? (int)(line % np) : (int)(line / g.ph[0]);
      const int y = a.rgb ? (int)(line / np) : (int)(line % g.ph[0]);
      const int v = act ? pcm_sample(a, g, f, p, x, y) : 0;
      for (int i = a.pcm_bits - 1; i >= 0; i--) {
        rac_core(L, act ? 128 : 0, (v >> i) & 1);
        renorm(L);
      }
      flush_if(L, S, kRing - 20);
    }
    if (again) {  // the reference's av_assert0(slice_coding_mode == 0) (ffv1enc.c:1209)
      atomicAdd(a.status + 2, 1);
    }
  }

  if (live) {
    const int64_t nbytes = terminate(L, S, true, kRing);
    if (nbytes > a.slice_cap) {
      atomicAdd(a.status, 1);
      atomicMax(a.status + 1, (int)nbytes);
    }
    a.slice_bytes[(int64_t)f * a.nslices + slice] = min(nbytes, a.slice_cap);  // never past the slot
    if (a.j == seg.nframes - 1 && seg.save_states) {
      uint4* dst = reinterpret_cast<uint4*>(a.persist_out + (int64_t)slice * a.state_bytes);
      for (int64_t i = 0; i < a.state_bytes / 16; i++) dst[i] = reinterpret_cast<const uint4*>(table)[i];
    }
  }
}

// ---------------------------------------------------------------------------
// Kernel 2, decision-stream form: every (frame, slice) stream of the batch,
// the states ffv1_walk recorded and the bits ffv1_bits placed, in three
// passes.  put_rac (rangecoder.h:85-102) makes `range` a function of
// (range, state, bit) alone: r1 = range * state >> 8, then range - r1 (a 0)
// or r1 (a 1), renormalised by << 8 while below 0x100; `low` never feeds
// back into it.  So:
//
//   ffv1_range  one lane per stream walks `range` only (about half the
//               work of a full put_rac per decision: this serial chain is
//               what sets the coder's time) and stores, at the start of
//               every segment of kSeg decisions, {range, shifts so far}.
//   ffv1_dseg   every segment codes in parallel from its checkpoint with
//               low = 0, writing the value of low at each of its shifts
//               (renorm_encoder's input, a "digit") at its place in the
//               stream, and its low at the end.
//   ffv1_dfix   one lane per stream joins the segments in order.  Only
//               additions and << 8 shifts act on low, so the real low is
//               the local one plus what entered from the previous segments;
//               that carry-in (< 2^17) is out of the 16-bit window after two
//               shifts, so it changes the segment's first two digits only.
//
// ffv1_sink then replays renorm_encoder's outstanding-byte logic over the
// digits as before, and the bytes are those of the serial coder.

// the first rem state bytes of a 16-byte block (rem may be <= 0 or >= 16)
__device__ __forceinline__ uint32_t tail_word(uint32_t w, int rem) {
  return rem >= 4 ? w : rem <= 0 ? 0u : (w & ((1u << (8 * rem)) - 1u));
}
__device__ __forceinline__ uint4 tail_mask(const uint4& v, int rem) {
  return make_uint4(tail_word(v.x, rem), tail_word(v.y, rem - 4), tail_word(v.z, rem - 8), tail_word(v.w, rem - 12));
}

// state byte J of a block of 32 (two uint4)
template <int J>
__device__ __forceinline__ uint32_t state_word(const uint4& wa, const uint4& wb) {
  if constexpr (J < 4) return wa.x;
  else if constexpr (J < 8) return wa.y;
  else if constexpr (J < 12) return wa.z;
  else if constexpr (J < 16) return wa.w;
  else if constexpr (J < 20) return wb.x;
  else if constexpr (J < 24) return wb.y;
  else if constexpr (J < 28) return wb.z;
  else return wb.w;
}

// The decision masks of 8 decisions (all ones for a 1), made opaque to the
// compiler together: seen as a sign-extended bit, a mask would be turned
// into a compare + v_cndmask (with its vcc wait states) instead of one
// bitwise select, and an empty asm per decision costs a wait state each.
struct Masks8 {
  int m[8];
};
template <int G>
__device__ __forceinline__ Masks8 masks8(uint32_t bw) {
  Masks8 k;
  static_for<0, 8>([&](auto jc) {
    constexpr int J = decltype(jc)::value;
    k.m[J] = __builtin_amdgcn_sbfe((int)bw, 8 * G + J, 1);
  });
  asm volatile("" : "+v"(k.m[0]), "+v"(k.m[1]), "+v"(k.m[2]), "+v"(k.m[3]), "+v"(k.m[4]), "+v"(k.m[5]),
               "+v"(k.m[6]), "+v"(k.m[7]));
  return k;
}

// 32 decisions on `range` alone; shifts counts the renormalisations (x 8).  A
// state-0 decision of bit 0 (the zeroed tail of a stream) leaves range as
// it is: r1 = 0, range - r1 = range.
// (Measured slower: put_rac's two outcomes as one multiply-add, P = range *
// (bit ? s : 256 - s) + (bit ? 0 : 255), renormalised by a compare on P: a
// three-deep chain per decision instead of seven, but more instructions, and
// the pass is issue-bound: 72 vs 63 ms alone at 21 GOPs.)
__device__ __forceinline__ void range32(int& range, int& shifts, const uint4& wa, const uint4& wb, uint32_t bw) {
  static_for<0, 4>([&](auto gc) {
    constexpr int G = decltype(gc)::value;
    const Masks8 k = masks8<G>(bw);
    static_for<0, 8>([&](auto jc) {
      constexpr int J = 8 * G + decltype(jc)::value;
      constexpr int SH = (J & 3) * 8;
      const uint32_t w = state_word<J>(wa, wb);
      const int m = k.m[J & 7];
      const int r1 = (int)(__umul24((unsigned)range, (w >> SH) & 0xFFu) >> 8);
      const int d = range - r1;
      const int nr = (m & r1) | (~m & d);  // m ? r1 : d, one bitwise select
      // renormalisation without a compare: nr in [1, 0xFFFF] has 16..31
      // leading zeros, 24 or more (bit 3 set) exactly when nr < 0x100
      const int sh = (int)(__builtin_clz((unsigned)nr) & 8u);
      shifts += sh;  // in units of 8
      range = nr << sh;
    });
  });
}

// The stream a lane codes: slice-major, so that the lanes of a wave code one
// slice of consecutive frames (streams of similar length).
struct StreamRef {
  bool live;
  int slice, f;
  int64_t st;  // [frame][slice] index of the per-stream arrays
};
__device__ __forceinline__ StreamRef stream_of(const CodeArgs& a, int64_t c) {
  StreamRef r;
  r.live = c < (int64_t)a.nframes * a.nslices;
  r.slice = r.live ? (int)(c / a.nframes) : 0;
  r.f = r.live ? (int)(c % a.nframes) : 0;
  r.st = (int64_t)r.f * a.nslices + r.slice;
  return r;
}

constexpr int kRangeThreads = kWave;
__device__ __forceinline__ void set_prio(int p) {
  switch (p) {
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    case 3: __builtin_amdgcn_s_setprio(3); break;
    default: break;
  }
}

// The range pass over stream lane c: the luma chain's decisions, then the
// chroma chain's at their own start.  pass 0: both; 1: the luma chain, its
// final {range, shifts} kept in rstate; 2: the chroma chain from there (the
// coder's dseg of the luma segments runs beside it, ffv1_range_dseg).
template <int AHEAD>
__device__ __forceinline__ void range_pass(const CodeArgs& a, int64_t c, int pass) {
  const StreamRef sr = stream_of(a, c);
  const int key = sr.live ? a.keyflags[sr.f] : 0;
  const HdrState h = a.hdr[key * a.nslices + sr.slice];
  const int* dc = a.ds.dcount + sr.st * 3;
  const int64_t base = sr.live ? a.ds.dbase[sr.st] : 0;  // a multiple of kStreamAlign
  const StreamSegs ss = sr.live ? a.segs_info[sr.st] : StreamSegs{0, 0, 0, 0};
  uint2* ck = a.ck + ss.seg_base + (pass == 2 ? ss.s_luma : 0);
  int range = h.range, shifts = h.ndig << 3;  // renormalisation shifts x 8
  if (pass == 2 && sr.live) {
    const int2 r = a.rstate[sr.st];
    range = r.x;
    shifts = r.y;
  }
  for (int part = pass == 2 ? 1 : 0; part < (pass == 1 ? 1 : 2); part++) {
    const int n = sr.live ? (part ? dc[1] + dc[2] : dc[0]) : 0;
    const int64_t pb = base + (part && sr.live ? chroma_start(dc[0]) : 0);  // multiple of 512
    const uint4* P = reinterpret_cast<const uint4*>(a.ds.pre + pb);
    const uint32_t* B = a.ds.bits + (pb >> 5);
    const int nmax = wave_max(n);
    // groups of four 32-decision blocks (32 state bytes + one bits word
    // each), the next group's loads issued while this one codes: 128-256
    // decisions ahead, enough to cover the memory latency with dseg's
    // streams beside it (chains are padded: reads stay inside the stream)
    // (AHEAD = 2: the next two groups, 256-384 decisions ahead, where the
    // registers are there: the range pass alone, one wave per SIMD)
    const uint4 z4 = make_uint4(0, 0, 0, 0);
    uint4 ca4[4], cb4[4], na4[4], nb4[4], ma4[4], mb4[4];
    uint32_t cw4[4], nw4[4], mw4[4];
    auto fetch = [&](int g, uint4* A, uint4* Bq, uint32_t* Wq) {
      static_for<0, 4>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        const int blk = g * 4 + J;
        A[J] = P[2 * blk];
        Bq[J] = P[2 * blk + 1];
        Wq[J] = B[blk];
      });
    };
    static_for<0, 4>([&](auto jc) {
      constexpr int J = decltype(jc)::value;
      ca4[J] = cb4[J] = na4[J] = nb4[J] = ma4[J] = mb4[J] = z4;
      cw4[J] = nw4[J] = mw4[J] = 0u;
    });
    if (n > 0) fetch(0, ca4, cb4, cw4);
    if (AHEAD > 1 && n > 128) fetch(1, na4, nb4, nw4);
    for (int i = 0; i < nmax; i += 128) {
      if (AHEAD > 1) {
        if (i + 256 < n) fetch((i >> 7) + 2, ma4, mb4, mw4);
      } else {
        if (i + 128 < n) fetch((i >> 7) + 1, na4, nb4, nw4);
      }
      static_for<0, 4>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        const int ii = i + 32 * J;
        if (ii < nmax) {  // wave-uniform
          if ((ii & (kSeg - 1)) == 0 && ii < n) *ck++ = make_uint2((uint32_t)range, (uint32_t)shifts >> 3);
          uint4 wa = ca4[J], wb = cb4[J];
          uint32_t bw = cw4[J];
          const int rem = n - ii;
          if (rem < 32) {
            wa = tail_mask(wa, rem);
            wb = tail_mask(wb, rem - 16);
            bw = rem > 0 ? bw & ((1u << rem) - 1u) : 0u;
          }
          range32(range, shifts, wa, wb, bw);
        }
      });
      static_for<0, 4>([&](auto jc) {
        constexpr int J = decltype(jc)::value;
        ca4[J] = na4[J];
        cb4[J] = nb4[J];
        cw4[J] = nw4[J];
        if (AHEAD > 1) {
          na4[J] = ma4[J];
          nb4[J] = mb4[J];
          nw4[J] = mw4[J];
        }
      });
    }
  }
  if (pass == 1 && sr.live) a.rstate[sr.st] = make_int2(range, shifts);
}

__global__ __launch_bounds__(kRangeThreads) void ffv1_range(CodeArgs a) {
  if (ds_over(a.ds)) {  // the batch is encoded again: flagged for the host (status[3])
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.status + 3, 1);
    return;
  }
  set_prio(a.range_prio);
  range_pass<2>(a, (int64_t)blockIdx.x * kRangeThreads + threadIdx.x, a.range_pass);
}

// ffv1_dseg: one wave per 64 consecutive segments of a stream, one lane per
// segment; no LDS, so that its waves fit beside the next batch's states walk
// (which holds the CUs' LDS).  The values of low at the shifts go straight
// to the stream's digit area (u32), at the stream-wide shift index the
// checkpoint gives.
constexpr int kDsegThreads = kWave;

// Where a segment's digits go: a buffer resource over its stream's digit
// area (the wave's 64 segments are one stream's) and the byte offset of the
// lane's next digit.  The hardware drops the stores of a stream running past
// its slot (the join then reports the overflow).
struct DigitOut {
  __amdgpu_buffer_rsrc_t rs;
  int kb;
};

// put_rac + renorm_encoder's shift (rangecoder.h:52-102): the value of low
// before a shift is stored as the lane's next digit.
__device__ __forceinline__ void put_dec(int& low, int& range, DigitOut& o, int s, int m) {
  const int r1 = (int)(__umul24((unsigned)range, (unsigned)s) >> 8);
  const int d = range - r1;
  low += d & m;
  const int nr = (m & r1) | (~m & d);  // m ? r1 : d, one bitwise select
  // a byte shifts out (nr < 0x100): one compare, whose VCC the selects
  // below read.  (A mask from the leading-zero count, as in range32, made
  // the compiler rebuild the same VCC for the low select and cost three
  // more VALU per decision: 17 vs 14.)
  const bool sh = nr < 0x100;
  // the store of the lanes that shift (an exec-masked store; issuing it for
  // every lane with an out-of-range offset for the others loaded the
  // address path with 64 lanes per decision: 19.23 -> 19.40 Gpix/s)
  if (sh) __builtin_amdgcn_raw_buffer_store_b32((uint32_t)low, o.rs, o.kb, 0, 0);
  o.kb += sh ? 4 : 0;
  low = sh ? (int)__builtin_amdgcn_perm(0u, (uint32_t)low, 0x0c0c000cu) : low;  // (low & 0xFF) << 8
  range = sh ? nr << 8 : nr;
}

// The segments of waves vb, vb + vgrid, ... (part: -1 all, 0 the luma
// chain's, 1 the chroma chain's; the other lanes idle).
__device__ __forceinline__ void dseg_body(const CodeArgs& a, int vb, int vgrid, int only_part) {
  const int lane = threadIdx.x;
  const int ngroups = a.seg_totals[1];
  for (int w = vb; w < ngroups; w += vgrid) {
    const int st = a.wmap[w];  // wave-uniform
    const StreamSegs ss = a.segs_info[st];
    const int s = (w - ss.wave_base) * kDsegThreads + lane;  // this lane's segment of the stream
    const int part = s >= ss.s_luma ? 1 : 0;
    const bool act = s < ss.s_all && (only_part < 0 || part == only_part);
    if (__ballot(act) == 0) continue;  // (wave-uniform) none of this group's segments in the part
    const int* dc = a.ds.dcount + (int64_t)st * 3;
    const int sp = part ? s - ss.s_luma : s;
    const int npart = part ? dc[1] + dc[2] : dc[0];
    const int off = sp * kSeg;
    int n = act ? min(kSeg, npart - off) : 0;
    const bool last = act && s == ss.s_all - 1;
    const int64_t cb = a.ds.dbase[st] + (part ? chroma_start(dc[0]) : 0);  // the chain's first decision
    const int64_t pb = cb + off;  // multiple of 64
    const uint2 ck = act ? a.ck[ss.seg_base + s] : make_uint2(0x100u, 0u);
    int range = (int)ck.x, low = 0;
    // the segment's digits: stream-wide shift index ck.y; stores past the
    // slot are dropped (the join sees the overflow and the batch is encoded
    // again with a larger budget)
    DigitOut o;
    o.rs = __builtin_amdgcn_make_buffer_rsrc(a.slice_out + (int64_t)st * a.slice_stride, 0,
                                            (int)(a.digit_cap * 4), kBufDword3);
    o.kb = (int)ck.y * 4;
    const int kb0 = o.kb;
    if constexpr (kBoundsCheck) {
      if (act && !bounds_ok(a.bnd, a.slice_out + (int64_t)st * a.slice_stride, a.digit_cap * 4, a.slice_out,
                            a.bnd.out_bytes, kBndDsegSlot))
        o.rs = __builtin_amdgcn_make_buffer_rsrc(a.slice_out, 0, 0, kBufDword3);  // every store dropped
      // the blocks it reads: inside its chain and pad (the chain's extent as the layout made it)
      const int64_t clen = chain_extent(npart);
      const int64_t rb = (int64_t)(n + 127) / 128 * 128;
      if (act && (!bounds_ok(a.bnd, a.ds.pre + pb, rb, a.ds.pre + cb, clen, kBndDsegRead) ||
                  !bounds_ok(a.bnd, a.ds.pre + pb, rb, a.ds.pre, a.bnd.pre_bytes, kBndDsegRead)))
        n = 0;
    }
    const uint4* P = reinterpret_cast<const uint4*>(a.ds.pre + pb);
    const uint4* B4 = reinterpret_cast<const uint4*>(a.ds.bits + (pb >> 5));  // 64-byte aligned (kStreamAlign)
    const int nmax = wave_max(n);
    // Blocks of 128 decisions: a whole 128-byte line of states per lane, the
    // next block's loaded while this one codes, and the decision bits of
    // four blocks (64 bytes) at a time, the next four's loaded a group
    // ahead.  The 64 lanes of a wave read 64 segments 4 KB apart, so a line
    // read a part at a time is fetched from HBM again for each part: states
    // 16-32 bytes at a time took 185 GB per launch for 34 GB of states and
    // bits, then whole state lines with 16 bytes of bits per block 71 GB.
    const uint4 z4 = make_uint4(0, 0, 0, 0);
    uint4 cur[8], nxt[8];
    uint4 bg[4], nbg[4];  // bits: this group of four blocks, the next group
    auto fetch = [&](int blk, uint4* q) {
      static_for<0, 8>([&](auto jc) { q[decltype(jc)::value] = P[blk * 8 + decltype(jc)::value]; });
    };
    static_for<0, 8>([&](auto jc) { cur[decltype(jc)::value] = nxt[decltype(jc)::value] = z4; });
    static_for<0, 4>([&](auto jc) { bg[decltype(jc)::value] = nbg[decltype(jc)::value] = z4; });
    if (n > 0) {  // (chains are padded to 512 decisions and more: reads stay inside the stream)
      fetch(0, cur);
      static_for<0, 4>([&](auto jc) { nbg[decltype(jc)::value] = B4[decltype(jc)::value]; });
    }
    for (int i = 0; i < nmax; i += 128) {
      const int q = (i >> 7) & 3;  // wave-uniform
      if (q == 0) {
        static_for<0, 4>([&](auto jc) { bg[decltype(jc)::value] = nbg[decltype(jc)::value]; });
        if (i + 512 < n) static_for<0, 4>([&](auto jc) { nbg[decltype(jc)::value] = B4[(i >> 7) + 4 + decltype(jc)::value]; });
      }
      if (i + 128 < n) fetch((i >> 7) + 1, nxt);
      // this block's bits are bg[0]; the group's others move up (a select
      // on q, wave-uniform as it is, became an indexed load from scratch)
      const uint4 b4 = bg[0];
      bg[0] = bg[1];
      bg[1] = bg[2];
      bg[2] = bg[3];
      const uint32_t cbw[4] = {b4.x, b4.y, b4.z, b4.w};
      static_for<0, 4>([&](auto sc) {
        constexpr int S = decltype(sc)::value;
        uint4 wa = cur[2 * S], wb = cur[2 * S + 1];
        uint32_t bw = cbw[S];
        const int rem = n - (i + 32 * S);
        if (rem < 32) {
          wa = tail_mask(wa, rem);
          wb = tail_mask(wb, rem - 16);
          bw = rem > 0 ? bw & ((1u << rem) - 1u) : 0u;
        }
        static_for<0, 4>([&](auto gc) {
          constexpr int G = decltype(gc)::value;
          const Masks8 k = masks8<G>(bw);
          static_for<0, 8>([&](auto jc) {
            constexpr int J = 8 * G + decltype(jc)::value;
            const uint32_t sw = state_word<J>(wa, wb);
            put_dec(low, range, o, (int)((sw >> ((J & 3) * 8)) & 0xFFu), k.m[J & 7]);
          });
        });
      });
      static_for<0, 8>([&](auto jc) { cur[decltype(jc)::value] = nxt[decltype(jc)::value]; });
    }
    if (last) {  // a 0 on state 129, then ff_rac_terminate (ffv1enc.c:1331-1334, rangecoder.c:104-116)
      {  // the trailer decision: at most one shift
        const int r1 = (int)(__umul24((unsigned)range, 129u) >> 8);
        range -= r1;
        if (range < 0x100) {
          __builtin_amdgcn_raw_buffer_store_b32((uint32_t)low, o.rs, o.kb, 0, 0);
          o.kb += 4;
          low = (low & 0xFF) << 8;
          range <<= 8;
        }
      }
      low += 0xFF;
      __builtin_amdgcn_raw_buffer_store_b32((uint32_t)low, o.rs, o.kb, 0, 0);  // range = 0xFF: one shift
      low = (low & 0xFF) << 8;
      __builtin_amdgcn_raw_buffer_store_b32((uint32_t)low, o.rs, o.kb + 4, 0, 0);  // range = 0xFF again
      low = (low & 0xFF) << 8;
      o.kb += 8;
    }
    if (act) a.segrec[ss.seg_base + s] = make_uint2((uint32_t)low, (uint32_t)((o.kb - kb0) >> 2));
  }
}

__global__ __launch_bounds__(kDsegThreads) void ffv1_dseg(CodeArgs a) {
  if (ds_over(a.ds)) return;
  set_prio(a.dseg_prio);
  dseg_body(a, blockIdx.x, gridDim.x, a.dseg_part);
}

// The chroma chains' range pass and the luma segments' dseg in one launch:
// blocks [0, range_blocks) continue every stream's range from its luma end
// (rstate), the rest code the luma segments, whose checkpoints the first
// range pass left.  The two roles share no data and never wait for each
// other; on one stream, so no fifth hardware queue (an extra stream for the
// same overlap serialised).
__global__ __launch_bounds__(kRangeThreads) void ffv1_range_dseg(CodeArgs a) {
  if (ds_over(a.ds)) return;
  if ((int)blockIdx.x < a.range_blocks) {
    set_prio(a.range_prio);
    range_pass<2>(a, (int64_t)blockIdx.x * kRangeThreads + threadIdx.x, 2);
  } else {
    set_prio(a.dseg_prio);
    dseg_body(a, (int)blockIdx.x - a.range_blocks, (int)gridDim.x - a.range_blocks, 0);
  }
}

// ffv1_dfix: one lane per stream.  The header's digits (fixed per key and
// slice, computed on the host) go first; then, segment by segment, with L
// the real low entering it and v, u its local lows at its first two shifts:
// the real lows there are x = L + v and u + ((x & 0xFF) - (v & 0xFF)) << 8
// (the window after the first shift is (low & 0xFF) << 8), and the low
// leaving it is its own from the second shift on, L + its local low when it
// has no shift.
constexpr int kFixThreads = kWave;
__global__ __launch_bounds__(kFixThreads) void ffv1_dfix(CodeArgs a) {
  const int64_t st = (int64_t)blockIdx.x * kFixThreads + threadIdx.x;
  if (ds_over(a.ds) || a.status[3]) return;  // skipped by the walk and the coder (ffv1_range flagged it)
  if (st >= (int64_t)a.nframes * a.nslices) return;
  const int f = (int)(st / a.nslices), slice = (int)(st % a.nslices);
  const HdrState h = a.hdr[a.keyflags[f] * a.nslices + slice];
  const StreamSegs ss = a.segs_info[st];
  uint32_t* const out = reinterpret_cast<uint32_t*>(a.slice_out + st * a.slice_stride);
  const int64_t cap = a.digit_cap;
  if (!bounds_ok(a.bnd, out, 4 * max(cap, (int64_t)h.ndig), a.slice_out, a.bnd.out_bytes, kBndDfixSlot) ||
      !bounds_ok(a.bnd, out, 4 * (int64_t)h.ndig, out, 4 * cap, kBndDfixSlot))
    return;
  for (int k = 0; k < h.ndig; k++) out[k] = a.hdr_digits[h.off + k];
  int L = h.low;
  int64_t total = h.ndig;
  const uint2* ck = a.ck + ss.seg_base;
  const uint2* sr = a.segrec + ss.seg_base;
  for (int s = 0; s < ss.s_all; s++) {
    const int64_t J = ck[s].y;
    const uint2 r = sr[s];
    const int e = (int)r.x, n = (int)r.y;
    total = J + n;
    if (J + 2 > cap) continue;  // past the slot (dropped): the batch is encoded again
    if (n == 0) {
      L += e;
      continue;
    }
    const int v = (int)out[J];
    const int x = L + v;
    out[J] = (uint32_t)x;
    const int delta = ((x & 0xFF) - (v & 0xFF)) << 8;
    if (n == 1) {
      L = e + delta;
    } else {
      out[J + 1] = out[J + 1] + (uint32_t)delta;
      L = e;
    }
  }
  // over the byte budget (the bytes are the digits but the last one or so):
  // the stores past the slot were dropped and the batch is encoded again
  if (total > a.slice_cap) {
    atomicAdd(a.status, 1);
    atomicMax(a.status + 1, (int)min(total, (int64_t)0x7FFFFFFF));
  }
  a.slice_bytes[st] = min(total, cap);  // digits, until ffv1_sink
}

// The byte writer of the decision-stream coder, one wave per (frame, slice)
// stream.  renorm_encoder (rangecoder.h:52-75) emits, for every digit j but
// the last non-run one and the 0xFF-run digits after it, the byte
// (qv_j + c_j) & 0xFF, where qv_j = low_j >> 8 and c_j is the carry
// (qv_k >> 8) of the first non-run digit k after j (a run digit: low in
// (0xFF00, 0x10000), qv = 0xFF with a non-zero low byte, never the first).
// So 64 digits at a time are turned into bytes in parallel; only the tail of
// a block, from its last non-run digit, waits for the next block with a
// non-run digit.  The bytes go over the digits (byte i never passes digit
// i, which sits at bytes 4i .. 4i+3).
constexpr int kSinkThreads = kWave;
__global__ __launch_bounds__(kSinkThreads) void ffv1_sink(CodeArgs a) {
  if (ds_over(a.ds) || a.status[3]) return;  // a skipped batch (ffv1_range flagged it): no digits to turn into bytes
  const int64_t st = blockIdx.x;
  const int lane = threadIdx.x;
  uint8_t* const out = a.slice_out + st * a.slice_stride;
  const uint32_t* const din = reinterpret_cast<const uint32_t*>(out);  // values of low at the shifts
  const int n = (int)a.slice_bytes[st];  // digits
  const int cap = (int)a.slice_cap;
  if (!bounds_ok(a.bnd, out, cap, a.slice_out, a.bnd.out_bytes, kBndSinkSlot) ||
      !bounds_ok(a.bnd, out, cap, out, a.slice_stride, kBndSinkSlot))
    return;
  int pend = -1;       // the last non-run digit so far: its byte and its run's wait for a carry
  uint32_t pqv = 0u;   // its qv
  uint32_t nx = lane < n ? din[lane] : 0u;
  for (int b = 0; b * kWave < n; b++) {
    const int j = b * kWave + lane;
    const uint32_t d = nx;
    nx = j + kWave < n ? din[j + kWave] : 0u;  // the next block, in flight
    const uint32_t qv = d >> 8;  // low < 2^17
    const bool nonrun = j < n && !(j > 0 && qv == 0xFFu && (d & 0xFFu));
    const uint64_t m = __ballot(nonrun);
    if (!m) continue;  // a run goes on
    __builtin_amdgcn_wave_barrier();  // every lane has read its digit before any byte lands
    const int first = __builtin_ctzll(m), last = 63 - __builtin_clzll(m);
    const uint32_t c0 = __builtin_amdgcn_readlane(qv >> 8, first);
    if (pend >= 0) {  // the waiting byte and its run: 0xFF, or 0x00 after a carry
      const int end = b * kWave + first;
      for (int i = pend + lane; i < end; i += kWave)
        if (i < cap) out[i] = (uint8_t)(i == pend ? (pqv + c0) & 0xFFu : (0xFFu + c0) & 0xFFu);
    }
    const uint64_t after = lane < 63 ? m & (~0ull << (lane + 1)) : 0ull;
    const uint32_t ck = __shfl(qv >> 8, after ? __builtin_ctzll(after) : 0);
    if (lane >= first && lane < last && j < cap) out[j] = (uint8_t)((qv + ck) & 0xFFu);
    pend = b * kWave + last;
    pqv = __builtin_amdgcn_readlane(qv, last);
  }
  if (lane == 0) {
    const int nbytes = pend < 0 ? 0 : pend;
    if (nbytes > cap) {  // the batch is encoded again; the assembly stays inside the slots
      atomicAdd(a.status, 1);
      atomicMax(a.status + 1, nbytes);
    }
    a.slice_bytes[st] = min(nbytes, cap);
  }
}

// ---------------------------------------------------------------------------
// Kernel 2a: context-state walk.  One wave per (segment, slice pair, plane
// group); group 0 = the luma contexts, 1 = the chroma contexts Cb and Cr
// share (ffv1enc.c:1194-1195): independent chains.  Half h = lane / 32 walks
// the chain of slice 2 * pair + h, lane k = lane % 32 owning slot k of the
// current symbol's row (put_symbol_inline, ffv1enc.c:185-231), with its
// group's [contexts][32] states in LDS.  A wave is issue-bound, so two
// chains per instruction stream walk at nearly twice the rate of one; LDS
// (one table per chain) caps chains per CU either way.
//
// Every decision's adaptive state is recorded at the decision's index in the
// stream.  Symbols come in chunks of 64 (ffv1_symbols' records, each with
// the row, 2-bit slot codes and the decision offsets); a chunk's recorded
// bytes are staged in LDS and go out, at the start of the next chunk, as
// whole 16-byte blocks: the bytes before the chunk's first decision are
// carried over from the previous chunk's stage, and the blocks past a
// chain's last decision land in the chain's pad (kChainPad).
//
// Critical path per symbol: one LDS lookup, N[code][state] (code 0/1 a
// decision bit, 2 no decision), plus a select: the next symbol's row states
// are read from LDS a step ahead and, when it is the same row, taken from
// the register just computed instead.
constexpr int kWalkThreads = kWave;
// N[row][state]: rows 0/1 a decision of that bit, 2 none, and the composed
// rows of the slots with several decisions (put_symbol_inline's min(i, 9)
// slots at e = 10, 11): 3 = N0.N1.N1 (slot 10, e = 11), 4..7 = N[b9].N[b10]
// (slot 31 at e = 11, row 4 + 2 b10 + b9; row 6 = N0.N1 is also slot 10 at
// e = 10)
constexpr int kT3Bytes = 8 * 256;
constexpr int kChunk = 64;                   // symbols per chunk (the records' D is chunk-relative)
constexpr int kPreStage = kChunk * 25;       // recorded bytes of a chunk of symbols with e <= 11
constexpr int kRecSlots = kChunk + 3;        // + three read-ahead slots (null records)
constexpr int kPreData = kPreStage + 16;     // a chain's stage: <= 15 bytes carried in, then the chunk
constexpr int kPreHalf = kPreData + 32;      // + one dummy byte per slot
constexpr int kCopyBlocks = 4;               // 16-byte blocks per lane that write a stage out
static_assert(kCopyBlocks * 32 * 16 >= kPreData, "the copy-out covers the stage");
static_assert(kCopyBlocks * 32 * 16 <= kChainPad, "the copy-out stays inside the chain and its pad");

// LDS image of the walk: a fixed part (static, so every offset below is an
// instruction immediate) and the two state tables (dynamic).
constexpr int kLdsN = 0;                                      // u8 [8][256]: a slot's next state (the block's)
constexpr int kLdsRecs = kLdsN + kT3Bytes;                    // wave 0: [2][kRecSlots] records
constexpr int kLdsPre = kLdsRecs + 2 * kRecSlots * 16;        // wave 0: [2][kPreHalf] recorded states
constexpr int kStageBytes = 2 * kRecSlots * 16 + 2 * kPreHalf;  // one wave's records and recorded states
constexpr int kLdsFixed = kLdsN + kT3Bytes + kStageBytes;     // a one-wave block

int64_t walk_lds_bytes_dev(int rows, int rowb);

// Any exponent, one symbol: lane k < 32 of a half applies all decisions of
// slot k in order (slot 10 takes e-8 exponent decisions beyond e = 9, slot
// 31 the mantissa bits >= 9, the sign goes to slot 21) to its state st,
// records the state for each (see walk_step) and returns the new state.
__device__ __forceinline__ int walk_long(int st, const uint8_t* ftab, int v, int k, uint8_t* pre) {
  const unsigned mag = v < 0 ? 0u - (unsigned)v : (unsigned)v;
  const int e = v ? 31 - __builtin_clz(mag) : -1;
  int n = 0, d0 = 0;  // decisions of this slot: indices d0 .. d0+n-1
  if (k == 0) {
    n = 1;
  } else if (v == 0) {
    n = 0;
  } else if (k <= 9) {
    n = k <= e + 1 ? 1 : 0;
    d0 = k;
  } else if (k == 10) {
    n = e >= 9 ? e - 8 : 0;
    d0 = 10;
  } else if (k <= 21) {
    n = k == 11 + min(e, 10) ? 1 : 0;
    d0 = 2 * e + 2;
  } else if (k <= 30) {
    n = k - 22 < e ? 1 : 0;
    d0 = 2 * e + 1 - (k - 22);
  } else {
    n = e >= 10 ? e - 9 : 0;
    d0 = e + 2;
  }
  for (int j = 0; j < n; j++) {
    const int di = d0 + j;
    int bit;
    if (k == 0) bit = v == 0;
    else if (k <= 10) bit = di <= e;
    else if (k <= 21) bit = v < 0;
    else bit = (mag >> (2 * e + 1 - di)) & 1;
    pre[di] = (uint8_t)st;  // the state it is coded with, as walk_step records it
    st = ftab[(bit << 8) | st];
  }
  return st;
}

// per-lane constants of the step
struct WalkLane {
  int k, hsh;         // the lane's slot; D or D+2e
  int kt;             // the slot's byte in a row (k; compact rows: walk_slot_pos, an unused slot the dummy row's byte k)
  uint32_t amask;     // 0xFFFF, 0 for an unused slot of compact rows (its byte is not in the symbol's row)
  int kk;             // kt + this half's table base
  int dummy;          // stage byte of untouched slots
  int msh, mwd, mbase;  // slots 10 / 31: where the record keeps the composed row (code 3)
  int csh;            // multi chunks: the lane's 2-bit code field in its code word
  uint32_t mlo;       // ... all ones: the code word is y (slots 0..15), else z
};

// A symbol as lane k of its chain sees it.
struct StepIn {
  uint32_t code;  // the slot's decision: 0/1 its bit, 2 none
  int pos;        // stage byte of the decision (the lane's dummy byte for none)
  int addr;       // the slot's state byte in the tables
  bool same;      // same row as the previous symbol
  bool same2;     // same row as the previous symbol or the one two back (same decides first)
};

template <bool MULTI = false>
__device__ __forceinline__ StepIn derive(const uint4& r, const WalkLane& W, int kc) {
  StepIn d;
  const int pos = (int)__builtin_amdgcn_ubfe(r.w, W.hsh, 12) + kc;
  if constexpr (MULTI) {  // records of 2-bit codes (expand_codes)
    const uint32_t sel = (r.y & W.mlo) | (r.z & ~W.mlo);  // bitwise: a select of members would go to scratch
    d.code = __builtin_amdgcn_ubfe(sel, W.csh, 2);
    d.pos = d.code == 2u ? W.dummy : pos;
  } else {  // records of slot masks (expand_rec)
    const uint32_t bit = __builtin_amdgcn_ubfe(r.y, W.k, 1);
    const int nd = __builtin_amdgcn_sbfe((int)r.z, W.k, 1);  // all ones: no decision
    // codes 0..2 only (no bit where there is no decision): code = nd & 2 |
    // bit, and a bitwise insert takes the dummy byte (no compare, so no VCC
    // write and the wait states a select of it would need)
    d.code = ((uint32_t)nd & 2u) | bit;
    d.pos = (nd & W.dummy) | (~nd & pos);
  }
  d.addr = (int)(r.x & W.amask) + W.kk;
  d.same = (int)r.w < 0;  // kRecSame
  d.same2 = r.w >= kRecSame2;  // bit 31 or 30: one compare, no mask (same wins in walk_step)
  return d;
}

// In a chunk with e = 10, 11 symbols: code 3 (the slot's several decisions)
// becomes the slot's composed N row, kept in the record (ffv1_symbols), so
// the state chain stays one lookup per symbol.
__device__ __forceinline__ StepIn derive_m(const uint4& r, const WalkLane& W, int kc) {
  StepIn d = derive<true>(r, W, kc);
  const uint32_t rowm = __builtin_amdgcn_ubfe(r.w, W.msh, W.mwd) + W.mbase;
  d.code = d.code == 3u ? rowm : d.code;
  return d;
}

// Symbol T: the lookup of T is issued first; T's recorded state, T-1's
// table write and the read of T+2's row then fill its latency.  The row of
// T+2 is read two symbols ahead, so it misses the writes of T and T+1: a
// symbol continuing its predecessor's row takes that state from the register
// (e1), one on the row of the symbol two back takes that one's (e2).  The
// step's critical path is then one LDS lookup and two selects.
// N[code][state] = the state after the slot's decision (code 0/1 its bit, 2
// none); the state before it is what the coder needs (put_rac's r1 = range *
// state >> 8).
__device__ __forceinline__ void walk_step(uint8_t* fixed, uint8_t* tbl, const StepIn& d, int addr_next2,
                                          uint32_t& e1, uint32_t& e2, uint32_t& l0, uint32_t& l1,
                                          int& addr_prev, uint32_t& st_out) {
  uint32_t a1 = e1, a2 = e2, a0 = l0;
  pin(a1);
  pin(a2);
  pin(a0);
  const uint32_t st = d.same ? a1 : (d.same2 ? a2 : a0);
  const uint32_t idx = (d.code << 8) | st;
  const uint32_t n = fixed[kLdsN + idx];
  fixed[kLdsPre + d.pos] = (uint8_t)st;      // T's recorded state
  tbl[addr_prev] = (uint8_t)a1;              // T-1's state
  l0 = l1;
  l1 = tbl[addr_next2];                      // T+2's row, after every earlier write but T's and T+1's
  addr_prev = d.addr;
  e2 = a1;
  e1 = n;
  st_out = st;
}

// After a chunk with e = 10, 11 symbols: the states the step did not record.
// The step recorded the state before the slot's first decision at pos (slot
// 10: D+10; slot 31: D+2e-8, its LAST decision, e = 11) and advanced the
// chain with the composed row; here, from that state x0, the states before
// the slot's later decisions: slot 10: N1(x0) at D+11 and, at e = 11,
// N1.N1(x0) at D+12; slot 31: x0 at D+13 and N[b10](x0) at D+14
// (put_symbol_inline, ffv1enc.c:199-220).  Lane k of a half takes its
// chain's symbols k and k + 32 (hm: the half's mask), all at once.
__device__ __forceinline__ void walk_multi_fill(uint8_t* fixed, const uint4* myrecs, uint64_t hm, int k, int base,
                                                int dummy) {
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const int t = k + 32 * i;
    const bool act = (hm >> t) & 1u;
    const uint4 r = myrecs[t];
    const int v = (int)(int16_t)(r.x >> 16);
    const unsigned mag = v < 0 ? 0u - (unsigned)v : (unsigned)v;
    const bool e11 = mag >= 2048u;
    const int p10 = base + (int)(r.w & 0xFFFu) + 10;
    const int p31 = base + (int)((r.w >> 16) & 0xFFFu) - 8;
    const uint32_t x10 = fixed[kLdsPre + (act ? p10 : dummy)];
    const uint32_t x31 = fixed[kLdsPre + (act ? p31 : dummy)];
    const uint32_t a1 = fixed[kLdsN + 256 + x10];                     // N1
    const uint32_t a2 = fixed[kLdsN + 7 * 256 + x10];                 // N1.N1
    const uint32_t b1 = fixed[kLdsN + (((mag >> 10) & 1u) << 8) + x31];  // N[b10]
    fixed[kLdsPre + (act ? p10 + 1 : dummy)] = (uint8_t)a1;
    fixed[kLdsPre + (act && e11 ? p10 + 2 : dummy)] = (uint8_t)a2;
    fixed[kLdsPre + (act && e11 ? p31 - 1 : dummy)] = (uint8_t)x31;
    fixed[kLdsPre + (act && e11 ? p31 : dummy)] = (uint8_t)b1;
  }
}

int64_t walk_lds_bytes_dev(int rows, int rowb) { return kLdsFixed + 2 * ((int64_t)rows * rowb + 32); }
// a block of `waves` walk waves: one N table, each wave its stage and two tables
int64_t walk_block_lds_dev(int rows, int waves, int rowb) {
  return kT3Bytes + (int64_t)waves * (kStageBytes + 2 * ((int64_t)rows * rowb + 32));
}

// The 8-byte record in HBM (ffv1_symbols) as the walk's step reads it from
// LDS: the slot masks (y = bits, z = no decision) follow from the residual
// in x (slot_masks), so they are derived here once per chunk instead of
// being stored and read back (16 -> 8 bytes per sample).
__device__ __forceinline__ uint4 expand_rec(const uint2& r) {
  uint32_t bm, nd;
  slot_masks((int)(int16_t)(r.x >> 16), bm, nd);
  return make_uint4(r.x, bm, nd, r.y);
}
// ... and in a chunk with e = 10, 11 symbols as 2-bit codes (slot_codes)
__device__ __forceinline__ uint4 expand_codes(const uint2& r) {
  uint32_t c0, c1;
  slot_codes((int)(int16_t)(r.x >> 16), c0, c1);
  return make_uint4(r.x, c0, c1, r.y);
}

// (Expanding the next chunk's records inside the step loop, in the shadow of
// the lookups, measured slower: 114 -> 131 cycles per step.)

// c ? a : b by value (b in registers, pinned there: a select between a load
// and a local would become a load from a selected address, via scratch).
// Pinning a instead would force a wait for its load right here.
__device__ __forceinline__ uint4 pick(bool c, uint4 a, uint4 b) {
  pin(b.x); pin(b.y); pin(b.z); pin(b.w);
  return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}


// WAVES = 1: one wave per block, items in grid order (a batch of several
// rounds).  WAVES = 4 or 5: one round, a block per CU whose waves 0-3 take a
// long or multi-segment item each and land on the CU's four SIMDs (a
// workgroup's waves go to them in turn), and wave 4 a one-segment item,
// which shares wave 0's SIMD as the younger wave (the arbiter favours the
// older): a wave of full length never shares its SIMD with another walk wave.
// ROWB: bytes per LDS row, 32 or kCompactRowBytes (8 bits: the 24 slots
// put_symbol_inline can use there)
template <int WAVES, int ROWB = 32>
__global__ __launch_bounds__(kWalkThreads * WAVES) void ffv1_walk(WalkArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t fixed[kT3Bytes + WAVES * kStageBytes];
  extern __shared__ __attribute__((aligned(16))) uint8_t tbl[];  // [wave][2][rows + 1 dummy row][32]
  if (ds_over(a.ds)) return;  // the batch is encoded again (uniform: before the barrier)
  const int64_t half = a.state_bytes / 2;  // one plane group's [contexts][32] in the persisted states
  const int64_t thalf = (int64_t)a.rows * ROWB;  // ... and its table in LDS (dense rows: 365 x 32; 8 bits: 666 x 24)
  const int tsz = (int)thalf + 32;
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = WAVES > 1 ? (int)(threadIdx.x >> 6) : 0;
  const int wo = wv * kStageBytes;  // this wave's stage, from wave 0's
  const int h = lane >> 5, k = lane & 31;
  for (int i = threadIdx.x; i < kT3Bytes; i += kWalkThreads * WAVES) {
    const int row = i >> 8, st = i & 255;
    const uint8_t* const t0 = a.ftab;
    const uint8_t* const t1 = a.ftab + 256;
    int v;
    switch (row) {
      case 0: v = t0[st]; break;
      case 1: v = t1[st]; break;
      case 2: v = st; break;
      case 3: v = t0[t1[t1[st]]]; break;
      case 4: v = t0[t0[st]]; break;
      case 5: v = t1[t0[st]]; break;
      case 6: v = t0[t1[st]]; break;
      default: v = t1[t1[st]]; break;
    }
    fixed[kLdsN + i] = (uint8_t)v;
  }
  __syncthreads();  // the block's N table (the only barrier: the waves run independent chains)
  // the longer plane group's chains first (luma at 4:2:0, twice as long as
  // chroma; chroma at 4:4:4, where Cb and Cr make one chain twice luma's),
  // one segment per wave; then the shorter group's: a.short_multi waves (per
  // slice pair) of a.per_short consecutive segments each, so that they walk
  // about as many symbols as a long wave, and the segments left one per wave
  // at the end of the launch, where they land on SIMDs that already hold a
  // walk wave and so run slower, on half the work (walk_split_short)
  // item = (plane group, segment(s), slice pair): the launch may cover a part
  // of the items (launch_walk's first / count)
  const int npairs = (a.nslices + 1) / 2;
  const int nlong = a.nsegs * npairs;
  const int covered = min(a.nsegs, a.short_multi * a.per_short);  // segments the multi waves take
  const int nmulti = a.short_multi * npairs;
  int item;
  if constexpr (WAVES == 1) {
    item = (int)blockIdx.x + a.item0;
  } else {
    const int nfull = nlong + nmulti;
    item = wv < 4 ? 4 * (int)blockIdx.x + wv : nfull + (int)blockIdx.x;
    if (wv < 4 ? item >= nfull : item >= a.nitems) return;  // (after the block's only barrier)
  }
  const SliceGeom& g0 = a.geom[0];
  const bool chroma_first = 2 * (int64_t)g0.pw[1] * g0.ph[1] > (int64_t)g0.pw[0] * g0.ph[0];
  const bool is_long = item < nlong;
  const int grp = is_long == chroma_first ? 1 : 0;  // long: luma (4:2:0) or chroma (4:4:4)
  const int bi = is_long ? item : (item - nlong < nmulti ? item - nlong : item - nlong - nmulti);
  const int pair = bi % npairs, j = bi / npairs;
  int seg_begin, seg_end;  // this wave's segments
  if (is_long) {
    seg_begin = j;
    seg_end = j + 1;
  } else if (item - nlong < nmulti) {
    seg_begin = min(j * a.per_short, covered);
    seg_end = min(seg_begin + a.per_short, covered);
  } else {
    seg_begin = covered + j;
    seg_end = seg_begin + 1;
  }
  const int sl = 2 * pair + h;              // this half's slice
  const bool live = sl < a.nslices;
  const SliceGeom& g = a.geom[live ? sl : 2 * pair];
  const int p0 = grp ? 1 : 0, p1 = grp ? 3 : 1;  // planes of this group's chain
  if (grp && g.plane_sym_off[1] >= g.nsym) return;  // no chroma (uniform: geometry of a frame)
  uint8_t* const mytbl = tbl + (2 * wv + h) * tsz;
  uint4* const myrecs = reinterpret_cast<uint4*>(fixed + kLdsRecs + wo) + h * kRecSlots;
  uint8_t* const stage = fixed + kLdsPre + wo + h * kPreHalf;
  uint4* const stage4 = reinterpret_cast<uint4*>(stage);
  const int64_t n16 = half / 16, t16 = thalf / 16;
  const int64_t goff = grp * half;
  const uint4 v128 = make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);

  WalkLane W;
  W.k = k;
  const bool isU = k <= 10;                // zero flag / exponent slots: decision D + k
  W.hsh = isU ? 0 : 16;                    // else from D + 2e: sign +2, mantissa 22+i: +1-i
  const int kslot = isU ? k : (k <= 21 ? 2 : 23 - k);
  if constexpr (ROWB == 32) {
    W.kt = k;
    W.amask = 0xFFFFu;
  } else {
    const int pk = walk_slot_pos(k);
    W.kt = pk >= 0 ? pk : (int)thalf + k;
    W.amask = pk >= 0 ? 0xFFFFu : 0u;
  }
  W.kk = (2 * wv + h) * tsz + W.kt;
  // one dummy byte per half for the slots without a decision: a shared
  // address, where 32 lanes' distinct bytes made the stage write a 4-way
  // conflict on 8 dwords
  W.dummy = wo + h * kPreHalf + kPreData;
  W.msh = k == 31 ? 28 : 12;
  W.mwd = k == 31 ? 2 : 3;
  W.mbase = k == 31 ? 4 : 0;
  W.csh = (2 * k) & 31;
  W.mlo = k < 16 ? ~0u : 0u;
  const uint4 nullrec = make_uint4((uint32_t)thalf, 0u, ~0u, 0u);  // dummy row, no decisions
  const uint4 nullcodes = make_uint4((uint32_t)thalf, 0xAAAAAAAAu, 0xAAAAAAAAu, 0u);  // ... as codes (2: none)

  // The stage of chunk c goes out at the start of chunk c+1, before its
  // loads are issued: vmcnt counts in issue order, so waiting for chunk
  // c+2's data then never waits for stores just issued.  LDS ops of a wave
  // run in order, so the copy-out reads the stage before chunk c+1's steps
  // write it.  Before the first chunk, and after a chunk recorded straight
  // to HBM, the copy goes to the scratch area.
  uint8_t* pdst = a.scratch;  // 16-aligned
  int plast = 0;              // stage block holding the chunk's last bytes
  auto copy_out = [&]() {
    static_for<0, kCopyBlocks>([&](auto ic) {
      constexpr int I = decltype(ic)::value;
      const uint4 v = stage4[I * 32 + k];
      reinterpret_cast<uint4*>(pdst)[I * 32 + k] = v;
    });
    const uint4 t = stage4[plast];  // the bytes before the next chunk's first decision
    stage4[0] = t;
  };

  // wave priority (run_batch's choice: 0 with the walk in one round, where
  // the coder's range pass is the longer chain and runs above it; the
  // walk_prio hook overrides)
  set_prio(a.prio);
  uint64_t t_loop = 0, n_steps = 0;
  const uint64_t t_all = a.dbg || a.trace ? __builtin_amdgcn_s_memtime() : 0;
  const uint64_t rt_all = a.dbg || a.trace ? __builtin_amdgcn_s_memrealtime() : 0;  // 100 MHz: the wave's shader clock
  for (int seg_i = seg_begin; seg_i < seg_end && seg_i < a.nsegs; seg_i++) {
  const Segment seg = a.segs[seg_i];
  // where the segment's states come from: the carry, the 2-pass initial
  // states (a keyframe), or all 128 (ff_ffv1_clear_slice_state); null: 128
  const uint4* const src = seg.load_states && live
                               ? reinterpret_cast<const uint4*>(a.persist_in + (int64_t)sl * a.state_bytes + goff)
                               : reinterpret_cast<const uint4*>(a.init);
  if constexpr (ROWB == 32) {
    uint4* const t4 = reinterpret_cast<uint4*>(mytbl);
    for (int64_t i = k; i < t16; i += 32) {  // table block i: row i / 2 (dense: its context's)
      const int64_t si = a.dense ? (int64_t)dense_ctx((int)(i >> 1)) * 2 + (i & 1) : i;
      t4[i] = src ? src[si] : v128;
    }
    if (k < 2) t4[t16 + k] = v128;  // dummy row
  } else {  // compact rows (not dense): lane k moves slot k of every row
    const uint8_t* const sb = reinterpret_cast<const uint8_t*>(src);
    if (W.amask)
      for (int r = 0; r < a.rows; r++) mytbl[r * ROWB + W.kt] = src ? sb[r * 32 + k] : (uint8_t)128;
    mytbl[thalf + k] = 128;  // dummy row
  }
  __builtin_amdgcn_wave_barrier();  // (a wave's LDS operations run in order)
  for (int j = 0; j < seg.nframes; j++) {
    const int f = seg.first_frame + j;
    const int64_t sid = (int64_t)f * a.nslices + (live ? sl : 0);
    const int* dc = a.ds.dcount + sid * 3;
    const int64_t gbase = live ? a.ds.dbase[sid] + (grp ? chroma_start(dc[0]) : 0) : 0;  // chain start
    // debug build: the chain's extent, its pad included (the layout's)
    const int64_t gend = !kBoundsCheck || !live ? 0 : gbase + chain_extent(grp ? (int64_t)dc[1] + dc[2] : dc[0]);
    auto in_chain = [&](int64_t off, int64_t n, uint32_t site) {
      return bounds_ok(a.bnd, a.ds.pre + off, n, a.ds.pre + gbase, gend - gbase, site) &&
             bounds_ok(a.bnd, a.ds.pre + off, n, a.ds.pre, a.bnd.pre_bytes, site);
    };
    int64_t run = 0;  // decisions so far in this frame's chain
    for (int pl = p0; pl < p1; pl++) {
      const int64_t nsym = live ? (pl < 2 ? g.plane_sym_off[pl + 1] : g.nsym) - g.plane_sym_off[pl] : 0;
      const uint2* rp = a.rec + (int64_t)f * a.frame_samples + g.sym_off + g.plane_sym_off[pl];
      const uint32_t* cp = a.cbits + ((int64_t)f * a.frame_chunks + g.chunk_off[pl]) * a.cwords;
      const int nch = (int)((nsym + kChunk - 1) / kChunk);
      const int nchunks = max(__builtin_amdgcn_readlane(nch, 0), __builtin_amdgcn_readlane(nch, 32));
      // a chunk's inputs: 2 records per lane and the chunk header
      struct In {
        uint2 m0, m1;
        uint32_t hd, mlo, mhi;  // header, multi-symbol mask
      };
      // raw loads (indices past the plane read record / chunk 0 of a plane of
      // the pair: valid memory); what is past the plane is masked where the
      // data is used, a chunk later: a select here would wait for the loads
      auto load = [&](int c) -> In {
        In x;
        const int64_t b = (int64_t)c * kChunk;
        x.m0 = rp[b + k < nsym ? b + k : 0];
        x.m1 = rp[b + 32 + k < nsym ? b + 32 + k : 0];
        const uint32_t* const ch = cp + (int64_t)(c < nch ? c : 0) * a.cwords;
        x.hd = ch[0];
        x.mlo = ch[a.cwords - 2];
        x.mhi = ch[a.cwords - 1];
        return x;
      };
      In nx = load(0);
      for (int c = 0; c < nchunks; c++) {
        In cx = nx;
        // wait for chunk c's data NOW, while everything older is long done;
        // after the stores and loads below, vmcnt would wait for those too
        pin(cx.m0.x); pin(cx.m0.y);
        pin(cx.m1.x); pin(cx.m1.y);
        pin(cx.hd);
        pin(cx.mlo);
        pin(cx.mhi);
        copy_out();                             // chunk c-1's stage, then ...
        if (c + 1 < nchunks) nx = load(c + 1);  // ... chunk c+1's loads
        const int cnt = (int)min((int64_t)kChunk, max((int64_t)0, nsym - (int64_t)c * kChunk));
        const uint32_t hd = c < nch ? cx.hd : 0u;
        const int total = (int)(hd & ~kChunkFlags);
        const bool lng = __ballot((hd & kChunkLong) != 0) != 0;
        // the symbols with e = 10, 11 of either chain: a wave-uniform mask
        const uint32_t mlo = c < nch ? cx.mlo : 0u, mhi = c < nch ? cx.mhi : 0u;
        const uint64_t msk = ((uint64_t)(__builtin_amdgcn_readlane(mhi, 0) | __builtin_amdgcn_readlane(mhi, 32)) << 32) |
                             (uint64_t)(__builtin_amdgcn_readlane(mlo, 0) | __builtin_amdgcn_readlane(mlo, 32));
        const bool mul = msk != 0 || a.force_multi;
        const int64_t pos0 = gbase + run;  // decision index of the chunk's first decision
        if (!mul) {
          myrecs[k] = pick(k < cnt, expand_rec(cx.m0), nullrec);
          myrecs[k + 32] = pick(k + 32 < cnt, expand_rec(cx.m1), nullrec);
          if (k < kRecSlots - kChunk) myrecs[kChunk + k] = nullrec;
        } else {  // (uniform) the multi step's codes
          myrecs[k] = pick(k < cnt, expand_codes(cx.m0), nullcodes);
          myrecs[k + 32] = pick(k + 32 < cnt, expand_codes(cx.m1), nullcodes);
          if (k < kRecSlots - kChunk) myrecs[kChunk + k] = nullcodes;
        }
        __builtin_amdgcn_wave_barrier();

        if (lng) {  // e >= 12 somewhere: one symbol at a time, recorded straight to HBM
          const int cmax = max(__builtin_amdgcn_readlane(cnt, 0), __builtin_amdgcn_readlane(cnt, 32));
          const bool lok = !kBoundsCheck || !live || in_chain(pos0, (int64_t)total + 16, kBndWalkLong);
          // the next symbol's row is read before this symbol's write (a symbol
          // on its predecessor's row takes the state from the register), so a
          // symbol waits on its transition lookups only
          uint4 r = myrecs[0];
          int st = mytbl[(int)(r.x & W.amask) + W.kt];
          for (int t = 0; t < cmax; t++) {
            const uint4 rn = myrecs[t + 1];
            const int stn = mytbl[(int)(rn.x & W.amask) + W.kt];
            if (t < cnt && lok) {
              st = walk_long(st, fixed + kLdsN, (int)(int16_t)(r.x >> 16), k,
                             a.ds.pre + pos0 + (int)(r.w & 0xFFFu));
              mytbl[(int)(r.x & W.amask) + W.kt] = (uint8_t)st;
            }
            st = (int)rn.w < 0 ? st : stn;
            r = rn;
          }
          // the next chunk's carried bytes: read back what was just written
          __builtin_amdgcn_s_waitcnt(0);
          const uint32_t* src = reinterpret_cast<const uint32_t*>(a.ds.pre + ((pos0 + total) & ~(int64_t)15));
          uint4 tb;
          tb.x = __hip_atomic_load(src + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          tb.y = __hip_atomic_load(src + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          tb.z = __hip_atomic_load(src + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          tb.w = __hip_atomic_load(src + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          stage4[0] = tb;
          pdst = a.scratch;
          plast = 0;
          __builtin_amdgcn_wave_barrier();
          run += total;
          continue;
        }

        const int align = (int)(pos0 & 15);  // stage byte i <-> HBM byte pos0 - align + i
        const int kc = kslot + wo + h * kPreHalf + align;
        StepIn d0 = derive(myrecs[0], W, kc), d1 = derive(myrecs[1], W, kc);
        uint4 rn = myrecs[2];
        uint32_t l0 = tbl[d0.addr], l1 = tbl[d1.addr];
        uint32_t e1 = 0u, e2 = 0u, st = 0u;
        int addr_prev = (int)((stage + kPreData + k) - tbl);  // no T-1 yet: the dummy byte
        const uint64_t t0 = a.dbg || a.trace ? __builtin_amdgcn_s_memtime() : 0;
        if (!mul) {
          static_for<0, kChunk>([&](auto tc) {
            constexpr int T = decltype(tc)::value;
            walk_step(fixed, tbl, d0, (int)(rn.x & W.amask) + W.kk, e1, e2, l0, l1, addr_prev, st);
            const uint4 r3 = myrecs[T + 3];  // three ahead
            __builtin_amdgcn_sched_barrier(0);  // keeps the read here, not sunk to its use a step later
            d0 = d1;
            d1 = derive(rn, W, kc);
            rn = r3;
          });
        } else {  // a symbol with e = 10 or 11 in the chunk: composed rows, then the fill
          StepIn m0 = derive_m(myrecs[0], W, kc), m1 = derive_m(myrecs[1], W, kc);
          static_for<0, kChunk>([&](auto tc) {
            constexpr int T = decltype(tc)::value;
            walk_step(fixed, tbl, m0, (int)(rn.x & W.amask) + W.kk, e1, e2, l0, l1, addr_prev, st);
            const uint4 r3 = myrecs[T + 3];
            __builtin_amdgcn_sched_barrier(0);
            m0 = m1;
            m1 = derive_m(rn, W, kc);
            rn = r3;
          });
          const uint64_t hm = c < nch ? ((uint64_t)cx.mhi << 32) | cx.mlo : 0ull;  // this half's chain
          walk_multi_fill(fixed, myrecs, hm, k, wo + h * kPreHalf + align, W.dummy);
        }
        tbl[addr_prev] = (uint8_t)e1;  // the chunk's last symbol
        if (a.dbg) {
          __builtin_amdgcn_s_waitcnt(0);
          t_loop += __builtin_amdgcn_s_memtime() - t0;
          n_steps += kChunk;
        } else if (a.trace) {  // the step loop's issue time (no wait: the schedule is not disturbed)
          t_loop += __builtin_amdgcn_s_memtime() - t0;
          n_steps += kChunk;
        }
        // one select (a pointer assigned before the bounds check and again
        // inside it once compiled to a register the check had reused)
        bool sok = live;
        if constexpr (kBoundsCheck) sok = sok && in_chain(pos0 & ~(int64_t)15, kCopyBlocks * 32 * 16, kBndWalkStage);
        pdst = sok ? a.ds.pre + (pos0 & ~(int64_t)15) : a.scratch;
        plast = (align + total) >> 4;
        __builtin_amdgcn_wave_barrier();
        run += total;
      }
    }
  }
  copy_out();
  __builtin_amdgcn_wave_barrier();
  pdst = a.scratch;  // the next segment's first copy-out has nothing to write
  plast = 0;
  if (seg.save_states && live &&
      bounds_ok(a.bnd, a.persist_out + (int64_t)sl * a.state_bytes + goff, n16 * 16, a.persist_out,
                a.bnd.persist_bytes, kBndWalkStates)) {
    uint4* dst = reinterpret_cast<uint4*>(a.persist_out + (int64_t)sl * a.state_bytes + goff);
    const uint4* t4 = reinterpret_cast<const uint4*>(mytbl);
    if constexpr (ROWB != 32) {  // compact rows: an unused slot keeps its state (it never codes)
      uint8_t* const db = reinterpret_cast<uint8_t*>(dst);
      const uint8_t* const sb = reinterpret_cast<const uint8_t*>(src);
      for (int r = 0; r < a.rows; r++)
        db[r * 32 + k] = W.amask ? mytbl[r * ROWB + W.kt] : (src ? sb[r * 32 + k] : (uint8_t)128);
    } else if (!a.dense) {
      for (int64_t i = k; i < n16; i += 32) dst[i] = t4[i];
    } else {  // contexts that cannot occur keep the states the segment started from
      for (int64_t i = k; i < n16; i += 32) {
        const int row = dense_row((int)(i >> 1));
        dst[i] = row >= 0 ? t4[row * 2 + (i & 1)] : (src ? src[i] : v128);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();  // the table is read out before the next segment loads its own
  }  // segments of this wave
  if (a.trace && lane == 0) {
    a.trace[item * kTraceWords + 0] = rt_all;
    a.trace[item * kTraceWords + 1] = __builtin_amdgcn_s_memrealtime();
    a.trace[item * kTraceWords + 2] = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_REG_HW_ID
    a.trace[item * kTraceWords + 3] = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // HW_REG_XCC_ID
    a.trace[item * kTraceWords + 4] = t_loop;                                        // step loops, shader cycles
    a.trace[item * kTraceWords + 5] = n_steps;
    a.trace[item * kTraceWords + 6] = __builtin_amdgcn_s_memtime() - t_all;          // the wave, shader cycles
  }
  if (a.dbg && lane == 0) {
    a.dbg[item * 4 + 0] = __builtin_amdgcn_s_memtime() - t_all;
    a.dbg[item * 4 + 1] = t_loop;
    a.dbg[item * 4 + 2] = n_steps;
    a.dbg[item * 4 + 3] = __builtin_amdgcn_s_memrealtime() - rt_all;
  }
}

// Decision-stream layout: stream (frame, slice) i starts at the sum of the
// earlier streams' lengths: the luma chain, its pad, the chroma chain from
// chroma_start, its pad (ffv1_internal.h, DecisionStream).
constexpr int kLayoutThreads = 128;  // 2 KB of LDS: it runs beside the walk, which holds the rest
__global__ __launch_bounds__(kLayoutThreads) void ffv1_layout(const int* dcount, int nstreams, int64_t* dbase,
                                                              int64_t* total, StreamSegs* segs, int* seg_totals,
                                                              int* wmap, int64_t* total_host) {
  __shared__ int64_t part[kLayoutThreads];
  __shared__ int64_t spart[kLayoutThreads];  // segments << 32 | 64-segment groups
  const int t = threadIdx.x;
  const int per = (nstreams + kLayoutThreads - 1) / kLayoutThreads;
  const int lo = min(t * per, nstreams), hi = min(lo + per, nstreams);
  auto len = [&](int i) -> int64_t {
    const int64_t n = (int64_t)dcount[3 * i + 1] + dcount[3 * i + 2];
    return chroma_start(dcount[3 * i]) + chain_extent(n);
  };
  // the coder's segments: the luma chain's, then the chroma chain's (at
  // least one segment, which carries the terminate)
  auto nseg = [&](int i, int* sl) -> int {
    const int64_t nc = (int64_t)dcount[3 * i + 1] + dcount[3 * i + 2];
    const int a = (int)((dcount[3 * i] + kSeg - 1) / kSeg), b = (int)((nc + kSeg - 1) / kSeg);
    *sl = a;
    return max(1, a + b);
  };
  int64_t sum = 0, ssum = 0;
  for (int i = lo; i < hi; i++) {
    int sl;
    const int n = nseg(i, &sl);
    sum += len(i);
    ssum += ((int64_t)n << 32) | (int64_t)((n + 63) / 64);
  }
  part[t] = sum;
  spart[t] = ssum;
  __syncthreads();
  for (int o = 1; o < kLayoutThreads; o <<= 1) {
    const int64_t y = t >= o ? part[t - o] : 0;
    const int64_t z = t >= o ? spart[t - o] : 0;
    __syncthreads();
    part[t] += y;
    spart[t] += z;
    __syncthreads();
  }
  int64_t acc = part[t] - sum, sacc = spart[t] - ssum;
  for (int i = lo; i < hi; i++) {
    dbase[i] = acc;
    acc += len(i);
    int sl;
    const int n = nseg(i, &sl);
    StreamSegs g;
    g.seg_base = (int)(sacc >> 32);
    g.wave_base = (int)(sacc & 0xFFFFFFFF);
    g.s_luma = sl;
    g.s_all = n;
    segs[i] = g;
    for (int k = 0; k < (n + 63) / 64; k++) wmap[g.wave_base + k] = i;
    sacc += ((int64_t)n << 32) | (int64_t)((n + 63) / 64);
  }
  if (t == kLayoutThreads - 1) {
    *total = part[t];
    if (total_host) *total_host = part[t];  // mapped: the host's estimate for later batches
    seg_totals[0] = (int)(spart[t] >> 32);
    seg_totals[1] = (int)(spart[t] & 0xFFFFFFFF);
  }
}

// ---------------------------------------------------------------------------
// Kernel 2c: the decision bits.  ffv1_symbols packed each chunk's bits in
// coding order (word 1 + m = bits 32m .. 32m+31 of the chunk); one block
// per (frame, slice) stream scans the chunks' decision counts in coding
// order (luma, then the chroma chain from chroma_start) and funnel-shifts
// every chunk's words to their place.  A wave takes a run of consecutive
// chunks and carries the word a chunk shares with the next one in a
// register; only the words shared with another wave's run are OR-ed in
// (the array is zeroed first).
constexpr int kBitsThreads = 256;
constexpr int kBitsWaves = kBitsThreads / kWave;
__global__ __launch_bounds__(kBitsThreads) void ffv1_bits(BitsArgs a) {
  __shared__ int off[kBitsThreads];
  __shared__ int tot[kBitsThreads];
  __shared__ int wsum[kBitsWaves];
  if (ds_over(a.ds)) return;  // (uniform: before any barrier)
  const int t = threadIdx.x, lane = t & (kWave - 1), wv = t / kWave;
  // stream sid = frame * nslices + slice, strided over a grid that may be
  // smaller than the streams (a bounded grid: room for the walk beside it)
  for (int64_t sid = blockIdx.x; sid < (int64_t)a.nframes * a.nslices; sid += gridDim.x) {
  const int s = (int)(sid % a.nslices), f = (int)(sid / a.nslices);
  const SliceGeom& g = a.geom[s];
  const int* dc = a.ds.dcount + sid * 3;
  const int64_t base = a.ds.dbase[sid];
  const uint32_t* const fc = a.cbits + (int64_t)f * a.frame_chunks * a.cwords;
  int run = 0;  // stream-relative decision index of the next chunk
  for (int p = 0; p < 3; p++) {
    if (p == 1) run = (int)chroma_start(dc[0]);
    const int64_t nsym = (p < 2 ? g.plane_sym_off[p + 1] : g.nsym) - g.plane_sym_off[p];
    const int nch = (int)((nsym + kChunk - 1) / kChunk);
    const uint32_t* const pc = fc + g.chunk_off[p] * a.cwords;
    for (int c0 = 0; c0 < nch; c0 += kBitsThreads) {
      const int c = c0 + t;
      const int n = c < nch ? (int)(pc[(int64_t)c * a.cwords] & ~kChunkFlags) : 0;
      const int x = wave_incl_scan(n, lane);
      if (lane == kWave - 1) wsum[wv] = x;
      __syncthreads();
      int before = 0, all = 0;
      for (int w = 0; w < kBitsWaves; w++) {
        before += w < wv ? wsum[w] : 0;
        all += wsum[w];
      }
      off[t] = run + before + x - n;
      tot[t] = n;
      __syncthreads();
      // this wave's run of chunks
      const int cn = min(kBitsThreads, nch - c0);
      const int per = (cn + kBitsWaves - 1) / kBitsWaves;
      const int i0 = wv * per, i1 = min(cn, i0 + per);
      uint32_t carry = 0u;  // the previous chunk's last, partial word (lane 0)
      // word m of chunk i: lo/hi = its words m-1 and m (zero outside)
      auto word = [&](int i, int m, int64_t pos, int total, uint32_t hi, uint32_t lo, bool last_of_run,
                      uint32_t& lastw) {
        const int sh = (int)(pos & 31);
        const int nw = (sh + total + 31) >> 5;
        const bool partial = ((sh + total) & 31) != 0;
        uint32_t* const dst = a.ds.bits + (pos >> 5);
        uint32_t v = sh ? __builtin_amdgcn_alignbit(hi, lo, 32 - sh) : hi;
        if (m == 0 && sh) v |= carry;  // zero for the run's first chunk
        const bool shared_head = m == 0 && sh && i == i0;
        const bool tail = m == nw - 1 && partial;
        if (m < nw) {
          if (tail && !last_of_run) {
            // held for the next chunk of the run
          } else if (shared_head || tail) {
            atomicOr(&dst[m], v);
          } else {
            dst[m] = v;
          }
        }
        const int lm = nw - 1;
        if (lm >= (m & ~(kWave - 1)) && lm < (m & ~(kWave - 1)) + kWave)
          lastw = __builtin_amdgcn_readlane(v, lm & (kWave - 1));
      };
      // four chunks' words in flight at a time; the carry then runs through them
      for (int i = i0; i < i1; i += 4) {
        uint32_t H[4], L[4];
        int64_t P[4];
        int T[4], NW[4];
        static_for<0, 4>([&](auto kc) {
          constexpr int K = decltype(kc)::value;
          const bool ok = i + K < i1;
          const int ii = ok ? i + K : i;
          const uint32_t* const q = pc + (int64_t)(c0 + ii) * a.cwords;
          P[K] = base + __builtin_amdgcn_readfirstlane(off[ii]);
          T[K] = ok ? __builtin_amdgcn_readfirstlane(tot[ii]) : 0;
          NW[K] = ((int)(P[K] & 31) + T[K] + 31) >> 5;
          H[K] = lane < NW[K] ? q[1 + lane] : 0u;
          L[K] = lane && lane < NW[K] ? q[lane] : 0u;
        });
        static_for<0, 4>([&](auto kc) {
          constexpr int K = decltype(kc)::value;
          if (i + K < i1) {
            const bool last = i + K + 1 == i1;
            uint32_t lastw = 0u;
            word(i + K, lane, P[K], T[K], H[K], L[K], last, lastw);
            if (NW[K] > kWave) {  // long chunks (e >= 15 symbols): words 64..66
              const uint32_t* const q = pc + (int64_t)(c0 + i + K) * a.cwords;
              const int m = kWave + lane;
              const uint32_t hi = m < NW[K] ? q[1 + m] : 0u;
              const uint32_t lo = m < NW[K] ? q[m] : 0u;
              word(i + K, m, P[K], T[K], hi, lo, last, lastw);
            }
            carry = ((P[K] + T[K]) & 31) ? lastw : 0u;
          }
        });
      }
      run += all;
      __syncthreads();
    }
  }
  }
}

// ---------------------------------------------------------------------------
// Kernel 2b: SIMT Golomb-Rice coder (coder=0; ffv1enc.c:240-370,
// golomb.h:508-563, ffv1.h:192-224), one lane per (segment, slice) chain.
// Per-context VlcState lives in the chain's table as one 8-byte record:
// drift (int16) | error_sum (u16) << 16 | bias (int8) << 32 | count << 40.
__constant__ uint8_t kLog2Run[41] = {
    0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 5, 5, 6,
    6, 7, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24};

struct BitSink {
  uint64_t acc;
  int nacc;
  int64_t pos;  // bytes written
  uint8_t* out;
  int64_t cap;
  __device__ __forceinline__ void put(int n, uint32_t v) {  // put_bits: MSB first
    acc = (acc << n) | v;
    nacc += n;
    while (nacc >= 8) {
      nacc -= 8;
      if (pos < cap) out[pos] = (uint8_t)(acc >> nacc);
      pos++;
    }
    acc &= (1ull << nacc) - 1;
  }
  __device__ __forceinline__ void flush() {  // flush_put_bits: zero pad
    if (nacc) put(8 - nacc, 0);
  }
};

constexpr uint64_t kVlcInit = (uint64_t)4 << 16 | (uint64_t)1 << 40;

__device__ __forceinline__ void vlc_put(BitSink& b, uint64_t& rec, int v, int bits) {
  int drift = (int16_t)(rec & 0xFFFF);
  int error_sum = (int)((rec >> 16) & 0xFFFF);
  int bias = (int8_t)((rec >> 32) & 0xFF);
  int count = (int)((rec >> 40) & 0xFF);
  v = fold_bits(v - bias, bits);
  // k = smallest k with count << k >= error_sum
  int k = max(0, (31 - __builtin_clz((unsigned)max(error_sum, 1))) - (31 - __builtin_clz((unsigned)count)));
  if ((count << k) < error_sum) k++;
  const int code = v ^ ((2 * drift + count) >> 31);
  const unsigned u = code >= 0 ? 2u * (unsigned)code : (unsigned)(-2 * code - 1);
  const unsigned q = u >> k;
  if (q < 12)
    b.put((int)q + k + 1, (1u << k) + (u & ((1u << k) - 1)));
  else
    b.put(12 + bits, u - 11);
  // update_vlc_state
  error_sum = (error_sum + (v < 0 ? -v : v)) & 0xFFFF;
  drift += v;
  if (count == 128) {
    count >>= 1;
    drift >>= 1;
    error_sum >>= 1;
  }
  count++;
  if (drift <= -count) {
    if (bias > -128) bias--;
    drift += count;
    if (drift <= -count) drift = -count + 1;
  } else if (drift > 0) {
    if (bias < 127) bias++;
    drift -= count;
    if (drift > 0) drift = 0;
  }
  rec = (uint64_t)(uint16_t)drift | (uint64_t)(uint16_t)error_sum << 16 |
        (uint64_t)(uint8_t)bias << 32 | (uint64_t)(uint8_t)count << 40;
}

__global__ __launch_bounds__(kCodeThreads) void ffv1_code_golomb(CodeArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t tabs[1024];
  __shared__ __attribute__((aligned(16))) uint8_t opsets[kCodeThreads * kOpsetBytes];
  __shared__ __attribute__((aligned(16))) uint32_t ring[kRingStride * kWave];
  for (int i = threadIdx.x; i < 1024; i += kCodeThreads) tabs[i] = a.tabs[i];
  __syncthreads();
  const int lane = threadIdx.x;
  // a.cpw chains per wave, as ffv1_code (the other lanes idle: they leave
  // after the prefix and never touch a table)
  const int64_t chain = (int64_t)blockIdx.x * a.cpw + (lane < a.cpw ? lane : 0);
  const int seg_i = (int)(chain / a.nslices), slice = (int)(chain % a.nslices);
  bool live = lane < a.cpw && seg_i < a.nsegs;
  Segment seg{0, 0, 0, 0};
  if (live) seg = a.segs[seg_i];
  live = live && a.j < seg.nframes;
  const int f = seg.first_frame + a.j;
  const int key = live ? a.keyflags[f] : 0;
  uint64_t* table = reinterpret_cast<uint64_t*>(a.tables + chain * a.state_bytes);
  const int64_t nrec = a.state_bytes / 32;  // pcount * contexts records
  const int contexts = (int)(nrec / a.pcount);

  if (live) {
    if (a.j == 0 && seg.load_states) {
      const uint64_t* src = reinterpret_cast<const uint64_t*>(a.persist_in + (int64_t)slice * a.state_bytes);
      for (int64_t i = 0; i < nrec; i++) table[i] = src[i];
    } else if (key) {
      for (int64_t i = 0; i < nrec; i++) table[i] = kVlcInit;  // ff_ffv1_clear_slice_state
    }
  }

  // range-coded prefix: key bit / header / slice header, then (v3) a 0 on
  // state 129 and ff_rac_terminate (ffv1enc.c:1173-1183); below version 3
  // only the slice at the origin has one (v2's other slices start with their
  // Golomb bits: they code no decision, and their sink takes no byte)
  const bool prefix = a.version > 2 || slice == 0;
  Lane L;
  lane_init(L, ring + lane * kRingStride);
  uint8_t* const out = a.slice_out + ((int64_t)(live ? f : 0) * a.nslices + slice) * a.slice_stride;
  Sink S = make_sink(out, live && prefix ? a.slice_cap : 0);  // idle lanes write nothing
  run_header_ops(a, L, S, opsets + lane * kOpsetBytes, key, slice, live, tabs, tabs + 512, kOpsetBytes,
                 kHeaderFlushAt, live ? f : 0);
  const int64_t acb = terminate(L, S, a.version > 2, kRing);
  const int64_t ac_bytes = prefix ? acb : 0;
  if (!live) return;

  BitSink b{0ull, 0, ac_bytes, out, a.slice_cap};
  const SliceGeom& g = a.geom[slice];
  const uint32_t* sp = a.sym + (int64_t)seg_i * a.frame_samples + g.sym_off;
  const int bits = a.coded_bits;
  int64_t idx = 0;
  int run_index = 0;
  // one row of encode_line's Golomb branch (ffv1enc.c:318-368)
  auto code_row = [&](int pw, int set) {
    int run_count = 0, run_mode = 0;
    for (int x = 0; x < pw; x++, idx++) {
      const uint32_t sv = sp[idx];
      const int row = (int)(sv >> 16);
      const int ctx = row - set * contexts;  // context inside its plane context
      int diff = (int16_t)(sv & 0xFFFF);
      if (ctx == 0) run_mode = 1;
      if (run_mode) {
        if (diff) {
          while (run_count >= (1 << kLog2Run[run_index])) {
            run_count -= 1 << kLog2Run[run_index];
            run_index++;
            b.put(1, 1);
          }
          b.put(1 + kLog2Run[run_index], run_count);
          if (run_index) run_index--;
          run_count = 0;
          run_mode = 0;
          if (diff > 0) diff--;
        } else {
          run_count++;
        }
      }
      if (!run_mode) vlc_put(b, table[row], diff, bits);
    }
    if (run_mode) {
      while (run_count >= (1 << kLog2Run[run_index])) {
        run_count -= 1 << kLog2Run[run_index];
        run_index++;
        b.put(1, 1);
      }
      if (run_count) b.put(1, 1);
    }
  };
  if (a.rgb) {  // rows of G', B', R' (A) in turn, one run index per slice (ffv1enc.c:423)
    for (int y = 0; y < g.ph[0]; y++)
      for (int p = 0; p < a.nplanes; p++) code_row(g.pw[0], a.pset[p]);
  } else {
    for (int p = 0; p < a.nplanes; p++) {
      run_index = 0;  // per plane (ffv1enc.c:379)
      for (int y = 0; y < g.ph[p]; y++) code_row(g.pw[p], a.pset[p]);
    }
  }
  b.flush();
  const int64_t nbytes = b.pos;
  if (nbytes > a.slice_cap) {
    atomicAdd(a.status, 1);
    atomicMax(a.status + 1, (int)nbytes);
  }
  a.slice_bytes[(int64_t)f * a.nslices + slice] = min(nbytes, a.slice_cap);  // never past the slot
  if (a.j == seg.nframes - 1 && seg.save_states) {
    uint64_t* dst = reinterpret_cast<uint64_t*>(a.persist_out + (int64_t)slice * a.state_bytes);
    for (int64_t i = 0; i < nrec; i++) dst[i] = table[i];
  }
}

// ---------------------------------------------------------------------------
// Pass-1 statistics (ffv1enc.c:190-199, summed over slices at :1241-1258).
// rc_stat[state][bit]: one block per (frame, slice) stream histograms the
// recorded state byte and bit of every decision in LDS.  rc_stat2[context]
// [slot][bit]: the decisions of a symbol and their slots follow from its
// residual alone (put_symbol_inline's binarisation), so one thread per
// sample counts them from the walk record; the busiest contexts (smooth
// content lands in the low ones) count in LDS first.
constexpr int kStatsThreads = 256;
constexpr int kStatsLdsCtx = 32;

__global__ __launch_bounds__(kStatsThreads) void ffv1_stats_states(StatsArgs a) {
  __shared__ uint32_t h[512];
  if (ds_over(a.ds)) return;
  for (int i = threadIdx.x; i < 512; i += kStatsThreads) h[i] = 0;
  __syncthreads();
  const int64_t st = (int64_t)blockIdx.y * a.nslices + blockIdx.x;
  const int* dc = a.ds.dcount + st * 3;
  const int64_t base = a.ds.dbase[st];
  for (int part = 0; part < 2; part++) {
    const int64_t n = part ? (int64_t)dc[1] + dc[2] : dc[0];
    const int64_t pb = base + (part ? chroma_start(dc[0]) : 0);
    for (int64_t d = threadIdx.x; d < n; d += kStatsThreads) {
      const int64_t i = pb + d;
      const int bit = (a.ds.bits[i >> 5] >> (i & 31)) & 1;
      atomicAdd(&h[2 * a.ds.pre[i] + bit], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += kStatsThreads)
    if (h[i]) atomicAdd(&a.rc_stat[i], (unsigned long long)h[i]);
}

__global__ __launch_bounds__(kStatsThreads) void ffv1_stats_slots(StatsArgs a) {
  __shared__ uint32_t h[kStatsLdsCtx * 64];
  for (int i = threadIdx.x; i < kStatsLdsCtx * 64; i += kStatsThreads) h[i] = 0;
  __syncthreads();
  const int slice = blockIdx.x, f = blockIdx.y, p = blockIdx.z;
  const SliceGeom& g = a.geom[slice];
  const int64_t n = (int64_t)g.pw[p] * g.ph[p];
  const uint2* r = a.rec + (int64_t)f * a.frame_samples + g.sym_off + g.plane_sym_off[p];
  for (int64_t i = threadIdx.x; i < n; i += kStatsThreads) {
    const uint2 v = r[i];
    const int row = (int)(v.x & 0xFFFFu) / a.rowb;
    const int ctx = a.dense ? dense_ctx(row) : row;
    const int diff = (int16_t)(v.x >> 16);
    const bool lds = ctx < kStatsLdsCtx;
    uint32_t* hl = h + ctx * 64;
    unsigned long long* hg = a.rc_stat2 + (int64_t)ctx * 64;
    auto count = [&](int slot, int bit) {
      if (lds) atomicAdd(&hl[2 * slot + bit], 1u);
      else atomicAdd(&hg[2 * slot + bit], 1ull);
    };
    if (!diff) {
      count(0, 1);
      continue;
    }
    const unsigned mag = diff < 0 ? 0u - (unsigned)diff : (unsigned)diff;
    const int e = 31 - __builtin_clz(mag);
    count(0, 0);
    for (int k = 0; k < e; k++) count(1 + min(k, 9), 1);
    count(1 + min(e, 9), 0);
    for (int k = e - 1; k >= 0; k--) count(22 + min(k, 9), (mag >> k) & 1);
    count(11 + min(e, 10), diff < 0);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kStatsLdsCtx * 64; i += kStatsThreads)
    if (h[i]) atomicAdd(&a.rc_stat2[i], (unsigned long long)h[i]);
}

// ---------------------------------------------------------------------------
// Packet assembly + slice CRC.
constexpr uint32_t kCrcPoly = 0x04C11DB7u;

__device__ __forceinline__ uint32_t gf2_mulmod(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int i = 31; i >= 0; i--) {
    r = (r << 1) ^ ((r & 0x80000000u) ? kCrcPoly : 0u);
    if ((b >> i) & 1u) r ^= a;
  }
  return r;
}

// x^(8n) mod P via squaring table pw[k] = x^(8*2^k) mod P
__device__ __forceinline__ uint32_t xpow8(int64_t n, const uint32_t* pw) {
  uint32_t r = 1u;  // x^0
  for (int k = 0; n; k++, n >>= 1)
    if (n & 1) r = gf2_mulmod(r, pw[k]);
  return r;
}

constexpr int kAsmThreads = 256;

__global__ __launch_bounds__(kAsmThreads) void ffv1_assemble_packets(AssembleArgs a) {
  __shared__ uint32_t crc_tab[256];
  __shared__ uint32_t pw[40];
  __shared__ int64_t part[kAsmThreads];
  __shared__ uint32_t crc_part[kAsmThreads];
  if (a.skip && *a.skip) return;  // a skipped batch (status[3]): its slices were never coded
  const int t = threadIdx.x;
  const int s = blockIdx.x, f = blockIdx.y;
  const int64_t* sb = a.slice_bytes + (int64_t)f * a.nslices;

  {  // MSB-first CRC-32 byte table
    uint32_t r = (uint32_t)t << 24;
    for (int k = 0; k < 8; k++) r = (r & 0x80000000u) ? (r << 1) ^ kCrcPoly : (r << 1);
    crc_tab[t] = r;
  }
  if (t == 0) {
    uint32_t v = 1u << 8;  // x^8
    for (int k = 0; k < 40; k++) {
      pw[k] = v;
      v = gf2_mulmod(v, v);
    }
  }
  // packet offset of this slice = sum of earlier slices + their trailers
  int64_t acc = 0;
  for (int j = t; j < s; j += kAsmThreads) {
    const int tr = ((j > 0 || a.version > 2) ? 3 : 0) + (a.ec ? 5 : 0);
    acc += sb[j] + tr;
  }
  part[t] = acc;
  __syncthreads();
  for (int w = kAsmThreads / 2; w > 0; w >>= 1) {
    if (t < w) part[t] += part[t + w];
    __syncthreads();
  }
  const int64_t off = part[0];
  const int64_t n = sb[s];
  const bool has_size = s > 0 || a.version > 2;
  const int64_t body = n + (has_size ? 3 : 0) + (a.ec ? 1 : 0);  // bytes covered by the CRC
  const uint8_t* src = a.slice_out + ((int64_t)f * a.nslices + s) * a.slice_stride;
  uint8_t* dst = a.packets + (int64_t)f * a.packet_stride + off;

  auto body_byte = [&](int64_t i) -> uint32_t {
    if (i < n) return src[i];
    const int64_t k = i - n;
    if (has_size && k < 3) return (uint32_t)(n >> (8 * (2 - k))) & 0xFF;
    return 0u;  // the 0x00 before the CRC
  };

  for (int64_t i = t; i < body; i += kAsmThreads) dst[i] = (uint8_t)body_byte(i);

  if (a.ec) {
    // a thread's run of the body: whole 16-byte blocks of the slice bytes
    // (slots are 256-aligned) read as vectors, then the few trailing bytes
    const int64_t chunk = ((body + kAsmThreads - 1) / kAsmThreads + 15) & ~(int64_t)15;
    const int64_t b0 = min((int64_t)t * chunk, body), b1 = min(b0 + chunk, body);
    uint32_t crc = 0;
    auto crc_word = [&](uint32_t w) {
      crc = (crc << 8) ^ crc_tab[(crc >> 24) ^ (w & 0xFFu)];
      crc = (crc << 8) ^ crc_tab[(crc >> 24) ^ ((w >> 8) & 0xFFu)];
      crc = (crc << 8) ^ crc_tab[(crc >> 24) ^ ((w >> 16) & 0xFFu)];
      crc = (crc << 8) ^ crc_tab[(crc >> 24) ^ (w >> 24)];
    };
    int64_t i = b0;
    const int64_t vend = min(b1, n);
    for (; i + 16 <= vend; i += 16) {
      const uint4 v = *reinterpret_cast<const uint4*>(src + i);
      crc_word(v.x);
      crc_word(v.y);
      crc_word(v.z);
      crc_word(v.w);
    }
    for (; i < b1; i++) crc = (crc << 8) ^ crc_tab[(crc >> 24) ^ body_byte(i)];
    __syncthreads();
    crc_part[t] = (b1 > b0) ? gf2_mulmod(crc, xpow8(body - b1, pw)) : 0u;
    __syncthreads();
    for (int w = kAsmThreads / 2; w > 0; w >>= 1) {
      if (t < w) crc_part[t] ^= crc_part[t + w];
      __syncthreads();
    }
    if (t < 4) dst[body + t] = (uint8_t)(crc_part[0] >> (8 * (3 - t)));
  }
  if (s == a.nslices - 1 && t == 0) a.packet_size[f] = off + body + (a.ec ? 4 : 0);
}

// ---------------------------------------------------------------------------
// choose_rct_params (ffv1enc.c:1064-1144), one block per (slice, frame).  A
// pixel's contribution to the 15 sums needs its row's left neighbour and
// the same two pixels one row up: ag = g - g(x-1) (0 left of the slice),
// bg = ag - ag(x, y-1) with the row-up value as the reference keeps it in
// its int16 sample buffer; likewise b, r; br -= bg, bb -= bg; sum i adds
// |bg + ((br * c0 + bb * c1) >> 2)|.  The sums wrap like the reference's
// ints (mod 2^32 in any order), compared as int; the first minimum wins.
constexpr int kRctThreads = 256;
__constant__ int kRctCoef[15][2] = {{0, 0}, {1, 1}, {2, 2}, {0, 2}, {2, 0}, {4, 0}, {0, 4}, {0, 3},
                                    {3, 0}, {3, 1}, {1, 3}, {1, 2}, {2, 1}, {0, 1}, {1, 0}};

__device__ __forceinline__ int3 rct_bgr(const RctArgs& a, const uint8_t* fr, int x, int y) {
  if (a.sample_bytes == 4) {
    const uint32_t v = reinterpret_cast<const uint32_t*>(fr + a.plane_off[0] + (int64_t)y * a.plane_stride[0])[x];
    return make_int3(v & 0xFF, (v >> 8) & 0xFF, (v >> 16) & 0xFF);
  }
  return make_int3(reinterpret_cast<const uint16_t*>(fr + a.plane_off[0] + (int64_t)y * a.plane_stride[0])[x],
                   reinterpret_cast<const uint16_t*>(fr + a.plane_off[1] + (int64_t)y * a.plane_stride[1])[x],
                   reinterpret_cast<const uint16_t*>(fr + a.plane_off[2] + (int64_t)y * a.plane_stride[2])[x]);
}

__global__ __launch_bounds__(kRctThreads) void ffv1_rct_params(RctArgs a) {
  __shared__ uint32_t part[15][kRctThreads];
  const int slice = blockIdx.x, f = blockIdx.y;
  const SliceGeom& g = a.geom[slice];
  const uint8_t* const fr = a.frames + (int64_t)f * a.frame_bytes;
  const int w = g.pw[0], h = g.ph[0], x0 = g.px[0], y0 = g.py[0];
  uint32_t st[15];
#pragma unroll
  for (int i = 0; i < 15; i++) st[i] = 0u;
  const int64_t n = (int64_t)(w - 1) * (h - 1);  // pixels with x, y >= 1
  for (int64_t k = threadIdx.x; k < n; k += kRctThreads) {
    const int x = 1 + (int)(k % (w - 1)), y = 1 + (int)(k / (w - 1));
    const int3 c = rct_bgr(a, fr, x0 + x, y0 + y), l = rct_bgr(a, fr, x0 + x - 1, y0 + y);
    const int3 u = rct_bgr(a, fr, x0 + x, y0 + y - 1), ul = rct_bgr(a, fr, x0 + x - 1, y0 + y - 1);
    const int bg = (c.y - l.y) - (int)(int16_t)(u.y - ul.y);
    int bb = (c.x - l.x) - (int)(int16_t)(u.x - ul.x);
    int br = (c.z - l.z) - (int)(int16_t)(u.z - ul.z);
    br -= bg;
    bb -= bg;
#pragma unroll
    for (int i = 0; i < 15; i++) {
      const int v = bg + ((br * kRctCoef[i][0] + bb * kRctCoef[i][1]) >> 2);
      st[i] += (uint32_t)(v < 0 ? -v : v);
    }
  }
#pragma unroll
  for (int i = 0; i < 15; i++) part[i][threadIdx.x] = st[i];
  __syncthreads();
  for (int s = kRctThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s)
      for (int i = 0; i < 15; i++) part[i][threadIdx.x] += part[i][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int best = 0;
    for (int i = 1; i < 15; i++)
      if ((int)part[i][0] < (int)part[best][0]) best = i;
    a.rct[(int64_t)f * a.nslices + slice] = make_int2(kRctCoef[best][1], kRctCoef[best][0]);
  }
}

}  // namespace

int launch_rct_params(const RctArgs& a, void* stream) {
  if (a.nframes <= 0) return 0;
  hipLaunchKernelGGL(ffv1_rct_params, dim3(a.nslices, a.nframes), dim3(kRctThreads), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_symbols(const SymbolArgs& a, void* stream) {
  const int np = a.p_hi > a.p_lo ? a.p_hi - a.p_lo : a.nplanes - a.p_lo;
  if (np <= 0 || a.nslots <= 0) return 0;
  SymbolArgs b = a;
  b.nz = np * kSymSplit;
  const int64_t items = (int64_t)a.nslices * a.nslots * b.nz;
  dim3 grid((unsigned)(a.max_blocks > 0 ? std::min<int64_t>(items, a.max_blocks) : items)), block(kSymThreads);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a.sample_bytes == 1 && !a.rgb)
    hipLaunchKernelGGL((ffv1_symbols<1, false>), grid, block, 0, st, b);
  else if (a.sample_bytes == 4 && a.rgb)
    hipLaunchKernelGGL((ffv1_symbols<4, true>), grid, block, 0, st, b);
  else if (a.sample_bytes == 2 && a.rgb)
    hipLaunchKernelGGL((ffv1_symbols<2, true>), grid, block, 0, st, b);
  else if (a.sample_bytes == 2)
    hipLaunchKernelGGL((ffv1_symbols<2, false>), grid, block, 0, st, b);
  else
    return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_code(const CodeArgs& a, void* stream) {
  const int64_t chains = (int64_t)a.nsegs * a.nslices;
  if (a.cpw < 1 || a.cpw > kCodeThreads) return -1;
  dim3 grid((unsigned)((chains + a.cpw - 1) / a.cpw)), block(kCodeThreads);
  hipLaunchKernelGGL(ffv1_code, grid, block, code_lds_bytes(kCodeThreads), reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_range(const CodeArgs& a, void* stream) {
  const int64_t streams = (int64_t)a.nframes * a.nslices;
  dim3 grid((unsigned)((streams + kRangeThreads - 1) / kRangeThreads)), block(kRangeThreads);
  hipLaunchKernelGGL(ffv1_range, grid, block, 0, reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_dseg(const CodeArgs& a, void* stream) {
  hipLaunchKernelGGL(ffv1_dseg, dim3((unsigned)a.dseg_blocks), dim3(kDsegThreads), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_range_dseg(const CodeArgs& a, void* stream) {
  static_assert(kRangeThreads == kDsegThreads, "one block size for both roles");
  const int64_t streams = (int64_t)a.nframes * a.nslices;
  CodeArgs b = a;
  b.range_blocks = (int)((streams + kRangeThreads - 1) / kRangeThreads);
  hipLaunchKernelGGL(ffv1_range_dseg, dim3((unsigned)(b.range_blocks + a.dseg_blocks)), dim3(kRangeThreads), 0,
                     reinterpret_cast<hipStream_t>(stream), b);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_dfix(const CodeArgs& a, void* stream) {
  const int64_t streams = (int64_t)a.nframes * a.nslices;
  dim3 grid((unsigned)((streams + kFixThreads - 1) / kFixThreads)), block(kFixThreads);
  hipLaunchKernelGGL(ffv1_dfix, grid, block, 0, reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int64_t walk_lds_bytes(int rows, int rowb) { return walk_lds_bytes_dev(rows, rowb); }

int launch_walk(const WalkArgs& a, int nsegs, void* stream, int first, int count) {
  if ((a.rowb != 32 && (a.rowb != kCompactRowBytes || a.dense)) || walk_lds_bytes_dev(a.rows, a.rowb) > kWalkLdsMax ||
      a.rows * a.rowb > 0xFFFF)
    return -1;
  WalkArgs b = a;
  if (b.per_short < 1) b.per_short = 1;
  b.nsegs = nsegs;
  b.short_multi = std::max(0, std::min(b.short_multi, (nsegs + b.per_short - 1) / b.per_short));
  b.nitems = walk_items(nsegs, a.nslices, b.per_short, b.short_multi);
  const size_t tables = (size_t)(2 * ((int64_t)a.rows * a.rowb + 32));  // one wave's; the fixed part is static
  const bool compact = a.rowb == kCompactRowBytes;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a.block_waves > 1) {  // one round: a block per CU (walk_block_waves)
    const int npairs = (a.nslices + 1) / 2;
    const int nfull = npairs * (nsegs + b.short_multi);
    const int nsingle = b.nitems - nfull;
    const int blocks = std::max((nfull + 3) / 4, nsingle);
    b.item0 = 0;
    if (a.block_waves == 5)
      hipLaunchKernelGGL((compact ? ffv1_walk<5, kCompactRowBytes> : ffv1_walk<5>), dim3((unsigned)blocks),
                         dim3(kWalkThreads * 5), 5 * tables, st, b);
    else
      hipLaunchKernelGGL((compact ? ffv1_walk<4, kCompactRowBytes> : ffv1_walk<4>), dim3((unsigned)blocks),
                         dim3(kWalkThreads * 4), 4 * tables, st, b);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (count < 0) count = b.nitems - first;
  if (first < 0 || count <= 0 || first + count > b.nitems) return count == 0 ? 0 : -1;
  b.item0 = first;
  hipLaunchKernelGGL((compact ? ffv1_walk<1, kCompactRowBytes> : ffv1_walk<1>), dim3((unsigned)count), dim3(kWalkThreads),
                     tables, st, b);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Block shape of a batch's walk: 4 or 5 waves per block when the batch is
// one round with every full-length wave alone on a SIMD (at most 4 per CU
// of them, at most one one-segment wave per CU) and the block's LDS fits a
// CU; else 1 (waves placed by the dispatcher, several rounds).
int walk_block_waves(int nsegs, int nslices, int per_short, int short_multi, int rows, int rowb, int cus,
                     int lds_block) {
  const int npairs = (nslices + 1) / 2;
  const int nfull = npairs * (nsegs + short_multi);
  const int nsingle = walk_items(nsegs, nslices, per_short, short_multi) - nfull;
  if (nfull > 4 * cus || nsingle > cus) return 1;
  const int w = nsingle > 0 ? 5 : 4;
  // the block's LDS against what one workgroup may take on this device
  // (queried once at create; a part with less falls back to one-wave blocks
  // instead of failing the launch)
  return walk_block_lds_dev(rows, w, rowb) <= lds_block ? w : 1;
}

int walk_items(int nsegs, int nslices, int per_short, int short_multi) {
  const int npairs = (nslices + 1) / 2;
  const int covered = std::min(nsegs, short_multi * per_short);
  return npairs * (nsegs + short_multi + (nsegs - covered));
}

// How many of the shorter group's waves take per_short segments: all of them
// when the long waves and those fit one per SIMD (4 per CU); else as many as
// still fit one per SIMD beside the long ones, the segments left going one
// per wave onto SIMDs that already hold a walk wave (where they run ~1.4x
// slower, on half the work), provided every wave is then resident at once
// (`resident`).  Otherwise none: the walk takes several rounds anyway, and
// the shorter group's one-segment waves, last in the launch, fill the last
// round's gaps (c2: 13.3 vs 12.4 Gpix/s with two segments per wave).
int walk_split_short(int nsegs, int nslices, int per_short, int simds, int resident) {
  const int npairs = (nslices + 1) / 2;
  const int all = (nsegs + per_short - 1) / per_short;
  if (per_short < 2 || npairs * (nsegs + all) <= simds) return all;
  for (int m = all; m >= 0; m--)
    if (npairs * (nsegs + m) <= simds && walk_items(nsegs, nslices, per_short, m) <= resident) return m;
  return 0;
}

int walk_per_short(const SliceGeom& g) {
  const int64_t l = (int64_t)g.pw[0] * g.ph[0];
  const int64_t c = (int64_t)g.pw[1] * g.ph[1] + (int64_t)g.pw[2] * g.ph[2];
  if (l <= 0 || c <= 0) return 1;
  const int64_t lo = std::min(l, c), hi = std::max(l, c);
  return (int)std::max<int64_t>(1, std::min<int64_t>(4, (hi + lo / 2) / lo));
}

// Walk waves one CU holds at once (LDS-bound), for launch splitting.
int walk_resident(const WalkArgs& a) {
  const size_t dyn = (size_t)(2 * ((int64_t)a.rows * a.rowb + 32));
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ffv1_walk<1>, kWalkThreads, dyn) != hipSuccess ||
      hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return per_cu * cus;
}

int launch_bits(const BitsArgs& a, void* stream) {
  const int64_t streams = (int64_t)a.nslices * a.nframes;
  const int64_t grid = a.max_blocks > 0 ? std::min<int64_t>(streams, a.max_blocks) : streams;
  hipLaunchKernelGGL(ffv1_bits, dim3((unsigned)grid), dim3(kBitsThreads), 0, reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_layout(const int* dcount, int nstreams, int64_t* dbase, int64_t* total, StreamSegs* segs,
                  int* seg_totals, int* wmap, int64_t* total_host, void* stream) {
  hipLaunchKernelGGL(ffv1_layout, dim3(1), dim3(kLayoutThreads), 0, reinterpret_cast<hipStream_t>(stream), dcount,
                     nstreams, dbase, total, segs, seg_totals, wmap, total_host);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The decision bits of a guarded batch zeroed on the device, as far as its
// total (the host does not know it): min(total, cap) decisions
constexpr int kZeroThreads = 256;
__global__ __launch_bounds__(kZeroThreads) void ffv1_zero_bits(uint32_t* bits, const int64_t* total, int64_t cap) {
  const int64_t n = (min(*total, cap) + 31) / 32 / 4;  // uint4 words
  uint4* const b4 = reinterpret_cast<uint4*>(bits);
  for (int64_t i = (int64_t)blockIdx.x * kZeroThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kZeroThreads)
    b4[i] = make_uint4(0, 0, 0, 0);
}

int launch_zero_bits(uint32_t* bits, const int64_t* total, int64_t cap, void* stream) {
  hipLaunchKernelGGL(ffv1_zero_bits, dim3(512), dim3(kZeroThreads), 0, reinterpret_cast<hipStream_t>(stream), bits,
                     total, cap);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_stats(const StatsArgs& a, bool states, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (states)
    hipLaunchKernelGGL(ffv1_stats_states, dim3(a.nslices, a.nframes), dim3(kStatsThreads), 0, st, a);
  else
    hipLaunchKernelGGL(ffv1_stats_slots, dim3(a.nslices, a.nframes, 3), dim3(kStatsThreads), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_sink(const CodeArgs& a, void* stream) {
  const int64_t streams = (int64_t)a.nframes * a.nslices;
  dim3 grid((unsigned)streams), block(kSinkThreads);
  hipLaunchKernelGGL(ffv1_sink, grid, block, 0, reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_code_golomb(const CodeArgs& a, void* stream) {
  const int64_t chains = (int64_t)a.nsegs * a.nslices;
  if (a.cpw < 1 || a.cpw > kCodeThreads) return -1;
  dim3 grid((unsigned)((chains + a.cpw - 1) / a.cpw)), block(kCodeThreads);
  hipLaunchKernelGGL(ffv1_code_golomb, grid, block, 0, reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

namespace {
// The host-frame path's packets, back to back for one D2H copy: block i
// sums the sizes before packet i and copies packet i there (16-byte loads
// from its aligned slot, byte stores to the unaligned place).
constexpr int kCompactThreads = 256;
__global__ __launch_bounds__(kCompactThreads) void ffv1_compact_packets(const uint8_t* packets, int64_t stride,
                                                                         const int64_t* sizes, int n, uint8_t* out,
                                                                         const int* skip) {
  __shared__ int64_t part[kCompactThreads];
  if (skip && *skip) return;  // a skipped batch: no packets (the host encodes it again)
  const int i = blockIdx.x;
  int64_t s = 0;
  for (int k = threadIdx.x; k < i; k += kCompactThreads) s += sizes[k];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = kCompactThreads / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  const int64_t off = part[0], sz = sizes[i];
  const uint4* src = reinterpret_cast<const uint4*>(packets + (int64_t)i * stride);
  uint8_t* dst = out + off;
  for (int64_t k = threadIdx.x; k * 16 < sz; k += kCompactThreads) {
    const uint4 v = src[k];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (int b = 0; b < 16 && k * 16 + b < sz; b++) dst[k * 16 + b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
  }
}
// A batch's packet sizes into host memory (mapped pinned), written by the
// kernel itself: a DMA copy of them would queue behind the next batch's
// frames going the other way.
__global__ __launch_bounds__(256) void ffv1_sizes_out(const int64_t* sizes, int n, int64_t* host) {
  for (int i = threadIdx.x; i < n; i += 256) host[i] = sizes[i];
}
__global__ __launch_bounds__(64) void ffv1_ints_out(const int* src, int n, int* host) {
  if ((int)threadIdx.x < n) host[threadIdx.x] = src[threadIdx.x];
}
}  // namespace

int launch_sizes_out(const int64_t* sizes, int n, int64_t* host_mapped, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(ffv1_sizes_out, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), sizes, n,
                     host_mapped);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_ints_out(const int* src, int n, int* host_mapped, void* stream) {
  if (n <= 0 || n > 64) return -1;
  hipLaunchKernelGGL(ffv1_ints_out, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), src, n, host_mapped);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Host-frame path, 10-bit samples: the host packs three samples to a 32-bit
// word (bits 0-9, 10-19, 20-29; a row's last word holds one to three), so a
// frame crosses PCIe in 2/3 of its bytes; here they go back to 16-bit
// samples in the frame slot, one block row per (frame, plane).  A frame the
// host staged as is (a sample over 10 bits, or caller-pinned) is skipped.
__global__ __launch_bounds__(256) void ffv1_unpack10(UnpackArgs a) {
  const int f = (int)blockIdx.y / a.np, p = (int)blockIdx.y - f * a.np;
  if ((a.raw[f >> 5] >> (f & 31)) & 1u) return;
  const int wpr = a.prow[p], width = a.width[p];
  const int nw = wpr * a.rows[p];
  const uint32_t* const src =
      reinterpret_cast<const uint32_t*>(a.packed + (int64_t)(a.f0 + f) * a.packed_frame_bytes + a.poff[p]);
  uint8_t* const dst = a.frames + (int64_t)(a.f0 + f) * a.frame_bytes + a.off[p];
  for (int i = (int)(blockIdx.x * blockDim.x + threadIdx.x); i < nw; i += (int)(gridDim.x * blockDim.x)) {
    const int r = i / wpr, j = i - r * wpr, x = 3 * j;
    const uint32_t w = src[i];
    uint16_t* const row = reinterpret_cast<uint16_t*>(dst + (int64_t)r * a.pst[p]);
    row[x] = (uint16_t)(w & 0x3FFu);
    if (x + 1 < width) row[x + 1] = (uint16_t)((w >> 10) & 0x3FFu);
    if (x + 2 < width) row[x + 2] = (uint16_t)((w >> 20) & 0x3FFu);
  }
}

int launch_unpack10(const UnpackArgs& a, int nframes, void* stream) {
  if (nframes <= 0) return 0;
  if (nframes > kUnpackFrames || a.np < 1 || a.np > kMaxPlanes) return -1;
  int maxw = 0;
  for (int p = 0; p < a.np; p++) maxw = max(maxw, a.prow[p] * a.rows[p]);
  dim3 grid((unsigned)max(1, min(512, (maxw + 255) / 256)), (unsigned)(nframes * a.np)), block(256);
  hipLaunchKernelGGL(ffv1_unpack10, grid, block, 0, reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_compact_packets(const uint8_t* packets, int64_t stride, const int64_t* sizes, int n, uint8_t* out,
                           const int* skip, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(ffv1_compact_packets, dim3(n), dim3(kCompactThreads), 0, reinterpret_cast<hipStream_t>(stream),
                     packets, stride, sizes, n, out, skip);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_assemble(const AssembleArgs& a, int nframes, void* stream) {
  dim3 grid(a.nslices, nframes), block(kAsmThreads);
  hipLaunchKernelGGL(ffv1_assemble_packets, grid, block, 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace ffv1hip
