// ffv1_decode.hip -- FFV1 range-coded slice decoder on gfx950 (the
// on-device lossless self-check of SURVEY §8f, row 1).
//
// Reference: ffv1dec.c decode_slice (:248-280 + :361-474), decode_line
// (:42-117, the range-coder branch), get_symbol_inline (:44-66);
// rangecoder.h get_rac / refill (:104-147).  Decoding is a serial chain per
// (GOP segment, slice): each decision's context state and each sample's
// neighbourhood depend on the decisions before it.  One workgroup of one
// wave per chain keeps the chain's adaptive states (2 x 666 x 32 bytes),
// the transition table, the quant tables and two sample rows in LDS; lane 0
// runs the chain, the other lanes do the bulk state resets and copies.
#include "ffv1_internal.h"

namespace ffv1hip {
namespace {

constexpr int kDecThreads = 64;

struct RacDec {
  uint32_t low, range;
  int64_t ptr, end;  // byte offsets into the packet buffer
  int64_t wi;        // index of the 8-byte word w0 holds
  uint64_t w0, w1;   // the word holding ptr and the one after it (in flight)
};

__device__ inline void rac_init(RacDec& c, const uint8_t* pk, int64_t start, int64_t end) {
  // ff_init_range_decoder + the first two bytes (rangecoder.c:53-61)
  c.range = 0xFF00;
  c.low = (uint32_t(pk[start]) << 8) | pk[start + 1];
  c.ptr = start + 2;
  c.end = end;
  const uint64_t* w = reinterpret_cast<const uint64_t*>(pk);
  c.wi = c.ptr >> 3;
  c.w0 = w[c.wi];
  c.w1 = w[c.wi + 1];
}

// refill (rangecoder.h:104-115): ptr advances one byte at a time, so the
// next word is always w1; the word after it is loaded a word ahead.
__device__ inline void rac_refill(RacDec& c, const uint64_t* w) {
  c.range <<= 8;
  c.low <<= 8;
  if (c.ptr < c.end) {
    const int64_t wi = c.ptr >> 3;
    if (wi != c.wi) {
      c.w0 = c.w1;
      c.w1 = w[wi + 1];
      c.wi = wi;
    }
    c.low += uint32_t(c.w0 >> ((c.ptr & 7) * 8)) & 0xFF;
  }
  c.ptr++;
}

// get_rac (rangecoder.h:117-147), branch-free: the transition pair of the
// state (tt[s] = to0[s] | to1[s] << 8) is read beside the range arithmetic,
// so a decision waits on two LDS reads (state, pair) rather than three.
__device__ inline int rac_get(RacDec& c, uint8_t* st, const uint16_t* tt, const uint64_t* w) {
  const uint32_t s = *st;
  const uint32_t pair = tt[s];
  const uint32_t r1 = (c.range * s) >> 8;
  const uint32_t rr = c.range - r1;
  const int bit = c.low >= rr;
  c.low -= bit ? rr : 0u;
  c.range = bit ? r1 : rr;
  *st = uint8_t(bit ? pair >> 8 : pair);
  if (c.range < 0x100) rac_refill(c, w);
  return bit;
}

// get_symbol_inline (ffv1dec.c:44-66)
__device__ inline int rac_symbol(RacDec& c, uint8_t* st, int is_signed, const uint16_t* tt,
                                 const uint64_t* w) {
  if (rac_get(c, st, tt, w)) return 0;
  int e = 0;
  while (rac_get(c, st + 1 + (e < 9 ? e : 9), tt, w)) {
    if (++e > 31) return 0;
  }
  int a = 1;
  for (int i = e - 1; i >= 0; i--) a = 2 * a + rac_get(c, st + 22 + (i < 9 ? i : 9), tt, w);
  if (is_signed && rac_get(c, st + 11 + (e < 10 ? e : 10), tt, w)) return -a;
  return a;
}

__device__ inline int median3(int a, int b, int c) {
  return max(min(a, b), min(max(a, b), c));
}

__global__ void __launch_bounds__(kDecThreads) ffv1_decode_slices(DecodeArgs a) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int s = blockIdx.x, seg = blockIdx.y, lane = threadIdx.x;
  const Segment sg = a.segs[seg];
  const SliceGeom* g = a.geom + s;  // read through the pointer: a by-value copy indexed by plane spills
  uint8_t* states = lds;                                         // [2][contexts][32]
  uint16_t* tt = reinterpret_cast<uint16_t*>(lds + a.state_bytes);  // [256] to0 | to1 << 8
  uint8_t* hdr = lds + a.state_bytes + 512;                      // [32] slice-header states
  int16_t* qt = reinterpret_cast<int16_t*>(hdr + 32);            // [3][256]
  int16_t* ring = qt + 3 * 256;                                  // [2][row_cap]
  __shared__ int bad;
  const uint64_t* pkw = reinterpret_cast<const uint64_t*>(a.pkts);
  for (int i = lane; i < 256; i += kDecThreads) tt[i] = uint16_t(a.ftab[i] | (a.ftab[256 + i] << 8));
  for (int i = lane; i < 3 * 256; i += kDecThreads) qt[i] = a.qt[i];
  if (lane == 0) bad = 0;
  const int mask = (1 << a.coded_bits) - 1;
  const int planes = a.nplanes;
  RacDec c{};
  for (int j = 0; j < sg.nframes; j++) {
    const int f = sg.first_frame + j;
    const int key = a.keyflags[f];
    uint32_t* st4 = reinterpret_cast<uint32_t*>(states);
    const int64_t words = a.state_bytes / 4;
    if (key) {  // ff_ffv1_clear_slice_state on keyframes (ffv1dec.c:261-263)
      for (int64_t i = lane; i < words; i += kDecThreads) st4[i] = 0x80808080u;
    } else if (j == 0) {  // continue the previous call's chain
      const uint32_t* src = reinterpret_cast<const uint32_t*>(a.persist_in + int64_t(s) * a.state_bytes);
      for (int64_t i = lane; i < words; i += kDecThreads) st4[i] = src[i];
    }
    __syncthreads();
    if (lane == 0) {
      const int64_t fs = int64_t(f) * a.nslices + s;
      rac_init(c, a.pkts, a.slice_start[fs], a.slice_end[fs]);
      int ok = 1;
      if (s == 0) {  // the key bit, state 128 (ffv1dec.c:931-933)
        hdr[0] = 128;
        ok &= rac_get(c, hdr, tt, pkw) == key;
      }
      // decode_slice_header (ffv1dec.c:169-215), checked against the grid
      for (int i = 0; i < 32; i++) hdr[i] = 128;
      const int sx = rac_symbol(c, hdr, 0, tt, pkw);
      const int sy = rac_symbol(c, hdr, 0, tt, pkw);
      const int sw = rac_symbol(c, hdr, 0, tt, pkw);
      const int sh = rac_symbol(c, hdr, 0, tt, pkw);
      const int x0 = int(int64_t(sx) * a.width / a.num_h), y0 = int(int64_t(sy) * a.height / a.num_v);
      const int x1 = int(int64_t(sx + sw + 1) * a.width / a.num_h);
      const int y1 = int(int64_t(sy + sh + 1) * a.height / a.num_v);
      ok &= x0 == g->px[0] && y0 == g->py[0] && x1 - x0 == g->pw[0] && y1 - y0 == g->ph[0];
      for (int i = 0; i < 2; i++) ok &= rac_symbol(c, hdr, 0, tt, pkw) == a.context_model;
      (void)rac_symbol(c, hdr, 0, tt, pkw);  // picture structure
      (void)rac_symbol(c, hdr, 0, tt, pkw);  // sample aspect ratio
      (void)rac_symbol(c, hdr, 0, tt, pkw);
      if (!ok) {
        bad = 1;
        atomicAdd(&a.status[0], 1);
      }
    }
    __syncthreads();
    if (bad) return;
    for (int p = 0; p < planes; p++) {
      for (int i = lane; i < 2 * a.row_cap; i += kDecThreads) ring[i] = 0;
      __syncthreads();
      // decode_plane / decode_line (ffv1dec.c:42-117, :248-280): the same
      // zeroed-ring neighbourhood as the encoder's encode_plane.  Lane 0
      // decodes a row into LDS; the wave then stores it (coalesced), so the
      // serial loop issues no global stores.
      uint8_t* pst = states + (p ? a.state_bytes / 2 : 0);
      const int w = g->pw[p], h = g->ph[p];
      const int64_t poff = p == 0 ? a.plane_off[0] : (p == 1 ? a.plane_off[1] : a.plane_off[2]);
      const int pw = p == 0 ? a.plane_w[0] : (p == 1 ? a.plane_w[1] : a.plane_w[2]);
      uint8_t* obase = a.out + int64_t(f) * a.frame_bytes + poff;
      const int16_t* q0 = qt;
      const int16_t* q1 = qt + 256;
      const int16_t* q2 = qt + 512;
      for (int y = 0; y < h; y++) {
        int16_t* cur = ring + (y & 1) * a.row_cap;  // holds row y-2 until written
        const int16_t* up = ring + ((y + 1) & 1) * a.row_cap;
        if (lane == 0) {
          int T = up[0];
          int L = T;
          int LT = cur[0];  // two rows up, column 0
          for (int x = 0; x < w; x++) {
            const int RT = x + 1 < w ? up[x + 1] : T;
            const int ctx = q0[(L - LT) & 0xFF] + q1[(LT - T) & 0xFF] + q2[(T - RT) & 0xFF];
            const int pred = median3(L, L + T - LT, T);
            // one call site: the symbol decoder is the kernel's hot code
            const int sym = rac_symbol(c, pst + (ctx < 0 ? -ctx : ctx) * 32, 1, tt, pkw);
            const int diff = ctx < 0 ? -sym : sym;
            const int16_t v = int16_t((pred + diff) & mask);
            cur[x] = v;
            LT = T;
            T = RT;
            L = v;
          }
        }
        __syncthreads();
        const int64_t orow = int64_t(g->py[p] + y) * pw + g->px[p];
        if (a.sample_bytes == 1) {
          for (int x = lane; x < w; x += kDecThreads) obase[orow + x] = uint8_t(cur[x]);
        } else {
          uint16_t* o16 = reinterpret_cast<uint16_t*>(obase) + orow;
          for (int x = lane; x < w; x += kDecThreads) {
            const uint32_t u = uint16_t(cur[x]);
            o16[x] = uint16_t(a.packed_at_lsb ? u : (u << a.msb_shift));
          }
        }
      }
      __syncthreads();
    }
  }
  if (sg.save_states) {
    const uint32_t* st4 = reinterpret_cast<const uint32_t*>(states);
    uint32_t* dst = reinterpret_cast<uint32_t*>(a.persist_out + int64_t(s) * a.state_bytes);
    for (int64_t i = lane; i < a.state_bytes / 4; i += kDecThreads) dst[i] = st4[i];
  }
}

}  // namespace

int64_t decode_lds_bytes(int64_t state_bytes, int row_cap) {
  return state_bytes + 512 + 32 + 3 * 256 * 2 + int64_t(2) * row_cap * 2;
}

int launch_decode(const DecodeArgs& a, int nsegs, void* stream) {
  dim3 grid(a.nslices, nsegs), block(kDecThreads);
  hipLaunchKernelGGL(ffv1_decode_slices, grid, block, decode_lds_bytes(a.state_bytes, a.row_cap),
                     reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace ffv1hip
