// ffv1_kernels.hip -- CDNA4 (gfx950) kernels of the FFV1 P-frame encoder.
//
// Hot path:
//   ffv1_encode_slices  one 64-lane wavefront per (slice, frame segment).
//     * rows of the slice plane are staged through LDS; the 64 lanes
//       compute median prediction + quantised-gradient contexts + fold for
//       a whole row in parallel (ffv1.h:148-190, ffv1enc.c:306-317);
//     * the adaptive binary range coder (rangecoder.h:52-102) and symbol
//       binarisation (ffv1enc.c:185-231) then run wave-uniformly over that
//       row: it is the serial part of the bitstream;
//     * the per-slice context-state table (the P-frame carry,
//       ffv1enc.c:1171-1172) lives in LDS for the whole frame segment.
//   ffv1_assemble_packets  one workgroup per (slice, frame): packet
//     placement (prefix over slice sizes), 3-byte size, 0x00 and the slice
//     CRC-32 computed chunk-parallel and combined in GF(2)
//     (ffv1enc.c:1326-1354, crc.c:357).
#include <hip/hip_runtime.h>

#include "ffv1_internal.h"

namespace ffv1hip {

namespace {

constexpr int kWave = 64;

// ---------------------------------------------------------------------------
// Range coder: wave-uniform register state.  Bytes are packed into a 32-bit
// word and lane 0 stores whole dwords; the pending-byte / 0xFF-run logic of
// renorm_encoder is kept verbatim in meaning so the output is identical.
struct Rac {
  int low, range;
  int pending;    // outstanding_byte (-1 = none yet)
  int run;        // outstanding_count (deferred 0xFF bytes)
  uint32_t word;  // bytes not yet stored
  int nword;
  int64_t pos;    // bytes stored so far
};

struct Sink {
  uint8_t* out;
  int64_t cap;
  bool lane0;
};

__device__ __forceinline__ void rac_emit(Rac& c, const Sink& s, int b) {
  c.word |= (uint32_t)(b & 0xFF) << (8 * c.nword);
  if (++c.nword == 4) {
    if (s.lane0 && c.pos + 4 <= s.cap)
      *reinterpret_cast<uint32_t*>(s.out + c.pos) = c.word;
    c.pos += 4;
    c.word = 0;
    c.nword = 0;
  }
}

__device__ __forceinline__ void rac_shift(Rac& c, const Sink& s) {
  if (c.pending < 0) {
    c.pending = c.low >> 8;
  } else if (c.low <= 0xFF00) {
    rac_emit(c, s, c.pending);
    for (; c.run; c.run--) rac_emit(c, s, 0xFF);
    c.pending = c.low >> 8;
  } else if (c.low >= 0x10000) {
    rac_emit(c, s, c.pending + 1);
    for (; c.run; c.run--) rac_emit(c, s, 0x00);
    c.pending = (c.low >> 8) & 0xFF;
  } else {
    c.run++;
  }
  c.low = (c.low & 0xFF) << 8;
  c.range <<= 8;
}

// One binary decision with adaptive state st; returns the next state.
// tab = [to0[256] | to1[256]] in LDS.
__device__ __forceinline__ int rac_put(Rac& c, const Sink& s, int st, int bit,
                                       const uint8_t* tab) {
  const int r1 = (c.range * st) >> 8;
  if (bit) {
    c.low += c.range - r1;
    c.range = r1;
  } else {
    c.range -= r1;
  }
  // the interval never shrinks below 1, so one byte shift always suffices
  if (c.range < 0x100) rac_shift(c, s);
  return tab[(bit << 8) | st];
}

__device__ __forceinline__ void rac_put_mem(Rac& c, const Sink& s, uint8_t* sp,
                                            int bit, const uint8_t* tab) {
  *sp = (uint8_t)rac_put(c, s, *sp, bit, tab);
}

// put_symbol: zero flag, unary exponent, mantissa MSB first, sign.
__device__ __forceinline__ void rac_symbol(Rac& c, const Sink& s, uint8_t* st,
                                           int v, bool is_signed,
                                           const uint8_t* tab) {
  if (v == 0) {
    rac_put_mem(c, s, st, 1, tab);
    return;
  }
  const unsigned a = v < 0 ? 0u - (unsigned)v : (unsigned)v;
  const int e = 31 - __builtin_clz(a);
  rac_put_mem(c, s, st, 0, tab);
  for (int i = 0; i < e; i++) rac_put_mem(c, s, st + 1 + min(i, 9), 1, tab);
  rac_put_mem(c, s, st + 1 + min(e, 9), 0, tab);
  for (int i = e - 1; i >= 0; i--)
    rac_put_mem(c, s, st + 22 + min(i, 9), (a >> i) & 1, tab);
  if (is_signed) rac_put_mem(c, s, st + 11 + min(e, 10), v < 0, tab);
}

__device__ __forceinline__ int64_t rac_finish(Rac& c, const Sink& s) {
  c.range = 0xFF;
  c.low += 0xFF;
  while (c.range < 0x100) rac_shift(c, s);
  c.range = 0xFF;
  while (c.range < 0x100) rac_shift(c, s);
  // flush the partial word byte by byte
  if (s.lane0)
    for (int k = 0; k < c.nword; k++)
      if (c.pos + k < s.cap) s.out[c.pos + k] = (uint8_t)(c.word >> (8 * k));
  return c.pos + c.nword;
}

__device__ __forceinline__ int median3(int a, int b, int c) {
  return max(min(a, b), min(max(a, b), c));
}

__device__ __forceinline__ int fold_bits(int d, int bits) {
  if (bits == 8) return (int)(int8_t)d;
  const int sh = 32 - bits;
  return (d << sh) >> sh;  // sign-extend the low `bits` bits
}

__device__ __forceinline__ size_t align16(size_t v) { return (v + 15) & ~size_t(15); }

struct LdsLayout {
  size_t states, tabs, qt, opsets, rows, sym, total;
};

__host__ __device__ inline LdsLayout lds_layout(const EncodeArgs& a, bool lds_states) {
  LdsLayout L;
  size_t off = 0;
  L.states = off;
  if (lds_states) off += ((size_t)2 * a.contexts * 32 + 15) & ~size_t(15);
  L.tabs = off;   off += 1024;
  L.qt = off;     off += 5 * 256 * 2;
  L.opsets = off; off += kOpSets * 32;
  L.rows = off;   off += ((size_t)3 * a.row_len * 2 + 15) & ~size_t(15);
  L.sym = off;    off += (size_t)a.row_len * 4;
  L.total = off;
  return L;
}

// ---------------------------------------------------------------------------
template <bool kLdsStates>
__global__ __launch_bounds__(kWave) void ffv1_encode_slices(EncodeArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const LdsLayout L = lds_layout(a, kLdsStates);
  const int lane = threadIdx.x;
  const int slice = blockIdx.x;
  const Segment seg = a.segs[blockIdx.y];

  uint8_t* tabs = smem + L.tabs;
  int16_t* qt = reinterpret_cast<int16_t*>(smem + L.qt);
  uint8_t* opsets = smem + L.opsets;
  int16_t* rows = reinterpret_cast<int16_t*>(smem + L.rows);
  int32_t* sym = reinterpret_cast<int32_t*>(smem + L.sym);
  const int64_t state_bytes = (int64_t)2 * a.contexts * 32;
  uint8_t* states =
      kLdsStates ? smem + L.states
                 : a.gstates + ((int64_t)blockIdx.y * a.nslices + slice) * state_bytes;

  for (int i = lane; i < 1024; i += kWave) tabs[i] = a.tabs[i];
  for (int i = lane; i < 5 * 256; i += kWave) qt[i] = a.qt[i];
  if (seg.load_states) {
    const uint8_t* src = a.persist + (int64_t)slice * state_bytes;
    for (int64_t i = lane * 4; i < state_bytes; i += kWave * 4)
      *reinterpret_cast<uint32_t*>(states + i) = *reinterpret_cast<const uint32_t*>(src + i);
  }
  __syncthreads();

  // slice rectangle (ffv1.c:117-145)
  const int sx = slice % a.nh, sy = slice / a.nh;
  const int x0 = (int)((int64_t)a.width * sx / a.nh);
  const int y0 = (int)((int64_t)a.height * sy / a.nv);
  const int sw = (int)((int64_t)a.width * (sx + 1) / a.nh) - x0;
  const int sh = (int)((int64_t)a.height * (sy + 1) / a.nv) - y0;
  const uint8_t* ftab = tabs + 512;
  const int nplanes = a.chroma_planes ? 3 : 1;

  for (int f = seg.first_frame; f < seg.first_frame + seg.nframes; f++) {
    const int key = a.keyflags[f];
    if (key) {  // ff_ffv1_clear_slice_state: initial states are all 128
      for (int64_t i = lane * 4; i < state_bytes; i += kWave * 4)
        *reinterpret_cast<uint32_t*>(states + i) = 0x80808080u;
    }
    for (int i = lane; i < kOpSets * 32; i += kWave) opsets[i] = 128;
    __syncthreads();

    Rac c{0, 0xFF00, -1, 0, 0u, 0, 0};
    const Sink snk{a.slice_out + ((int64_t)f * a.nslices + slice) * a.slice_cap,
                   a.slice_cap, lane == 0};

    // key bit / in-band header / slice header
    {
      const int sel = key * a.nslices + slice;
      const Op* ops = a.ops + (int64_t)sel * kMaxOps;
      const int n = a.nops[sel];
      for (int k = 0; k < n; k++) {
        const Op op = ops[k];
        const uint8_t* t = tabs + (op.tab ? 512 : 0);
        uint8_t* st = opsets + op.set * 32;
        if (op.kind == kOpBit)
          rac_put_mem(c, snk, st, op.value, t);
        else
          rac_symbol(c, snk, st, op.value, op.kind == kOpSymS, t);
      }
    }

    for (int p = 0; p < nplanes; p++) {
      int px = x0, py = y0, pw = sw, ph = sh;
      if (p) {
        pw = -((-sw) >> a.hs);
        ph = -((-sh) >> a.vs);
        px = x0 >> a.hs;
        py = y0 >> a.vs;
      }
      uint8_t* pst = states + (int64_t)(p ? 1 : 0) * a.contexts * 32;
      const uint8_t* pbase = a.frames + (int64_t)f * a.frame_bytes + a.plane_off[p];
      const int stride = a.plane_stride[p];

      for (int i = lane; i < 3 * a.row_len; i += kWave) rows[i] = 0;
      __syncthreads();

      for (int y = 0; y < ph; y++) {
        int16_t* cur = rows + (y % 3) * a.row_len + 4;
        int16_t* prev = rows + ((y + 2) % 3) * a.row_len + 4;
        int16_t* prev2 = rows + ((y + 1) % 3) * a.row_len + 4;
        const uint8_t* src = pbase + (int64_t)(py + y) * stride;
        if (a.sample_bytes == 1) {
          for (int x = lane; x < pw; x += kWave) cur[x] = src[px + x];
        } else {
          const uint16_t* s16 = reinterpret_cast<const uint16_t*>(src) + px;
          for (int x = lane; x < pw; x += kWave) {
            unsigned v = s16[x];
            if (!a.packed_at_lsb) v >>= a.msb_shift;
            cur[x] = (int16_t)v;
          }
        }
        __syncthreads();
        if (lane == 0) {  // ring-buffer edge taps (ffv1enc.c:387-388)
          cur[-1] = prev[0];
          prev[pw] = prev[pw - 1];
        }
        __syncthreads();
        for (int x = lane; x < pw; x += kWave) {
          const int X = cur[x], L = cur[x - 1], T = prev[x], LT = prev[x - 1], RT = prev[x + 1];
          int ctx = qt[(L - LT) & 0xFF] + qt[256 + ((LT - T) & 0xFF)] + qt[512 + ((T - RT) & 0xFF)];
          if (a.model1)
            ctx += qt[768 + ((cur[x - 2] - L) & 0xFF)] + qt[1024 + ((prev2[x] - T) & 0xFF)];
          int diff = X - median3(L, L + T - LT, T);
          if (ctx < 0) {
            ctx = -ctx;
            diff = -diff;
          }
          diff = fold_bits(diff, a.coded_bits);
          sym[x] = (int32_t)(((uint32_t)ctx << 16) | (uint16_t)diff);
        }
        __syncthreads();
        for (int x = 0; x < pw; x++) {
          const int32_t s = sym[x];
          rac_symbol(c, snk, pst + (int64_t)(s >> 16) * 32, (int16_t)(s & 0xFFFF), true, ftab);
        }
        __syncthreads();
      }
    }
    // slice end: a 0 decision on state 129, then terminate (ffv1enc.c:1331-1334)
    (void)rac_put(c, snk, 129, 0, ftab);
    const int64_t bytes = rac_finish(c, snk);
    if (lane == 0) {
      a.slice_bytes[(int64_t)f * a.nslices + slice] = bytes;
      if (bytes > a.slice_cap) atomicAdd(a.status, 1);
    }
    __syncthreads();
  }

  if (seg.save_states) {
    uint8_t* dst = a.persist + (int64_t)slice * state_bytes;
    for (int64_t i = lane * 4; i < state_bytes; i += kWave * 4)
      *reinterpret_cast<uint32_t*>(dst + i) = *reinterpret_cast<const uint32_t*>(states + i);
  }
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
  const uint8_t* src = a.slice_out + ((int64_t)f * a.nslices + s) * a.slice_cap;
  uint8_t* dst = a.packets + (int64_t)f * a.packet_stride + off;

  auto body_byte = [&](int64_t i) -> uint32_t {
    if (i < n) return src[i];
    const int64_t k = i - n;
    if (has_size && k < 3) return (uint32_t)(n >> (8 * (2 - k))) & 0xFF;
    return 0u;  // the 0x00 before the CRC
  };

  for (int64_t i = t; i < body; i += kAsmThreads) dst[i] = (uint8_t)body_byte(i);

  if (a.ec) {
    const int64_t chunk = (body + kAsmThreads - 1) / kAsmThreads;
    const int64_t b0 = min((int64_t)t * chunk, body), b1 = min(b0 + chunk, body);
    uint32_t crc = 0;
    for (int64_t i = b0; i < b1; i++) crc = (crc << 8) ^ crc_tab[(crc >> 24) ^ body_byte(i)];
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

}  // namespace

size_t encode_lds_bytes(const EncodeArgs& a, bool lds_states) {
  return lds_layout(a, lds_states).total;
}

int launch_encode(const EncodeArgs& a, bool lds_states, void* stream) {
  const size_t lds = encode_lds_bytes(a, lds_states);
  dim3 grid(a.nslices, a.nsegs), block(kWave);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (lds_states) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&ffv1_encode_slices<true>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return -1;
    hipLaunchKernelGGL(ffv1_encode_slices<true>, grid, block, lds, st, a);
  } else {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&ffv1_encode_slices<false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return -1;
    hipLaunchKernelGGL(ffv1_encode_slices<false>, grid, block, lds, st, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_assemble(const AssembleArgs& a, int nframes, void* stream) {
  dim3 grid(a.nslices, nframes), block(kAsmThreads);
  hipLaunchKernelGGL(ffv1_assemble_packets, grid, block, 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace ffv1hip
