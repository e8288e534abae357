// ffv1_decode.hip -- FFV1 slice decoder on gfx950: the
// streams this library encodes, range coder or Golomb-Rice, context model 0
// or 1, YCbCr or RGB, versions 0, 1 and 3, with the reference's damaged-slice
// concealment.
//
// Reference: ffv1dec.c decode_frame (:896-1030), decode_slice (:361-474),
// decode_slice_header (:282-359), read_header for v0/v1 (:639-700),
// decode_line (:42-117 range and Golomb branches), decode_plane (:200-224),
// decode_rgb_frame (:226-280), get_symbol_inline (:44-66), get_vlc_symbol
// (:68-95); rangecoder.h get_rac / refill (:104-147); golomb.h get_ur_golomb
// / get_sr_golomb.  Decoding is a serial chain per (GOP segment, slice):
// each decision's context state and each sample's neighbourhood depend on
// the decisions before it.  One workgroup of one wave per chain keeps the
// chain's adaptive states (in LDS when they fit, else in a per-chain global
// table), the transition tables, the quant tables and two rows per plane in
// LDS; lane 0 runs the chain, the wave stores each decoded row (coalesced)
// and does the bulk state resets and copies.  A second kernel
// (ffv1_conceal) replaces damaged slices by the previous picture's
// rectangle, frame by frame, as decode_frame does after its slices.
#include "ffv1_internal.h"

namespace ffv1hip {
namespace {

constexpr int kDecThreads = 64;
constexpr int kInvalidData = -1094995529;  // AVERROR_INVALIDDATA, which get_symbol_inline returns as a value
constexpr uint64_t kVlcInit = (uint64_t)4 << 16 | (uint64_t)1 << 40;  // drift 0, error_sum 4, bias 0, count 1
constexpr uint8_t kDamageHeader = 2, kDamageEnd = 4;  // bit 0: the host's CRC check

__constant__ uint8_t kLog2Run[41] = {  // ff_log2_run (bitstream.c:40-46)
    0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 5, 5, 6,
    6, 7, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24};

struct RacDec {
  uint32_t low, range;
  int64_t ptr, end;  // byte offsets into the packet buffer
  uint64_t win;      // the bytes from ptr to the end of its 8-byte word, the one at ptr lowest
  uint64_t nxt;      // the word after it; bytes at or past end read as 0 in both
};

// word k of the packet buffer with the bytes at or past `end` zeroed (no
// load at all past it)
__device__ inline uint64_t rac_word(const uint64_t* w, int64_t k, int64_t end) {
  const int64_t b = k * 8;
  if (b >= end) return 0;
  const uint64_t v = w[k];
  return end - b >= 8 ? v : v & ((uint64_t(1) << ((end - b) * 8)) - 1u);
}

__device__ inline void rac_init(RacDec& c, const uint8_t* pk, int64_t start, int64_t end) {
  // ff_init_range_decoder + the first two bytes (rangecoder.c:53-61)
  const uint64_t* w = reinterpret_cast<const uint64_t*>(pk);
  c.range = 0xFF00;
  c.low = (uint32_t(pk[start]) << 8) | pk[start + 1];
  c.ptr = start + 2;
  c.end = end;
  c.win = rac_word(w, c.ptr >> 3, end) >> ((c.ptr & 7) * 8);
  c.nxt = rac_word(w, (c.ptr >> 3) + 1, end);
}

// refill (rangecoder.h:104-115): the byte at ptr is the window's lowest (0
// past the end); at a word boundary the next word moves in and the one after
// it is loaded, eight refills ahead of its use
__device__ inline void rac_refill(RacDec& c, const uint64_t* w) {
  c.range <<= 8;
  c.low = (c.low << 8) | uint32_t(c.win & 0xFFu);
  c.win >>= 8;
  c.ptr++;
  if (__builtin_amdgcn_ballot_w64((c.ptr & 7) == 0)) {  // (the active lanes agree)
    c.win = c.nxt;
    c.nxt = rac_word(w, (c.ptr >> 3) + 1, c.end);
  }
}

// get_rac (rangecoder.h:117-147), branch-free: the transition pair of the
// state (tt[s] = to0[s] | to1[s] << 8) is read beside the range arithmetic,
// so a decision waits on two LDS reads (state, pair) rather than three.
__device__ inline int rac_get(RacDec& c, uint8_t* st, const uint16_t* tt, const uint64_t* w) {
  const uint32_t s = *st;
  const uint32_t pair = tt[s];
  const uint32_t r1 = __umul24(c.range, s) >> 8;
  const uint32_t rr = c.range - r1;
  const int bit = c.low >= rr;
  c.low -= bit ? rr : 0u;
  c.range = bit ? r1 : rr;
  *st = uint8_t(bit ? pair >> 8 : pair);
  if (c.range < 0x100) rac_refill(c, w);
  return bit;
}

// get_symbol_inline (ffv1dec.c:44-66); an exponent past 31 returns
// AVERROR_INVALIDDATA, which decode_line then uses as the residual
__device__ inline int rac_symbol(RacDec& c, uint8_t* st, int is_signed, const uint16_t* tt,
                                 const uint64_t* w) {
  if (rac_get(c, st, tt, w)) return 0;
  int e = 0;
  while (rac_get(c, st + 1 + (e < 9 ? e : 9), tt, w)) {
    if (++e > 31) return kInvalidData;
  }
  uint32_t a = 1;
  for (int i = e - 1; i >= 0; i--) a = 2 * a + uint32_t(rac_get(c, st + 22 + (i < 9 ? i : 9), tt, w));
  if (is_signed && rac_get(c, st + 11 + (e < 10 ? e : 10), tt, w)) return int(0u - a);
  return int(a);
}

// readfirstlane: lane 0's value as a wave-uniform one
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t uni(int64_t v) {
  return int64_t((uint64_t(uni(uint32_t(uint64_t(v) >> 32))) << 32) | uni(uint32_t(v)));
}
__device__ __forceinline__ uint64_t uni(uint64_t v) { return (uint64_t(uni(uint32_t(v >> 32))) << 32) | uni(uint32_t(v)); }

__device__ inline int median3u(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }

// The range-coded rows on the vector units: the same chain on every lane in
// VGPRs (the compiler sees LDS-loaded, hence per-lane, values), so the CU's
// chains code on their SIMDs' VALUs in parallel instead of queueing on the
// CU's one scalar unit (six chains per CU: the scalar version spent ~100 CU
// cycles per decision, 6.6 s for a 288-frame 4K batch).  A decision reads
// its state from the row image (registers), looks its successor pair up in
// the LDS table off the decision chain, and a row's image is written back by
// lane 0 once per symbol.
__device__ __forceinline__ uint32_t vreg(uint32_t v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ uint64_t vreg(uint64_t v) { return (uint64_t(vreg(uint32_t(v >> 32))) << 32) | vreg(uint32_t(v)); }
__device__ __forceinline__ int64_t vreg(int64_t v) { return int64_t(vreg(uint64_t(v))); }

// lane 0's coder (after the slice header) on every lane, in VGPRs
__device__ __forceinline__ void vec_coder(RacDec& c) {
  c.low = vreg(uni(c.low));
  c.range = vreg(uni(c.range));
  c.ptr = vreg(uni(c.ptr));
  c.end = vreg(uni(c.end));
  c.win = vreg(uni(c.win));
  c.nxt = vreg(uni(c.nxt));
}

__device__ __forceinline__ int get_v(RacDec& c, uint32_t src, uint32_t& dst, int SH, const uint16_t* tt,
                                     const uint64_t* w) {
  const uint32_t s = (src >> SH) & 0xFFu;
  const uint32_t pair = tt[s];  // to0 | to1 << 8, for the row image only
  const uint32_t r1 = __umul24(c.range, s) >> 8;
  const uint32_t rr = c.range - r1;
  // every lane holds the same coder: the selects take the compare's lane
  // mask as it is, and its ballot is the bit, so the branches on it are
  // scalar (no exec-mask save and restore)
  const bool lb = c.low >= rr;
  c.low -= lb ? rr : 0u;
  c.range = lb ? r1 : rr;
  const bool bit = __builtin_amdgcn_ballot_w64(lb) != 0;
  // the successor into byte SH / 8 of the image: one byte permute (pair's
  // byte 1 on a 1, byte 0 on a 0; the image's other bytes as they are)
  const uint32_t keep = 0x03020100u & ~(0xFFu << SH);
  dst = __builtin_amdgcn_perm(pair, dst, keep | ((bit ? 5u : 4u) << SH));
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(c.range < 0x100u) != 0, 0)) rac_refill(c, w);
  return bit;
}
// (Reading the pairs of the likely next decisions one decision ahead
// measured slower: 3.37 -> 3.66 s for a 12-frame 4K GOP; the waits for the
// in-order LDS counter then cover the prefetches too.)

// get_rac on state s, the decision alone: symbol_v updates the row's states
// once per symbol, one slot per lane
__device__ __forceinline__ bool dec_s(RacDec& c, uint32_t s, const uint64_t* w) {
  const uint32_t r1 = __umul24(c.range, s) >> 8;
  const uint32_t rr = c.range - r1;
  const bool lb = c.low >= rr;  // (see get_v)
  c.low -= lb ? rr : 0u;
  c.range = lb ? r1 : rr;
  // a refill is the rare case: the common path falls through
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(c.range < 0x100u) != 0, 0)) rac_refill(c, w);
  return __builtin_amdgcn_ballot_w64(lb) != 0;
}

template <int K>
__device__ __forceinline__ bool dec_k(RacDec& c, const uint32_t (&r)[8], const uint64_t* w) {
  return dec_s(c, (r[K >> 2] >> ((K & 3) * 8)) & 0xFFu, w);
}

// the exponent's unary run on slots K..9 (e = K-1 on entry)
template <int K>
__device__ __forceinline__ void unary_v(RacDec& c, const uint32_t (&r)[8], int& e, const uint64_t* w) {
  if constexpr (K <= 9) {
    if (dec_k<K>(c, r, w)) {
      e = K;
      unary_v<K + 1>(c, r, e, w);
    }
  }
}

// mantissa bits i = min(e, 9) - 1 .. 0 on slots 22 + i: one jump into the
// run by the bit count (a compare and branch per bit before)
__device__ __forceinline__ void mant_v(RacDec& c, const uint32_t (&r)[8], int e, uint32_t& a, const uint64_t* w) {
#define FFV1_MANT(I) a = 2 * a + uint32_t(dec_k<22 + (I)>(c, r, w))
  switch (e < 9 ? e : 9) {
    case 9: FFV1_MANT(8); [[fallthrough]];
    case 8: FFV1_MANT(7); [[fallthrough]];
    case 7: FFV1_MANT(6); [[fallthrough]];
    case 6: FFV1_MANT(5); [[fallthrough]];
    case 5: FFV1_MANT(4); [[fallthrough]];
    case 4: FFV1_MANT(3); [[fallthrough]];
    case 3: FFV1_MANT(2); [[fallthrough]];
    case 2: FFV1_MANT(1); [[fallthrough]];
    case 1: FFV1_MANT(0); [[fallthrough]];
    default: break;
  }
#undef FFV1_MANT
}

// get_symbol_inline (ffv1dec.c:44-66), signed, on the row at `row`.  The
// decisions read their states from the row as read (every slot but 10 and 31
// codes at most one decision of a symbol); then each lane k < 32 (and its
// twin k + 32) moves slot k's state on by the slot's decision, if it had
// one, with the successor pair it looked up when the symbol started, and
// writes it back: no table lookup and no wait on the decision chain.  Slots
// 10 and 31, which repeat past e = 9, go through get_v in the row image n.
__device__ inline int symbol_v(RacDec& c, uint8_t* row, const uint16_t* tt, const uint64_t* w) {
  const int k = threadIdx.x & 31;
  const uint4* r4 = reinterpret_cast<const uint4*>(row);
  const uint4 a0 = r4[0], a1 = r4[1];
  const uint32_t sk = row[k];     // this lane's slot state
  const uint32_t pk = tt[sk];     // and its successor pair, beside the decisions
  const uint32_t r[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
  uint32_t n2 = r[2], n7 = r[7];  // slots 10 and 31 after their runs
  int ret;
  // what the symbol coded: zero flag zf; else the exponent e (> 31: invalid,
  // slots 1..10 only), the magnitude and the sign
  bool zf, neg = false;
  int e = 0;
  uint32_t a = 1;
  zf = dec_k<0>(c, r, w);
  if (zf) {
    ret = 0;
  } else {
    unary_v<1>(c, r, e, w);
    if (e == 9) {  // slot 10 for the rest of the run: its state from n after its first decision
      uint32_t src = r[2];
      while (get_v(c, src, n2, 16, tt, w)) {
        src = n2;
        if (++e > 31) break;
      }
    }
    if (e > 31) {
      ret = kInvalidData;
    } else {
      uint32_t src = r[7];
      for (int i = e - 1; i >= 9; i--) {  // slot 31
        a = 2 * a + uint32_t(get_v(c, src, n7, 24, tt, w));
        src = n7;
      }
      mant_v(c, r, e, a, w);
      const int j = 11 + (e < 10 ? e : 10);  // the sign slot, row words 2..5
      const int q = j >> 2;
      const uint32_t wd = q == 2 ? r[2] : q == 3 ? r[3] : q == 4 ? r[4] : r[5];
      neg = dec_s(c, (wd >> ((j & 3) * 8)) & 0xFFu, w);
      ret = neg ? int(0u - a) : int(a);
    }
  }
  // lane k: slot k's decision (put_symbol_inline's slot order, ffv1enc.c:185-231)
  const bool ok = e <= 31;
  const int em = e < 9 ? e : 9;
  bool t, b;
  if (k == 0) {
    t = true;
    b = zf;
  } else if (zf) {
    t = b = false;
  } else if (k <= 9) {
    t = k <= e + 1;
    b = k <= e;
  } else if (k >= 11 && k <= 21) {
    t = ok && k == 11 + (e < 10 ? e : 10);
    b = neg;
  } else if (k >= 22 && k <= 30) {
    t = ok && k - 22 < em;
    b = ((a >> (k - 22)) & 1u) != 0;
  } else {
    t = b = false;  // 10, 31: from n2 / n7
  }
  uint32_t ns = t ? (b ? (pk >> 8) & 0xFFu : pk & 0xFFu) : sk;
  ns = k == 10 ? (n2 >> 16) & 0xFFu : (k == 31 ? n7 >> 24 : ns);
  row[k] = uint8_t(ns);
  return ret;
}

// decode_line (ffv1dec.c:42-117), range coder, by the whole wave on
// per-lane copies of the same values (see symbol_v); quant tables in LDS
__device__ inline void decode_row_v(RacDec& c, uint8_t* st8, const uint16_t* tt, const uint64_t* pkw,
                                    const int16_t* qt, bool model1, int16_t* cur, const int16_t* up, int w,
                                    int bits) {
  const int mask = int((1u << bits) - 1u);
  int T = up[0];
  const int T0 = T;
  int L = T;
  int LT = cur[0];
  int RT = w > 1 ? up[1] : T;
  for (int x = 0; x < w; x++) {
    const int RTn = x + 2 < w ? up[x + 2] : (x + 1 < w ? RT : T);  // the next sample's, read a sample ahead
    int ctx = qt[(L - LT) & 0xFF] + qt[256 + ((LT - T) & 0xFF)] + qt[512 + ((T - RT) & 0xFF)];
    if (model1) {
      const int LL = x >= 2 ? int(cur[x - 2]) : (x == 1 ? T0 : 0);
      const int TT = cur[x];
      ctx += qt[768 + ((LL - L) & 0xFF)] + qt[1024 + ((TT - T) & 0xFF)];
    }
    const int actx = ctx < 0 ? -ctx : ctx;
    int diff = symbol_v(c, st8 + actx * 32, tt, pkw);
    if (ctx < 0) diff = -diff;
    const int pred = median3u(L, L + T - LT, T);
    const int v = int(int16_t((pred + diff) & mask));
    cur[x] = int16_t(v);  // every lane the same value to the same address: no exec mask to set up
    LT = T;
    T = RT;
    RT = RTn;
    L = v;
  }
}

// decode_line's slice_coding_mode 1 (version 4 PCM, ffv1dec.c:111-120): every
// sample's bits MSB first, each on a fresh state 128, on vector registers
__device__ inline void decode_row_pcm_v(RacDec& c, const uint64_t* pkw, int16_t* cur, int w, int bits) {
  for (int x = 0; x < w; x++) {
    int v = 0;
    for (int i = 0; i < bits; i++) {
      const uint32_t r1 = c.range >> 1;  // range * 128 >> 8
      const uint32_t rr = c.range - r1;
      const int bit = __builtin_amdgcn_ballot_w64(c.low >= rr) != 0;
      c.low -= bit ? rr : 0u;
      c.range = bit ? r1 : rr;
      if (__builtin_amdgcn_ballot_w64(c.range < 0x100u)) rac_refill(c, pkw);
      v = 2 * v + bit;
    }
    cur[x] = int16_t(v);
  }
}

// GetBitContext over a slice's Golomb bits: MSB first, zeros past the end
// (the safe bitstream reader).
struct BitRd {
  const uint8_t* pk;
  int64_t pos, end;  // next byte to load, end of the slice
  uint64_t cache;    // valid bits MSB-aligned
  int nc;
};

__device__ inline void br_fill(BitRd& b) {
  while (b.nc <= 56) {
    const uint64_t v = b.pos < b.end ? b.pk[b.pos] : 0u;
    b.pos++;
    b.cache |= v << (56 - b.nc);
    b.nc += 8;
  }
}

__device__ inline uint32_t br_bits(BitRd& b, int n) {
  if (n == 0) return 0;
  br_fill(b);
  const uint32_t v = uint32_t(b.cache >> (64 - n));
  b.cache <<= n;
  b.nc -= n;
  return v;
}

__device__ inline int fold_bits(int d, int bits) {
  const int sh = 32 - bits;
  return (d << sh) >> sh;
}

// get_vlc_symbol (ffv1dec.c:68-95): get_sr_golomb(k, limit 12, esc bits)
// and update_vlc_state (ffv1.h:192-224) on the packed VlcState record
// drift (int16) | error_sum (u16) << 16 | bias (int8) << 32 | count << 40.
__device__ inline int vlc_get(BitRd& b, uint64_t& rec, int bits) {
  int drift = int16_t(rec & 0xFFFF);
  int error_sum = int((rec >> 16) & 0xFFFF);
  int bias = int8_t((rec >> 32) & 0xFF);
  int count = int((rec >> 40) & 0xFF);
  int k = 0;
  for (int i = count; i < error_sum; i += i) k++;
  br_fill(b);
  const int q = b.cache ? __clzll(b.cache) : 64;
  uint32_t u;
  if (q < 12) {
    b.cache <<= q + 1;
    b.nc -= q + 1;
    u = (uint32_t(q) << k) | br_bits(b, k);
  } else {
    b.cache <<= 12;
    b.nc -= 12;
    u = br_bits(b, bits) + 11;
  }
  int v = (u & 1) ? -int((u + 1) >> 1) : int(u >> 1);
  v ^= (2 * drift + count) >> 31;
  const int ret = fold_bits(v + bias, bits);
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
  rec = (uint64_t)(uint16_t)drift | (uint64_t)(uint16_t)error_sum << 16 | (uint64_t)(uint8_t)bias << 32 |
        (uint64_t)(uint8_t)count << 40;
  return ret;
}

__device__ inline int median3(int a, int b, int c) {
  return max(min(a, b), min(max(a, b), c));
}

// decode_line (ffv1dec.c:42-117) for one row into `cur`, which holds row y-2
// until each sample is written; `up` is row y-1.  The neighbourhood is the
// reference's zeroed ring: L(0) = T(0), LT(0) = row y-2 at 0, RT past the
// edge = T, LL(0) = 0, LL(1) = T(0), TT = row y-2.
template <bool GOLOMB>
__device__ inline void decode_row(RacDec& c, BitRd& b, uint8_t* st8, uint64_t* st64, const uint16_t* tt,
                                  const uint64_t* pkw, const int16_t* qt, bool model1, int16_t* cur,
                                  const int16_t* up, int w, int bits, int& run_index) {
  const int mask = int((1u << bits) - 1u);
  int T = up[0];
  const int T0 = T;
  int L = T;
  int LT = cur[0];
  int run_count = 0, run_mode = 0;
  for (int x = 0; x < w; x++) {
    const int RT = x + 1 < w ? up[x + 1] : T;
    int ctx = qt[(L - LT) & 0xFF] + qt[256 + ((LT - T) & 0xFF)] + qt[512 + ((T - RT) & 0xFF)];
    if (model1) {
      const int LL = x >= 2 ? cur[x - 2] : (x == 1 ? T0 : 0);
      const int TT = cur[x];
      ctx += qt[768 + ((LL - L) & 0xFF)] + qt[1024 + ((TT - T) & 0xFF)];
    }
    const int actx = ctx < 0 ? -ctx : ctx;
    int diff;
    if constexpr (!GOLOMB) {
      // one call site: the symbol decoder is the kernel's hot code
      diff = rac_symbol(c, st8 + actx * 32, 1, tt, pkw);
    } else {
      if (actx == 0 && run_mode == 0) run_mode = 1;
      if (run_mode) {
        if (run_count == 0 && run_mode == 1) {
          if (br_bits(b, 1)) {
            run_count = 1 << kLog2Run[run_index];
            if (x + run_count <= w) run_index++;
          } else {
            run_count = kLog2Run[run_index] ? int(br_bits(b, kLog2Run[run_index])) : 0;
            if (run_index) run_index--;
            run_mode = 2;
          }
        }
        run_count--;
        if (run_count < 0) {
          run_mode = 0;
          run_count = 0;
          diff = vlc_get(b, st64[actx], bits);
          if (diff >= 0) diff++;
        } else {
          diff = 0;
        }
      } else {
        diff = vlc_get(b, st64[actx], bits);
      }
    }
    if (ctx < 0) diff = -diff;
    const int pred = median3(L, L + T - LT, T);
    const int16_t v = int16_t((pred + diff) & mask);
    cur[x] = v;
    LT = T;
    T = RT;
    L = v;
  }
}

// read_quant_table (ffv1dec.c:475-497): consumes one table's run lengths
__device__ inline bool skip_quant_table(RacDec& c, uint8_t* st, const uint16_t* tt, const uint64_t* w) {
  for (int i = 0; i < 32; i++) st[i] = 128;
  int i = 0;
  while (i < 128) {
    const unsigned len = unsigned(rac_symbol(c, st, 0, tt, w)) + 1u;
    if (len > unsigned(128 - i) || !len) return false;
    i += int(len);
  }
  return true;
}

template <bool GOLOMB, bool GSTATES>
__global__ void __launch_bounds__(kDecThreads) ffv1_decode_slices(DecodeArgs a) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int s = blockIdx.x, seg = blockIdx.y, lane = threadIdx.x;
  const Segment sg = a.segs[seg];
  const SliceGeom* g = a.geom + s;  // read through the pointer: a by-value copy indexed by plane spills
  // swap mode (range coder, YCbCr): the LDS holds one plane group's states,
  // the chain's other group waits in its global table (a.tables) and the two
  // trade places where the plane group changes (twice a frame), so that twice
  // the chains fit on a CU
  const bool swap = !GSTATES && a.swap;
  const int64_t sb = GSTATES ? 0 : ((swap ? a.state_bytes / 2 : a.state_bytes) + 15) & ~int64_t(15);
  uint8_t* const states = GSTATES ? a.tables + (int64_t(seg) * a.nslices + s) * a.state_bytes : lds;
  uint32_t* const bk4 = swap ? reinterpret_cast<uint32_t*>(a.tables + (int64_t(seg) * a.nslices + s) * a.state_bytes)
                             : nullptr;
  uint16_t* const tt = reinterpret_cast<uint16_t*>(lds + sb);  // [256] frame table to0 | to1 << 8
  uint16_t* const dtt = tt + 256;                              // [256] default table
  uint8_t* const hdr = reinterpret_cast<uint8_t*>(dtt + 256);  // [32] header states, [32] scratch
  int16_t* const qt = reinterpret_cast<int16_t*>(hdr + 64);    // [5][256]
  // [5][256] with context model 1, [3][256] otherwise (its LL / TT tables
  // unused): 1 KB less per chain, so that six chains fit on a CU (a 24-GOP
  // 4K batch, 1536 chains, then decodes in one round instead of two)
  const int nq = a.context_model ? 5 : 3;
  int16_t* const ring = qt + nq * 256;                         // [rgb ? 3 : 1][2][row_cap]
  __shared__ int bad;
  __shared__ int s_reset, s_pcm, s_by, s_ry;  // v4 slice header: reset, slice_coding_mode, RCT coefficients
  const uint64_t* pkw = reinterpret_cast<const uint64_t*>(a.pkts);
  for (int i = lane; i < 256; i += kDecThreads) {
    tt[i] = uint16_t(a.ftab[i] | (a.ftab[256 + i] << 8));
    dtt[i] = uint16_t(a.dtab[i] | (a.dtab[256 + i] << 8));
  }
  for (int i = lane; i < nq * 256; i += kDecThreads) qt[i] = a.qt[i];
  const int bits = a.coded_bits;
  const bool model1 = a.context_model != 0;
  const int64_t words = a.state_bytes / 4;
  const int64_t hw = words / 2;  // one plane group
  uint32_t* const st4 = reinterpret_cast<uint32_t*>(states);
  int cur = 0;  // swap mode: the plane group in the LDS
  // the chain continues the states the previous call left (the decoder
  // starts them reset)
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.persist_in + int64_t(s) * a.state_bytes);
    if (swap) {
      for (int64_t i = lane; i < hw; i += kDecThreads) {
        st4[i] = src[i];
        bk4[hw + i] = src[hw + i];
      }
    } else {
      for (int64_t i = lane; i < words; i += kDecThreads) st4[i] = src[i];
    }
  }
  RacDec c{};
  BitRd br{};
  for (int j = 0; j < sg.nframes; j++) {
    const int f = sg.first_frame + j;
    const int key = a.keyflags[f];
    const int64_t fs = int64_t(f) * a.nslices + s;
    __syncthreads();
    if (lane == 0) {
      rac_init(c, a.pkts, a.slice_start[fs], a.slice_end[fs]);
      int ok = 1, hok = 1;
      s_reset = 0;
      s_pcm = 0;
      s_by = s_ry = 1;
      if (s == 0) {  // the key bit, state 128 (ffv1dec.c:927-933)
        hdr[0] = 128;
        ok &= rac_get(c, hdr, dtt, pkw) == key;
        if (key && a.version < 2) {  // read_header, in band (ffv1dec.c:646-700)
          for (int i = 0; i < 32; i++) hdr[i] = 128;
          ok &= rac_symbol(c, hdr, 0, dtt, pkw) == a.version;
          ok &= rac_symbol(c, hdr, 0, dtt, pkw) == a.ac;
          if (a.ac == 2)
            for (int i = 1; i < 256; i++) (void)rac_symbol(c, hdr, 1, dtt, pkw);  // the table this decoder was built with
          ok &= rac_symbol(c, hdr, 0, dtt, pkw) == a.rgb;
          if (a.version > 0) ok &= rac_symbol(c, hdr, 0, dtt, pkw) == a.bits_per_raw_sample;
          ok &= rac_get(c, hdr, dtt, pkw) == a.chroma_planes;
          ok &= rac_symbol(c, hdr, 0, dtt, pkw) == a.chroma_h_shift;
          ok &= rac_symbol(c, hdr, 0, dtt, pkw) == a.chroma_v_shift;
          ok &= rac_get(c, hdr, dtt, pkw) == a.transparency;
          for (int t = 0; t < 5 && ok; t++) ok &= skip_quant_table(c, hdr + 32, dtt, pkw);
        } else if (key && a.version == 2) {
          // read_header's v2 branch (ffv1dec.c:801-868): the slice count,
          // each slice's rectangle in grid units and every plane's quant set,
          // one state array; a stream naming another layout than the grid's
          // is refused (distinct symbols name distinct rectangles here)
          for (int i = 0; i < 32; i++) hdr[i] = 128;
          const int n = a.num_h * a.num_v;
          ok &= rac_symbol(c, hdr, 0, dtt, pkw) == n;
          for (int j = 0; j < n && ok; j++) {
            const int jx = j % a.num_h, jy = j / a.num_h;
            const int x0 = int(int64_t(a.width) * jx / a.num_h), x1 = int(int64_t(a.width) * (jx + 1) / a.num_h);
            const int y0 = int(int64_t(a.height) * jy / a.num_v), y1 = int(int64_t(a.height) * (jy + 1) / a.num_v);
            ok &= rac_symbol(c, hdr, 0, dtt, pkw) == int(int64_t(x0 + 1) * a.num_h / a.width);
            ok &= rac_symbol(c, hdr, 0, dtt, pkw) == int(int64_t(y0 + 1) * a.num_v / a.height);
            ok &= rac_symbol(c, hdr, 0, dtt, pkw) == int(int64_t(x1 - x0 + 1) * a.num_h / a.width) - 1;
            ok &= rac_symbol(c, hdr, 0, dtt, pkw) == int(int64_t(y1 - y0 + 1) * a.num_v / a.height) - 1;
            for (int i = 0; i < a.pcount && ok; i++) ok &= rac_symbol(c, hdr, 0, dtt, pkw) == a.context_model;
          }
        }
      }
      if (a.version > 2) {
        // decode_slice_header (ffv1dec.c:282-359); a slice naming another
        // rectangle or quant set than the grid's counts as damaged
        for (int i = 0; i < 32; i++) hdr[i] = 128;
        const int sx = rac_symbol(c, hdr, 0, tt, pkw);
        const int sy = rac_symbol(c, hdr, 0, tt, pkw);
        const int sw = rac_symbol(c, hdr, 0, tt, pkw);
        const int sh = rac_symbol(c, hdr, 0, tt, pkw);
        const int x0 = int(int64_t(sx) * a.width / a.num_h), y0 = int(int64_t(sy) * a.height / a.num_v);
        const int x1 = int(int64_t(sx + sw + 1) * a.width / a.num_h);
        const int y1 = int(int64_t(sy + sh + 1) * a.height / a.num_v);
        hok &= sx >= 0 && sy >= 0 && sw >= 0 && sh >= 0;
        hok &= x0 == g->px[0] && y0 == g->py[0] && x1 - x0 == g->pw[0] && y1 - y0 == g->ph[0];
        for (int i = 0; i < a.pcount && hok; i++) hok &= rac_symbol(c, hdr, 0, tt, pkw) == a.context_model;
        if (hok) {
          (void)rac_symbol(c, hdr, 0, tt, pkw);  // picture structure
          (void)rac_symbol(c, hdr, 0, tt, pkw);  // sample aspect ratio
          (void)rac_symbol(c, hdr, 0, tt, pkw);
        }
        if (hok && a.version > 3) {  // ffv1dec.c:344-356
          s_reset = rac_get(c, hdr, tt, pkw);
          s_pcm = rac_symbol(c, hdr, 0, tt, pkw);
          if (s_pcm != 1) {
            s_by = rac_symbol(c, hdr, 0, tt, pkw);
            s_ry = rac_symbol(c, hdr, 0, tt, pkw);
            hok &= unsigned(s_by) + unsigned(s_ry) <= 4u;
          }
          hok &= s_pcm == 0 || s_pcm == 1;  // modes this decoder codes (the reference reads only these too)
        }
      }
      if (!ok) atomicAdd(&a.status[0], 1);
      bad = !ok ? 2 : !hok ? 1 : 0;
      if (!hok) a.damage[fs] |= kDamageHeader;
    }
    __syncthreads();
    if (bad == 2) return;
    if (bad) continue;  // not decoded: no state update (ffv1dec.c:410-414)
    const bool pcm = s_pcm == 1;
    const int rby = s_by, rry = s_ry;
    if (key || s_reset) {  // ff_ffv1_clear_slice_state, after the header (ffv1dec.c:418-419)
      if (swap) {  // the LDS group and the other group in the global table
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.init);
        for (int64_t i = lane; i < hw; i += kDecThreads) {
          const uint32_t v = a.init ? src[i] : 0x80808080u;
          st4[i] = v;
          bk4[(cur ^ 1) * hw + i] = v;
        }
      } else if (!GOLOMB && a.init) {  // initial states from the extradata (ffv1.c:185-189)
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.init);
        for (int64_t i = lane; i < words; i += kDecThreads) st4[i] = src[i % (words / a.pcount)];
      } else {
        const uint32_t v0 = GOLOMB ? uint32_t(kVlcInit) : 0x80808080u;
        const uint32_t v1 = GOLOMB ? uint32_t(kVlcInit >> 32) : 0x80808080u;
        for (int64_t i = lane; i < words; i += kDecThreads) st4[i] = (i & 1) ? v1 : v0;
      }
    }
    if (lane == 0 && GOLOMB) {  // ffv1dec.c:426-433
      if (a.version > 2) {        // micro_version 4: a 0 on state 129, then the Golomb bits
        hdr[32] = 129;
        (void)rac_get(c, hdr + 32, tt, pkw);
      }
      const int64_t start = a.slice_start[fs];
      const int64_t acb = (a.version > 2 || (g->px[0] == 0 && g->py[0] == 0)) ? c.ptr - start - 1 : 0;
      br.pk = a.pkts;
      br.pos = start + acb;
      br.end = a.slice_end[fs];
      br.cache = 0;
      br.nc = 0;
    }
    if constexpr (!GOLOMB) vec_coder(c);  // lane 0's coder after the header, to every lane
    int run_index = 0;
    uint8_t* const obase = a.out + int64_t(f) * a.frame_bytes;
    const int64_t per = a.state_bytes / a.pcount;  // one plane context's states
    if (!a.rgb) {
      // decode_slice (ffv1dec.c:435-453): Y, Cb, Cr (plane context 1), A
      // (plane context 2) at the luma size; YA8: Y and A (context 1) of the
      // one packed plane, every second byte
      const int ncoded = a.ya8 ? 2 : a.nplanes;
      for (int p = 0; p < ncoded; p++) {
        for (int i = lane; i < 2 * a.row_cap; i += kDecThreads) ring[i] = 0;
        const int grp = a.ya8 ? p : (p == 0 ? 0 : p < 3 ? 1 : 2);
        if (swap && grp != cur) {  // the other plane group's states into the LDS
          __syncthreads();
          for (int64_t i = lane; i < hw; i += kDecThreads) {
            const uint32_t v = bk4[grp * hw + i];
            bk4[cur * hw + i] = st4[i];
            st4[i] = v;
          }
          cur = grp;
        }
        __syncthreads();
        // decode_plane (ffv1dec.c:200-224): lane 0 decodes a row into LDS;
        // the wave then stores it (coalesced), so the serial loop issues no
        // global stores
        uint8_t* pst = states + (swap ? 0 : grp * per);
        const int gp = a.ya8 ? 0 : p;  // geometry of the plane
        const int w = g->pw[gp], h = g->ph[gp];
        const int op = a.ya8 ? 0 : p;  // output plane
        const int64_t poff = (op == 0 ? a.plane_off[0] : op == 1 ? a.plane_off[1] : op == 2 ? a.plane_off[2]
                                                                                      : a.plane_off[3]) +
                             (a.ya8 ? p : 0);
        const int pw = op == 0 ? a.plane_w[0] : op == 1 ? a.plane_w[1] : op == 2 ? a.plane_w[2] : a.plane_w[3];
        const int step = a.ya8 ? 2 : 1;
        run_index = 0;  // per plane (ffv1dec.c:204)
        for (int y = 0; y < h; y++) {
          int16_t* cur = ring + (y & 1) * a.row_cap;  // holds row y-2 until written
          const int16_t* up = ring + ((y + 1) & 1) * a.row_cap;
          if constexpr (!GOLOMB) {
            if (pcm)
              decode_row_pcm_v(c, pkw, cur, w, bits);
            else
              decode_row_v(c, pst, tt, pkw, qt, model1, cur, up, w, bits);
          } else if (lane == 0) {
            decode_row<GOLOMB>(c, br, pst, reinterpret_cast<uint64_t*>(pst), tt, pkw, qt, model1, cur, up, w, bits,
                               run_index);
          }
          __syncthreads();
          const int64_t orow = int64_t(g->py[gp] + y) * pw + int64_t(g->px[gp]) * step;
          if (a.sample_bytes == 1) {
            for (int x = lane; x < w; x += kDecThreads) obase[poff + orow + int64_t(x) * step] = uint8_t(cur[x]);
          } else {
            uint16_t* o16 = reinterpret_cast<uint16_t*>(obase + poff) + orow;
            for (int x = lane; x < w; x += kDecThreads) {
              const uint32_t u = uint16_t(cur[x]);
              o16[x] = uint16_t(a.packed_at_lsb ? u : (u << a.msb_shift));
            }
          }
          __syncthreads();
        }
      }
    } else {
      // decode_rgb_frame (ffv1dec.c:226-280): the rows of G', B', R' in
      // turn, one run index for the slice, then the inverse transform
      // (p + 1) / 2: G' context 0, B' and R' 1, A 2; PCM rows (v4 slice_coding_mode 1)
      // at the raw depth, untransformed
      const int np = 3 + (a.transparency ? 1 : 0);
      for (int i = lane; i < 2 * np * a.row_cap; i += kDecThreads) ring[i] = 0;
      __syncthreads();
      const int w = g->pw[0], h = g->ph[0];
      const int pbits = a.bits_per_raw_sample <= 8 ? 8 : a.bits_per_raw_sample;
      for (int y = 0; y < h; y++) {
        for (int p = 0; p < np; p++) {
          uint8_t* pst = states + ((p + 1) / 2) * per;
          int16_t* cur = ring + (2 * p + (y & 1)) * a.row_cap;
          const int16_t* up = ring + (2 * p + ((y + 1) & 1)) * a.row_cap;
          if constexpr (!GOLOMB) {
            if (pcm)
              decode_row_pcm_v(c, pkw, cur, w, pbits);
            else
              decode_row_v(c, pst, tt, pkw, qt, model1, cur, up, w, bits);
          } else if (lane == 0) {
            decode_row<GOLOMB>(c, br, pst, reinterpret_cast<uint64_t*>(pst), tt, pkw, qt, model1, cur, up, w, bits,
                               run_index);
          }
        }
        __syncthreads();
        const int16_t* G = ring + (y & 1) * a.row_cap;
        const int16_t* B = ring + (2 + (y & 1)) * a.row_cap;
        const int16_t* R = ring + (4 + (y & 1)) * a.row_cap;
        const int16_t* A = ring + (6 + (y & 1)) * a.row_cap;
        const int64_t Y = g->py[0] + y;
        for (int x = lane; x < w; x += kDecThreads) {
          int gg = G[x], bb = B[x], rr = R[x];
          if (!pcm) {  // ffv1dec.c:258-264, with the slice's RCT coefficients (1, 1 below v4)
            bb -= a.rct_offset;
            rr -= a.rct_offset;
            gg -= (bb * rby + rr * rry) >> 2;
            bb += gg;
            rr += gg;
          }
          const int64_t X = g->px[0] + x;
          if (a.sample_bytes == 4) {  // *(uint32_t *) = b + (g << 8) + (r << 16) + (a << 24)
            const uint32_t av = a.transparency ? uint32_t(uint16_t(A[x])) : 0u;
            reinterpret_cast<uint32_t*>(obase + a.plane_off[0] + Y * a.plane_w[0] * 4)[X] =
                uint32_t(bb) + (uint32_t(gg) << 8) + (uint32_t(rr) << 16) + (av << 24);
          } else {
            reinterpret_cast<uint16_t*>(obase + a.plane_off[0] + Y * a.plane_w[0] * 2)[X] = uint16_t(bb);
            reinterpret_cast<uint16_t*>(obase + a.plane_off[1] + Y * a.plane_w[1] * 2)[X] = uint16_t(gg);
            reinterpret_cast<uint16_t*>(obase + a.plane_off[2] + Y * a.plane_w[2] * 2)[X] = uint16_t(rr);
          }
        }
        __syncthreads();
      }
    }
    if (lane == 0 && !GOLOMB && a.version > 2) {  // ffv1dec.c:461-467: where the slice's bytes end
      hdr[32] = 129;
      (void)rac_get(c, hdr + 32, tt, pkw);
      if (c.end - c.ptr - 2 - 5 * a.ec) a.damage[fs] |= kDamageEnd;
    }
  }
  __syncthreads();
  if (sg.save_states) {
    uint32_t* dst = reinterpret_cast<uint32_t*>(a.persist_out + int64_t(s) * a.state_bytes);
    if (swap) {
      for (int64_t i = lane; i < hw; i += kDecThreads) {
        dst[cur * hw + i] = st4[i];
        dst[(cur ^ 1) * hw + i] = bk4[(cur ^ 1) * hw + i];
      }
    } else {
      for (int64_t i = lane; i < words; i += kDecThreads) dst[i] = st4[i];
    }
  }
}

// decode_frame's concealment (ffv1dec.c:998-1021), one block per slice over
// the batch's frames in order: slice_damaged is set by a CRC, header or end
// mismatch and cleared only by a keyframe's read_header (:820-825); a
// damaged slice with a rectangle takes the previous picture's.  The x offset
// is (slice_x >> shift) << (depth > 8), as the reference computes it, which
// for packed bgr0 is slice_x bytes.
__global__ void __launch_bounds__(256) ffv1_conceal(DecodeArgs a) {
  const int s = blockIdx.x;
  const SliceGeom* g = a.geom + s;
  uint8_t sticky = a.sticky[s];
  const int np = (a.rgb && a.sample_bytes == 4) || a.ya8 ? 1 : a.nplanes;
  for (int f = 0; f < a.nframes; f++) {
    if (a.keyflags[f]) sticky = 0;
    const uint8_t dmg = a.damage[int64_t(f) * a.nslices + s];
    sticky |= dmg != 0;
    const uint8_t* src = f ? a.out + int64_t(f - 1) * a.frame_bytes : a.last;
    if (!sticky || (dmg & kDamageHeader) || !src) continue;
    uint8_t* dst = a.out + int64_t(f) * a.frame_bytes;
    for (int k = 0; k < np; k++) {
      // planes 1 and 2 are the subsampled ones; the x offset takes the
      // component depth (> 8 bits: << 1), not the pixel size (ffv1dec.c:1006-1011)
      const bool sub = k == 1 || k == 2;
      const int hs = sub ? a.chroma_h_shift : 0, vs = sub ? a.chroma_v_shift : 0;
      const int bpp = a.sample_bytes;
      const int64_t row = int64_t(a.plane_w[k]) * bpp;
      const int64_t xoff = int64_t(g->px[0] >> hs) << (bpp == 2 ? 1 : 0);
      const int64_t bytes = int64_t(-((-g->pw[0]) >> hs)) * bpp * (a.ya8 ? 2 : 1);
      const int rows = -((-g->ph[0]) >> vs);
      const int64_t y0 = g->py[0] >> vs;
      const int64_t poff = a.plane_off[k];
      for (int64_t i = threadIdx.x; i < int64_t(rows) * bytes; i += blockDim.x) {
        const int64_t y = i / bytes, x = i - y * bytes;
        const int64_t o = poff + (y0 + y) * row + xoff + x;
        dst[o] = src[o];
      }
    }
    __syncthreads();  // the next frame's copy reads this one
  }
  if (threadIdx.x == 0) a.sticky[s] = sticky;
}

}  // namespace

int64_t decode_lds_bytes(const DecodeArgs& a, bool global_states) {
  const int64_t sb = global_states ? 0 : ((a.swap ? a.state_bytes / 2 : a.state_bytes) + 15) & ~int64_t(15);
  return sb + 1024 + 64 + (a.context_model ? 5 : 3) * 256 * 2 +
         int64_t(a.rgb ? 2 * (3 + (a.transparency ? 1 : 0)) : 2) * a.row_cap * 2;
}

int launch_decode(const DecodeArgs& a, int nsegs, void* stream) {
  dim3 grid(a.nslices, nsegs), block(kDecThreads);
  const bool glob = a.tables != nullptr && !a.swap;
  const int64_t lds = decode_lds_bytes(a, glob);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a.ac == 0) {
    if (glob) hipLaunchKernelGGL((ffv1_decode_slices<true, true>), grid, block, lds, st, a);
    else hipLaunchKernelGGL((ffv1_decode_slices<true, false>), grid, block, lds, st, a);
  } else {
    if (glob) hipLaunchKernelGGL((ffv1_decode_slices<false, true>), grid, block, lds, st, a);
    else hipLaunchKernelGGL((ffv1_decode_slices<false, false>), grid, block, lds, st, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_conceal(const DecodeArgs& a, void* stream) {
  hipLaunchKernelGGL(ffv1_conceal, dim3(a.nslices), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace ffv1hip
