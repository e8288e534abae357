// ffv1_internal.h -- shapes shared between the HIP kernels and the host side
// of the MI355X FFV1 encoder.  Not part of the public C-ABI (include/ffv1hip.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace ffv1hip {

// One "header op" coded before the planes of a slice: the key bit
// (ffv1enc.c:1299-1307), the v0/v1 in-band header (ffv1enc.c:498-522) and
// the v3 slice header (ffv1enc.c:1031-1062).  Every op names one of kOpSets
// private 32-byte state vectors (all 128 at slice start) and which
// transition table it adapts with.
// kOpSymRct: an unsigned symbol whose value is the frame's slice RCT
// coefficient (value 0: slice_rct_by_coef, 1: slice_rct_ry_coef; v4 slice
// header, ffv1enc.c:1058-1059), chosen on the device per (frame, slice)
// kOpBitMode / kOpSymMode: v4's slice_coding_mode bit and symbol
// (ffv1enc.c:1054-1056): 0, or 1 when the slice is coded again as PCM; the
// RCT symbols are then left out (:1057-1060).
enum OpKind : int16_t { kOpSymU = 0, kOpSymS = 1, kOpBit = 2, kOpSymRct = 3, kOpBitMode = 4, kOpSymMode = 5 };
struct Op {
  int16_t kind;
  uint8_t set;
  uint8_t tab;   // 0: default table (ff_build_rac_states), 1: frame table
  int32_t value;
};
static_assert(sizeof(Op) == 8, "op layout");
constexpr int kMaxOps = 512;
constexpr int kCodeLanesChained = 64;  // chained coder: one stream per lane of a full wave
constexpr int kOpSets = 8;

// A run of consecutive frames of one batch whose context states chain
// (ffv1enc.c:1171-1172: only keyframes reset them).  Every segment but the
// first of a batch starts at a keyframe.
struct Segment {
  int first_frame;
  int nframes;
  int load_states;  // 1: continue from the persistent per-slice states
  int save_states;  // 1: store the final states for the next call
};

// Coded planes of a slice: Y, Cb, Cr, then A (YUVA: ffv1enc.c:1191-1198);
// YA8 codes Y and A of one packed plane (:1199-1201).
constexpr int kMaxPlanes = 4;

// Per-slice geometry (ffv1.c:117-145 + the chroma rounding of
// ffv1enc.c:1185-1196) and the slice's place in a frame's symbol stream.
struct SliceGeom {
  int px[kMaxPlanes], py[kMaxPlanes], pw[kMaxPlanes], ph[kMaxPlanes];  // plane rectangles
  int64_t sym_off;                      // first symbol of this slice in the frame stream
  int64_t plane_sym_off[kMaxPlanes];    // first symbol of each plane, relative to sym_off
  int64_t nsym;                         // all planes
  int64_t chunk_off[kMaxPlanes];        // first 64-sample walk chunk of each plane in the frame
};

// Per walk chunk (64 consecutive samples of a plane), written by ffv1_symbols:
// word 0 = the chunk's decisions | kChunkLong / kChunkMulti flags, words
// 1.. = the decision bits in coding order (bit d in word 1 + d / 32), then a
// zero word; the last two words = which of the 64 symbols have e = 10 or 11.
// A chunk takes chunk_words(wmax) words, wmax the most decisions one symbol
// can take (2 x coded bits + 1): 46 at 10 bits, 54 at 12, 70 at 16.
constexpr int kChunkWords = 70;  // the largest: header, 66 bit words + a zero word, the 64-bit multi-symbol mask
__host__ __device__ constexpr int chunk_words(int wmax) { return 2 * wmax + 4; }
static_assert(chunk_words(33) == kChunkWords, "16 bits: the largest chunk");
constexpr uint32_t kChunkLong = 0x80000000u;   // a symbol with e >= 12 (|diff| >= 4096)
constexpr uint32_t kChunkMulti = 0x40000000u;  // a symbol with e = 10 or 11 (slot 10 / 31 repeat)
constexpr uint32_t kChunkFlags = kChunkLong | kChunkMulti;

// Kernel 1: prediction + context + fold for every sample of a set of frames.
struct SymbolArgs {
  const uint8_t* frames;
  int64_t frame_bytes;
  int64_t plane_off[kMaxPlanes];   // coded plane p's first sample (YA8's A: Y's + 1)
  int plane_stride[kMaxPlanes];
  int pstep[kMaxPlanes];           // samples between a plane's pixels (YA8: 2)
  int pset[kMaxPlanes];            // plane context set of coded plane p (ffv1enc.c:1191-1201, (p+1)/2 for RGB)
  const int* frame_of_slot;   // [slot] batch frame index coded in this launch, -1 = none
  int nslots;
  const SliceGeom* geom;
  int nslices, nplanes;
  int sample_bytes, packed_at_lsb, msb_shift, coded_bits;
  int rgb, rct_offset;        // RGB: the samples are G', B' + off, R' + off, rows interleaved
  int contexts, model1;
  const int16_t* qt;          // [5][256]
  uint32_t* sym;              // [slot][frame_samples]: (row << 16) | (uint16)diff
  int64_t frame_samples;
  int* dcount;                // optional [slot][slice][3]: range-coder decisions per plane
  uint2* rec;                 // optional, instead of sym: [slot][frame_samples] walk records
  uint32_t* cbits;            // with rec: [slot][frame_chunks][cwords]
  int64_t frame_chunks;
  int p_lo, p_hi;             // planes of this launch (p_hi 0: all); with rec, outputs by batch frame
  const int2* rct;            // v4: [batch frame][slice] {by, ry} RCT coefficients, else null (1, 1)
  int max_blocks;             // grid cap (0: one block per item); the blocks stride over the items
  int nz;                     // set by launch_symbols: plane parts per (slice, slot)
  int rowb = 32;              // with rec: the walk's bytes per row (a record's row address = row x rowb)
  int cwords = kChunkWords;   // with rec: words per chunk (chunk_words)
};

// v4's choose_rct_params (ffv1enc.c:1064-1144) for every (frame, slice) of
// a batch: the 15 candidate sums of one slice, then its coefficients.
struct RctArgs {
  const uint8_t* frames;
  int64_t frame_bytes;
  int64_t plane_off[3];
  int plane_stride[3];
  int sample_bytes;           // 4: one B, G, R, X word per pixel; 2: three u16 planes read as b, g, r
  const SliceGeom* geom;
  int nslices, nframes;
  int2* rct;                  // [frame][slice] {by, ry}
};

// Walk record of one sample (frame-parallel mode), written by ffv1_symbols.
// A plane is walked in chunks of 64 consecutive samples (one per lane).
// 8 bytes, uint2 {x, w}:
//   x: row * 32 inside the plane group's table (bits 0..15) | (int16)diff << 16
//   w: D | (D + 2e) << 16, D = the symbol's first decision counted from the
//      start of its chunk; bit 31: same row as the previous sample of the
//      chunk; bit 30: same row as the sample two back in the chunk; bits
//      12..14 / 28..29: the composed rows of slots 10 / 31 at e = 10, 11
// The walk expands a chunk's records in LDS to uint4 {x, y, z, w}: in a
// chunk of symbols with e <= 9, y and z are slot masks (one bit per slot:
// y the decision bit, z "no decision"); in a chunk with e = 10, 11 symbols,
// two bits per slot (y slots 0..15, z 16..31): 0/1 the slot's decision bit,
// 2 no decision, 3 several decisions (slot 10 at e >= 10, slot 31 at e >=
// 11); the chunks with a larger exponent take walk_long.
constexpr uint32_t kRecSame = 0x80000000u;
constexpr uint32_t kRecSame2 = 0x40000000u;

// Decision stream of one batch (frame-parallel mode).  Every (frame, slice)
// stream's binary decisions, in coding order, start at decision index
// dbase[frame][slice] (a multiple of kStreamAlign): the luma chain's dcount[0]
// decisions, then, from chroma_start(dcount[0]), the chroma chain's (Cb then
// Cr).  Each chain is followed by kChainPad unused decisions: the states
// walk writes a chunk's recorded bytes in whole 16-byte blocks, and the
// blocks past a chain's last decision land there.  Decision d has the
// adaptive state it is coded with in pre[d] and its value in bit d of
// bits[] (bit d & 31 of word d >> 5).
// Chains start at multiples of kStreamAlign = 512 decisions, so that every
// coder segment's decision bits start on a 64-byte boundary (ffv1_dseg reads
// them 64 bytes per lane at a time).
constexpr int kChainPad = 2048;
constexpr int kStreamAlign = 512;
// a chain of n decisions and its pad, rounded to the alignment
__host__ __device__ inline int64_t chain_extent(int64_t n) {
  return (n + kStreamAlign - 1) / kStreamAlign * kStreamAlign + kChainPad;
}
__host__ __device__ inline int64_t chroma_start(int64_t dc0) { return chain_extent(dc0); }
// decisions a stream takes beyond its own (alignment and the two pads)
constexpr int64_t kStreamSlack = 2 * kChainPad + 2 * kStreamAlign;
struct DecisionStream {
  const int* dcount;          // [frame][slice][3] decisions per plane
  const int64_t* dbase;       // [frame][slice]
  uint8_t* pre;
  uint32_t* bits;
  // A batch launched before its decision count is known on the host (the
  // layout's total not read back): the kernels that touch pre / bits skip
  // the batch when the total exceeds the set's capacity, ffv1_dfix flags it
  // (status[3]) and the host encodes it again with a larger set.  total null:
  // the set was sized from the read-back total.
  const int64_t* total;
  int64_t cap;
};
__device__ __forceinline__ bool ds_over(const DecisionStream& ds) { return ds.total && *ds.total > ds.cap; }

// Debug build (build.py --check: -DFFV1HIP_BOUNDS, lib/libffv1hip_check.so):
// the walk's, dseg's, dfix's and sink's writes are checked against the
// extents they own (a walk chain: its own chain and pad in pre, never a
// neighbour's; a coder stream: its slice slot); a write outside is dropped
// and the first offending site is recorded in *err, which the host turns
// into an error at the batch's settle (ffv1hip_debug_checks reports the
// build).  The release build compiles every check away.
#ifdef FFV1HIP_BOUNDS
constexpr bool kBoundsCheck = true;
#else
constexpr bool kBoundsCheck = false;
#endif
enum BoundsSite : uint32_t {
  kBndWalkStage = 1,   // ffv1_walk: a chunk's stage copied out to pre
  kBndWalkLong = 2,    // ffv1_walk: a walk_long chunk's states
  kBndWalkStates = 3,  // ffv1_walk: the carry it leaves in persist_out
  kBndDsegSlot = 4,    // ffv1_dseg: a stream's digits (its slice slot)
  kBndDsegRead = 5,    // ffv1_dseg: a segment's states and bits (its chain)
  kBndDfixSlot = 6,    // ffv1_dfix: a stream's joined digits
  kBndSinkSlot = 7,    // ffv1_sink: a stream's bytes
};
struct Bounds {
  uint32_t* err;           // first failing site (0: none); null in the release build
  int64_t pre_bytes;       // DecisionStream.pre
  int64_t out_bytes;       // slice_out
  int64_t persist_bytes;   // persist_out
};

// The decision-stream range coder runs in three passes (ffv1_kernels.hip):
// ffv1_range walks `range` alone per (frame, slice) stream and leaves a
// checkpoint every kSeg decisions, ffv1_dseg codes every segment from its
// checkpoint in parallel, ffv1_dfix joins the segments' low values.
constexpr int kSeg = 4096;  // decisions per segment (a multiple of 32 and of the part alignment 64)
// Per stream (layout): its segments, luma first (s_luma of them), then the
// chroma chain's; their first index over the batch; the first of the
// 64-segment groups ffv1_dseg takes one wave each.
struct StreamSegs {
  int seg_base, s_luma, s_all, wave_base;
};
// Per (key, slice): the range coder after the header decisions (key bit,
// v0/v1 header, v3 slice header), which do not depend on the pixels: low,
// range, how many renormalisation shifts they took, and where the values of
// low at those shifts (the stream's first digits) are in hdr_digits.
struct HdrState {
  int low, range, ndig, off;
};

// Kernel 2: the SIMT range coder.
//  chained (launch_code): one lane per (segment, slice) chain, one frame of
//    every segment per launch, context states carried in `tables`;
//  decision stream (launch_range / launch_dseg / launch_dfix): every
//    (frame, slice) stream of the whole batch, pure range arithmetic over
//    the states ffv1_walk recorded.
struct CodeArgs {
  const uint32_t* sym;        // from kernel 1 (slot = segment)
  int64_t frame_samples;
  const SliceGeom* geom;
  int nslices, nsegs;
  int j;                      // frame index inside each segment
  const Segment* segs;
  const uint8_t* keyflags;    // [batch frame]
  const Op* ops;              // [key][slice][kMaxOps]
  const int* nops;            // [key][slice]
  int max_ops;
  const uint8_t* tabs;        // [default to0|to1][frame to0|to1]
  int64_t state_bytes;        // pcount * contexts * 32
  uint8_t* tables;            // [chain][state_bytes] working context states (grid-padded)
  const uint8_t* persist_in;  // [slice][state_bytes]: the carry the batch starts from
  uint8_t* persist_out;       // [slice][state_bytes]: the carry it leaves (the other buffer)
  uint8_t* slice_out;         // [batch frame][slice][slice_stride]
  int64_t slice_cap;          // byte budget of a slice
  int64_t slice_stride;       // bytes per slice slot (decision-stream mode: 4 x (slice_cap + kSeg + 64),
                              // the values of low at the shifts, u32, then ffv1_sink's bytes over them)
  int64_t* slice_bytes;       // [batch frame][slice]
  int* status;                // [0] slices over the byte budget, [1] most bytes a slice needed
  int version;                // bitstream version (Golomb: v3 adds a 129/0 decision)
  int coded_bits;             // "bits" of encode_line (8 for <=8-bit)
  int rgb;                    // RGB: a slice's planes are row-interleaved (chained coders)
  int nplanes;                // coded planes (1 gray, 2 YA8, 3, 4 with alpha)
  int pset[kMaxPlanes];       // plane context set of each coded plane
  int pcount;                 // plane contexts (plane_count: 2, 3 with alpha)
  const int2* rct;            // v4: [batch frame][slice] RCT coefficients for the slice header ops
  // v4 range coder (chained): the reference's per-line buffer check
  // (ffv1enc.c:282-286) against its slice buffers (:1281-1282, 1317-1322) and
  // the PCM re-code of a slice that fails it (:1207-1217, 294-304), which
  // reads the samples from the frames
  int v4pcm;
  int64_t v4_cap0, v4_cap;    // the reference's buffer bytes: slice 0 (the packet), the others
  const uint8_t* frames;
  int64_t frame_bytes;
  int64_t plane_off[kMaxPlanes];
  int plane_stride[kMaxPlanes];
  int sample_bytes, packed_at_lsb, msb_shift, pcm_bits;
  int nframes;                // decision-stream mode: frames of the batch
  DecisionStream ds;
  const uint8_t* init;        // chained range coder: 2-pass initial states [contexts][32], or null
  // decision-stream mode (three passes)
  const HdrState* hdr;        // [key][slice]
  const uint32_t* hdr_digits; // values of low at the header's shifts
  const StreamSegs* segs_info;  // [stream]
  const int* seg_totals;      // device: [0] segments, [1] 64-segment groups of the batch
  const int* wmap;            // [group] its stream
  uint2* ck;                  // [segment] {range before it, shifts before it}
  uint2* segrec;              // [segment] {local low at its end, its shifts}
  int64_t digit_cap;          // values of low a slice slot holds (slice_stride / 4)
  int dseg_blocks;            // ffv1_dseg grid
  int range_prio, dseg_prio;  // wave priorities (s_setprio) of ffv1_range / ffv1_dseg beside the walk (2)
  Bounds bnd;                 // debug build: the extents of the writes
  // the range pass split at the luma / chroma boundary (launch_range_dseg)
  int2* rstate;               // [stream] {range, shifts} after the luma chain
  int range_pass;             // 0 whole streams, 1 the luma chains, 2 the chroma chains
  int dseg_part;              // ffv1_dseg: -1 every segment, 0 the luma chains', 1 the chroma chains'
  int range_blocks;           // set by launch_range_dseg
  // pass 1 (ffv1_code): put_symbol_inline's counts (ffv1enc.c:190-199),
  // rc_stat[256][2] by state, rc_stat2[contexts][32][2] by (context, slot)
  unsigned long long* rc_stat;
  unsigned long long* rc_stat2;
  // ffv1_code: chains per wave (lanes 0 .. cpw-1; launch_code spreads a batch
  // of few chains over more waves), and the first of the 64 dummy tables the
  // other lanes write their rows to
  int cpw = 64;
  int64_t table_dummy = 0;
};

// Pass-1 statistics (ffv1enc.c:190-199): rc_stat[state][bit] from the
// decision stream, rc_stat2[context][slot][bit] from the walk records.
struct StatsArgs {
  const uint2* rec;           // [batch frame][frame_samples]
  int64_t frame_samples;
  const SliceGeom* geom;
  int nslices, nframes;
  DecisionStream ds;
  unsigned long long* rc_stat;   // [256][2]
  unsigned long long* rc_stat2;  // [contexts][32][2]
  int dense;                     // the records address dense rows (dense_ctx)
  int rowb = 32;                 // the records' row address = row x rowb
};
int launch_stats(const StatsArgs& a, bool states, void* stream);

// Kernel 2a: the context-state walk.  The adaptive states a slice's range
// coder sees depend only on the decisions of the earlier symbols of its GOP,
// not on the coder's arithmetic.  One wave per (segment, slice, plane group)
// replays just the state transitions (table in LDS) and records, for every
// decision, the state it is coded with and its bit; the coding of all
// (frame, slice) streams then runs in parallel (launch_dcode).
struct WalkArgs {
  const uint2* rec;           // [batch frame][frame_samples] walk records
  const uint32_t* cbits;      // [batch frame][frame_chunks][cwords]
  int64_t frame_chunks;
  int64_t frame_samples;
  const SliceGeom* geom;
  int nslices;
  const Segment* segs;
  const uint8_t* ftab;        // frame transition table [bit][state]
  int64_t state_bytes;
  const uint8_t* persist_in;  // [slice][state_bytes]
  uint8_t* persist_out;       // [slice][state_bytes]
  DecisionStream ds;
  uint8_t* scratch;           // >= 2 KiB: where idle chains write their stage
  uint64_t* dbg;              // optional [block][4] cycle counters (FFV1HIP_WALKDBG)
  uint64_t* trace;            // optional [item][kTraceWords]: start / end s_memrealtime, HW_ID, XCC_ID, step-loop
                              // cycles, steps, the wave's cycles
  int force_multi;            // measurement hook: every chunk on the checked (multi) step
  const uint8_t* init;        // 2-pass initial states [contexts][32] at keyframes, or null (all 128)
  int nitems, item0;          // set by launch_walk: all items of the batch, the launch's first
  int nsegs;                  // segments of the batch
  int per_short;              // segments one wave of the shorter plane group walks, one after the other
  int short_multi;            // shorter-group waves (per slice pair) that take per_short segments; the rest take one
  int block_waves;            // 1, or 4 / 5 waves per block for a one-round batch (walk_block_waves)
  int prio;                   // wave priority (s_setprio)
  int rows;                   // context rows of a plane group's table in LDS (kDenseRows when dense)
  int dense;                  // records address dense rows (dense_row), the state tables keep contexts
  Bounds bnd;                 // debug build: the extents of the writes
  int rowb = 32;              // bytes per row in LDS: 32, or kCompactRowBytes at 8 bits (context model 0)
  int cwords = kChunkWords;   // words per chunk (chunk_words)
};

constexpr int kTraceWords = 8;

// Above 8 bits the quantisers of context model 0 have 9 levels (ffv1enc.c:
// 846-879, quant9_10bit), so only 365 of the 666 contexts q0 + 11 q1 + 121 q2
// (|q| <= 4, folded) occur.  The frame-parallel path then numbers rows
// densely, row = q0 + 9 q1 + 81 q2 (folded the same way: the sign of either
// sum is the sign of its highest nonzero digit), so that a plane group's
// table in the walk's LDS is 365 x 32 bytes instead of 666 x 32 and five
// walk waves fit on a CU instead of three.  Persisted / initial states keep
// the context numbering.
constexpr int kDenseRows = 365;

// At 8 bits a residual is folded to [-128, 127], so e <= 7 and
// put_symbol_inline (ffv1enc.c:185-231) uses only slots 0-8 (zero flag and
// exponent), 11-18 (sign) and 22-28 (mantissa): 24 of a row's 32.  The walk's
// LDS rows then hold those 24 (walk_slot_pos), a plane group's table is
// 666 x 24 bytes instead of 666 x 32, and four walk waves fit on a CU instead
// of three.  The records carry the row's byte offset (row x row bytes).
constexpr int kCompactRowBytes = 24;
__host__ __device__ constexpr int walk_slot_pos(int k) {  // compact position of slot k, -1: unused at 8 bits
  return k <= 8 ? k : (k >= 11 && k <= 18) ? k - 2 : (k >= 22 && k <= 28) ? k - 5 : -1;
}
__host__ __device__ inline int dense_ctx(int row) {  // row -> its context
  const int q0 = (row + 4) % 9 - 4;
  const int r1 = (row - q0) / 9;
  const int q1 = (r1 + 4) % 9 - 4;
  const int q2 = (r1 - q1) / 9;
  return q0 + 11 * q1 + 121 * q2;
}
__host__ __device__ inline int dense_row(int ctx) {  // context -> its row, -1 when it cannot occur
  const int q0 = (ctx + 5) % 11 - 5;
  const int r1 = (ctx - q0) / 11;
  const int q1 = (r1 + 5) % 11 - 5;
  const int q2 = (r1 - q1) / 11;
  if (q0 < -4 || q0 > 4 || q1 < -4 || q1 > 4 || q2 < -4 || q2 > 4) return -1;
  return q0 + 9 * q1 + 81 * q2;
}

// Kernel 2b: the decision bits, from the chunks' packed words to their place
// in the decision stream (one block per (frame, slice) stream).
struct BitsArgs {
  const uint32_t* cbits;      // [batch frame][frame_chunks][cwords]
  int64_t frame_chunks;
  const SliceGeom* geom;
  int nslices, nframes;
  DecisionStream ds;
  int max_blocks;             // grid cap (0: one block per stream); the blocks stride over the streams
  int cwords = kChunkWords;   // words per chunk (chunk_words)
};

struct AssembleArgs {
  const int* skip;             // frame-parallel mode: status[3], set when the batch was skipped (ds_over); or null
  const uint8_t* slice_out;
  int64_t slice_cap;
  int64_t slice_stride;
  const int64_t* slice_bytes;  // [frame][slice]
  uint8_t* packets;            // [frame] regions of packet_stride bytes
  int64_t packet_stride;
  int64_t* packet_size;        // [frame]
  int nslices;
  int version;
  int ec;
};

// Decoder (ffv1_decode.hip): one workgroup per (segment, slice) chain of a
// batch of packets, range coder, context model 0, version 3.
struct DecodeArgs {
  const uint8_t* pkts;         // packets back to back, 8-byte aligned, >= 64 bytes of pad
  const int64_t* slice_start;  // [frame][slice] byte offset of the slice in pkts
  const int64_t* slice_end;    // [frame][slice] end of the slice's bytes (trailer included)
  const uint8_t* keyflags;     // [frame]
  const Segment* segs;
  const SliceGeom* geom;
  int nslices, nplanes;
  const int16_t* qt;           // [5][256]
  const uint8_t* ftab;         // frame transition table: to0[256] | to1[256]
  const uint8_t* dtab;         // default table (key bit, v0/v1 header): to0 | to1
  int64_t state_bytes;         // range coder: 2 * contexts * 32; Golomb: 2 * contexts * 8
  const uint8_t* persist_in;   // [slice][state_bytes]: the chain carried across calls
  uint8_t* persist_out;        // (two buffers: a launch never reads what it writes)
  uint8_t* tables;             // global states [seg][slice][state_bytes] when they exceed the LDS
  uint8_t* out;                // [frame] regions of frame_bytes, planes tightly packed
  int64_t frame_bytes;
  int64_t plane_off[kMaxPlanes];  // output planes: Y, Cb, Cr, A (YUVA); one packed plane for bgr0 / RGB32 / YA8
  int plane_w[kMaxPlanes];
  int sample_bytes, packed_at_lsb, msb_shift, coded_bits;
  int width, height, num_h, num_v, context_model;
  int version, ac, ec, rgb, rct_offset, contexts;
  int chroma_planes, chroma_h_shift, chroma_v_shift, bits_per_raw_sample;
  int row_cap;                 // widest slice plane (samples)
  int* status;                 // [0] slices whose key bit or v0/v1 header disagrees
  uint8_t* damage;             // [frame][slice]: 2 slice header failed (not decoded), 4 end mismatch
  // concealment pass (ffv1_conceal)
  const uint8_t* last;         // the picture before frame 0 (previous call), or null
  uint8_t* sticky;             // [slice] slice_damaged carried across calls
  int nframes;
  const uint8_t* init;         // range coder: initial states [contexts][32] from the extradata, or null
  int swap;                    // one plane group's states in the LDS, the other in `tables` (range, YCbCr)
  int transparency, ya8;       // alpha: a third plane context (YUVA's A, RGB32's A rows); YA8: Y, A of one plane
  int pcount;                  // plane contexts: 2, 3 with alpha
  const int32_t* stab;         // [256] frame table pairs to0 | to1 << 8, then [5][256] quant tables (scalar loads)
};
int launch_decode(const DecodeArgs& a, int nsegs, void* stream);

// 2-pass host arithmetic (ffv1_twopass.cpp): pass-2 states from stats_in
// (stt: in, the custom table; out, sorted when custom) and the pass-1 text.
int pass2_states(const char* stats, bool custom, uint8_t stt[256], const uint8_t default_one[256],
                 std::vector<uint8_t> init[2], std::string* err);
std::string pass1_text(const uint64_t* rc_stat, const uint64_t* rc_stat2, int contexts, int model, int gob_count);
int launch_conceal(const DecodeArgs& a, void* stream);
int64_t decode_lds_bytes(const DecodeArgs& a, bool global_states);

int launch_symbols(const SymbolArgs& a, void* stream);
int launch_rct_params(const RctArgs& a, void* stream);
int launch_code(const CodeArgs& a, void* stream);
int launch_layout(const int* dcount, int nstreams, int64_t* dbase, int64_t* total, StreamSegs* segs,
                  int* seg_totals, int* wmap, int64_t* total_host, void* stream);
int launch_zero_bits(uint32_t* bits, const int64_t* total, int64_t cap, void* stream);
// items [first, first + count) of the batch's walk (count < 0: to the end)
int launch_walk(const WalkArgs& a, int nsegs, void* stream, int first = 0, int count = -1);
// Items (waves) of a batch's walk: the longer plane group's chains first, one
// segment per wave, then the shorter group's, per_short segments per wave one
// after the other, so that both kinds of wave walk about as many symbols
// (4:2:0 luma vs Cb + Cr, 4:4:4 Cb + Cr vs luma: 2).
int walk_items(int nsegs, int nslices, int per_short, int short_multi);
int walk_split_short(int nsegs, int nslices, int per_short, int simds, int resident);
int walk_block_waves(int nsegs, int nslices, int per_short, int short_multi, int rows, int rowb, int cus,
                     int lds_block);
int walk_per_short(const SliceGeom& g);
int walk_resident(const WalkArgs& a);  // (uses a.rows)
int launch_range(const CodeArgs& a, void* stream);
int launch_dseg(const CodeArgs& a, void* stream);
int launch_range_dseg(const CodeArgs& a, void* stream);
int launch_dfix(const CodeArgs& a, void* stream);
int launch_sink(const CodeArgs& a, void* stream);
int launch_bits(const BitsArgs& a, void* stream);
int64_t walk_lds_bytes(int rows, int rowb);  // one walk wave's LDS for tables of `rows` context rows of `rowb` bytes
constexpr int64_t kWalkLdsMax = 64 * 1024;  // states walk: one plane group's table + T9 + staging in LDS
int launch_code_golomb(const CodeArgs& a, void* stream);
int launch_assemble(const AssembleArgs& a, int nframes, void* stream);
int launch_compact_packets(const uint8_t* packets, int64_t stride, const int64_t* sizes, int n, uint8_t* out,
                           const int* skip, void* stream);
int launch_sizes_out(const int64_t* sizes, int n, int64_t* host_mapped, void* stream);
// ffv1_unpack10: frames f0 .. f0+n-1 of a batch's packed 10-bit samples
// (three to a word) into their 16-bit frame slots, n <= kUnpackFrames
constexpr int kUnpackFrames = 1024;
struct UnpackArgs {
  const uint8_t* packed;
  uint8_t* frames;
  int64_t packed_frame_bytes, frame_bytes;
  int64_t poff[kMaxPlanes], off[kMaxPlanes];  // a plane in a packed / 16-bit frame slot
  int prow[kMaxPlanes];                       // words per packed row
  int width[kMaxPlanes], rows[kMaxPlanes], pst[kMaxPlanes];
  int np, f0;
  uint32_t raw[kUnpackFrames / 32];  // frames staged as is
};
int launch_unpack10(const UnpackArgs& a, int nframes, void* stream);
int launch_ints_out(const int* src, int n, int* host_mapped, void* stream);

}  // namespace ffv1hip
