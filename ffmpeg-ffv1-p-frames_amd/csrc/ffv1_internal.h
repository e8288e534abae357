// ffv1_internal.h -- shapes shared between the HIP kernels and the host side
// of the MI355X FFV1 encoder.  Not part of the public C-ABI (include/ffv1hip.h).
#pragma once

#include <stdint.h>

namespace ffv1hip {

// One "header op" executed by the slice coder before the planes: the key
// bit (ffv1enc.c:1299-1307), the v0/v1 in-band header (ffv1enc.c:498-522)
// and the v3 slice header (ffv1enc.c:1031-1062).  Every op names one of
// kOpSets private 32-byte state vectors (all 128 at slice start) and which
// transition table it adapts with.
enum OpKind : int16_t { kOpSymU = 0, kOpSymS = 1, kOpBit = 2 };
struct Op {
  int16_t kind;
  uint8_t set;
  uint8_t tab;   // 0: default table (ff_build_rac_states), 1: frame table
  int32_t value;
};
static_assert(sizeof(Op) == 8, "op layout");
constexpr int kMaxOps = 512;
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

struct EncodeArgs {
  const uint8_t* frames;     // batch base in HBM
  int64_t frame_bytes;       // distance between frames
  int64_t plane_off[3];      // byte offset of Y, Cb, Cr inside a frame
  int plane_stride[3];       // row stride in bytes
  int width, height;
  int nh, nv, nslices;
  int chroma_planes, hs, vs;
  int sample_bytes, packed_at_lsb, msb_shift, coded_bits;
  int contexts;              // per plane context (666 / 7563)
  int model1;                // context model 1 (5 taps)
  int row_len;               // LDS row buffer length in samples (>= max plane width + 8)
  const int16_t* qt;         // [5][256]
  const uint8_t* tabs;       // [2 tables][to0[256], to1[256]]: default, frame
  const Segment* segs;
  int nsegs;
  const uint8_t* keyflags;   // [frame]
  const Op* ops;             // [key 0/1][slice][kMaxOps]
  const int* nops;           // [key 0/1][slice]
  uint8_t* slice_out;        // [frame][slice] regions of slice_cap bytes
  int64_t slice_cap;
  int64_t* slice_bytes;      // [frame][slice]
  uint8_t* persist;          // [slice][2][contexts][32]
  uint8_t* gstates;          // context model 1 working states [seg][slice][2][contexts][32]
  int* status;               // [0]: overflow count
};

struct AssembleArgs {
  const uint8_t* slice_out;
  int64_t slice_cap;
  const int64_t* slice_bytes;  // [frame][slice]
  uint8_t* packets;            // [frame] regions of packet_stride bytes
  int64_t packet_stride;
  int64_t* packet_size;        // [frame]
  int nslices;
  int version;
  int ec;
};

size_t encode_lds_bytes(const EncodeArgs& a, bool lds_states);
int launch_encode(const EncodeArgs& a, bool lds_states, void* stream);
int launch_assemble(const AssembleArgs& a, int nframes, void* stream);

}  // namespace ffv1hip
