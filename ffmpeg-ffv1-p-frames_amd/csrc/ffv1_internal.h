// ffv1_internal.h -- shapes shared between the HIP kernels and the host side
// of the MI355X FFV1 encoder.  Not part of the public C-ABI (include/ffv1hip.h).
#pragma once

#include <stdint.h>

namespace ffv1hip {

// One "header op" coded before the planes of a slice: the key bit
// (ffv1enc.c:1299-1307), the v0/v1 in-band header (ffv1enc.c:498-522) and
// the v3 slice header (ffv1enc.c:1031-1062).  Every op names one of kOpSets
// private 32-byte state vectors (all 128 at slice start) and which
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

// Per-slice geometry (ffv1.c:117-145 + the chroma rounding of
// ffv1enc.c:1185-1196) and the slice's place in a frame's symbol stream.
struct SliceGeom {
  int px[3], py[3], pw[3], ph[3];  // plane rectangles
  int64_t sym_off;                 // first symbol of this slice in the frame stream
  int64_t plane_sym_off[3];        // first symbol of each plane, relative to sym_off
  int64_t nsym;                    // all planes
};

// Kernel 1: prediction + context + fold for every sample of a set of frames.
struct SymbolArgs {
  const uint8_t* frames;
  int64_t frame_bytes;
  int64_t plane_off[3];
  int plane_stride[3];
  const int* frame_of_slot;   // [slot] batch frame index coded in this launch, -1 = none
  int nslots;
  const SliceGeom* geom;
  int nslices, nplanes;
  int sample_bytes, packed_at_lsb, msb_shift, coded_bits;
  int contexts, model1;
  const int16_t* qt;          // [5][256]
  uint32_t* sym;              // [slot][frame_samples]: (row << 16) | (uint16)diff
  int64_t frame_samples;
};

// Kernel 2: the SIMT range coder, one lane per (segment, slice) chain, one
// frame of every segment per launch.
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
  int64_t state_bytes;        // 2 * contexts * 32
  uint8_t* tables;            // [chain][state_bytes] working context states (grid-padded)
  uint8_t* persist;           // [slice][state_bytes]
  uint8_t* slice_out;         // [batch frame][slice][slice_cap]
  int64_t slice_cap;
  int64_t* slice_bytes;       // [batch frame][slice]
  int* status;                // [0] overflow count
  int version;                // bitstream version (Golomb: v3 adds a 129/0 decision)
  int coded_bits;             // "bits" of encode_line (8 for <=8-bit)
  // frame-parallel mode (launch_code_frames): one lane per (frame, slice),
  // starting from the per-frame state snapshots ffv1_states wrote
  uint8_t* snap;              // [frame][slice][state_bytes] + 64 spare tables for idle lanes
  int nframes;
  int lanes;                  // streams per wave (1..64); the other lanes idle
  int64_t spare;              // index of the first spare table
};

// Kernel 2a: the context-state walk.  The adaptive states a slice's range
// coder sees depend only on the decisions of the earlier frames of its GOP,
// not on the coder's arithmetic, so one wave per (segment, slice) replays
// just the state transitions (table in LDS) and writes the states at the
// start of every frame; the coding of all frames then runs in parallel.
struct StateArgs {
  const uint32_t* sym;        // [batch frame][frame_samples]
  int64_t frame_samples;
  const SliceGeom* geom;
  int nslices;
  const Segment* segs;
  const uint8_t* ftab;        // frame transition table [bit][state]
  int64_t state_bytes;
  uint8_t* persist;           // [slice][state_bytes]
  uint8_t* snap;              // [batch frame][slice][state_bytes]
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

int launch_symbols(const SymbolArgs& a, void* stream);
int launch_code(const CodeArgs& a, void* stream);
int launch_code_frames(const CodeArgs& a, void* stream);
int launch_states(const StateArgs& a, int nsegs, void* stream);
constexpr int64_t kStateLdsMax = 64 * 1024;  // states walk: table + transition table in LDS
int launch_code_golomb(const CodeArgs& a, void* stream);
int launch_assemble(const AssembleArgs& a, int nframes, void* stream);

}  // namespace ffv1hip
