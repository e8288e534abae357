/*
 * ffv1hip.h -- C-ABI of the MI355X FFV1 encoder (the drop-in boundary).
 *
 * The reference exposes this path as an AVCodec (libavcodec/ffv1enc.c:1415-
 * 1444, ff_ffv1_encoder) whose .init/.encode2/.close callbacks are invoked by
 * avcodec_open2 (libavcodec/utils.c:1571) and avcodec_encode_video2
 * (utils.c:1962).  This header is the plain-C surface a thin AVCodec shim
 *  binds instead; it carries no FFmpeg or torch types:
 * plain structs, pointers and sizes.  All functions return 0 (or a size) on
 * success and a negative errno-style code on failure:
 *   -EINVAL (-22) bad argument      -ENOSYS (-38) unsupported parameters
 *   -ENOMEM (-12) allocation        -ENOSPC (-28) slice byte budget exceeded
 *   -EIO     (-5) HIP runtime error (message via ffv1hip_last_error)
 *   -EFAULT (-14) debug build only: a kernel's write fell outside its buffer
 * plus FFV1HIP_AVERROR_INVALIDDATA for the reference's InvalidData cases.
 */
#ifndef FFV1HIP_H
#define FFV1HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FFV1HIP_ABI_VERSION 6
#define FFV1HIP_AVERROR_INVALIDDATA (-1094995529)

/* AVCodecContext fields + codec private options that encode_init reads
 * (ffv1enc.c:669-1029, options ffv1enc.c:1383-1399, defaults :1408-1413). */
typedef struct ffv1hip_options {
    int width, height;
    const char *pix_fmt;      /* "yuv420p", "yuv420p10", "yuv444p16", ...,
                                 "bgr0" / "gbrp9".."gbrp14" (RGB); with
                                 alpha "yuva420p".."yuva444p16", "ya8",
                                 "bgra" / "rgb32" (ffv1enc.c:725-786)      */
    int slices;               /* avctx->slices (0 = auto)                   */
    int level;                /* avctx->level (-1 = unset)                  */
    int coder;                /* -1 default, 0 rice, 1/2 range_tab, -2 range_def */
    int context;              /* context model 0/1                          */
    int gop_size;             /* avctx->gop_size (default 12)               */
    int bits_per_raw_sample;  /* 0 = from pix_fmt                           */
    int slicecrc;             /* -1 default (on for v3)                     */
    int allow_large_grid;     /* 1: accept up to 256 slices (16x16), which the
                                 reference decoder reads but its encoder
                                 refuses (ffv1enc.c:988-1000); used for 8K  */
    int pass;                 /* 1 / 2: AV_CODEC_FLAG_PASS1 / PASS2 (version
                                 >= 2, ffv1enc.c:680-682); see ffv1hip_set_pass */
    int experimental;         /* -strict experimental: admits version 4
                                 (level 4, ffv1enc.c:703-706) for the RGB
                                 formats and >8-bit 4:4:4 YCbCr, the formats
                                 whose choose_rct_params reads stay inside
                                 the frame (:1064-1144, 1163-1164)          */
} ffv1hip_options;

/* Effective bitstream parameters (what encode_init derives). */
typedef struct ffv1hip_params {
    int width, height;
    int chroma_planes;        /* 1 YUV, 0 gray                              */
    int chroma_h_shift, chroma_v_shift;
    int bits_per_raw_sample;
    int packed_at_lsb;        /* u16 samples LSB-aligned (yuv*p9/p10, gbrp) */
    int sample_bytes;         /* 1 or 2 bytes per stored sample; 4: bgr0,
                                 one packed B,G,R,X plane                   */
    int version;              /* 0, 1, 3, or 2 / 4 (experimental: the slice
                                 layout in the keyframe header / per-slice
                                 RCT coefficients in the slice header)      */
    int ac;                   /* 0 Golomb-Rice, 1 range default, 2 range custom */
    int ec;                   /* slice CRC-32 trailers                      */
    int context_model;        /* 0: 666 contexts, 1: 7563                   */
    int num_h_slices, num_v_slices;
    int gop_size;
    int sar_num, sar_den;
    int colorspace;           /* 0 YCbCr; 1 RGB through the reversible colour
                                 transform (ffv1enc.c:413-473): bgr0 or
                                 gbrp planes in AVFrame data[] order        */
    int transparency;         /* alpha (ffv1enc.c:774, 782): YUVA's plane 3
                                 (plane context 2), YA8's packed A bytes
                                 (plane context 1), RGB32's A byte; coded by
                                 the chained coders                         */
} ffv1hip_params;

/* Host planes per frame in the plane / stride arrays of ffv1hip_encode,
 * ffv1hip_encode2 and ffv1hip_encode_device: 4 (Y, Cb, Cr, A) for the YUVA
 * formats, else 3 (entries past the format's planes are not read: gray,
 * YA8, bgr0 and RGB32 use plane 0 only). */
#define FFV1HIP_PLANES_YUVA 4
#define FFV1HIP_PLANES 3

typedef struct ffv1hip_ctx ffv1hip_ctx;

/* encode_init's parameter contract (ffv1enc.c:669-1029). */
int ffv1hip_configure(ffv1hip_params *out, const ffv1hip_options *opt);

/* AVCodec.init (ffv1enc.c:669 encode_init): allocates device state for up
 * to max_batch_frames frames per call on HIP device `device`. */
ffv1hip_ctx *ffv1hip_create(const ffv1hip_params *params, int device,
                            int max_batch_frames, int *err);

/* 2-pass encoding (ffv1enc.c:898-986, 1236-1277), chosen after
 * ffv1hip_create and before the first frame, for parameters configured with
 * options.pass.  pass 1: the encoder counts every plane decision by state
 * value and by (context, slot); ffv1hip_stats_out then returns the text
 * encode_frame writes into avctx->stats_out at the end of the stream
 * (needs the frame-parallel range coder, or Golomb-Rice whose counts are
 * zero).  pass 2: stats_in is that text; the custom transition table is
 * re-sorted and every context's initial state derived from it, keyframes
 * start from those states and the extradata carries them.  Returns 0 or a
 * negative error (AVERROR_INVALIDDATA for malformed statistics). */
int ffv1hip_set_pass(ffv1hip_ctx *ctx, int pass, const char *stats_in);
/* Pass 1: the statistics so far as text (NUL-terminated in buf); returns
 * its length, or the length needed when buf is NULL. */
int64_t ffv1hip_stats_out(ffv1hip_ctx *ctx, char *buf, int64_t cap);

/* AVCodec.close (ffv1enc.c:1375 encode_close). */
void ffv1hip_destroy(ffv1hip_ctx *ctx);

/* avctx->extradata as written by write_extradata (ffv1enc.c:545-619); 0
 * bytes for version < 2.  Returns the size or a negative error. */
int ffv1hip_extradata(ffv1hip_ctx *ctx, uint8_t *buf, int cap);

/* Upper bound of one packet produced by this context: the slice byte budget
 * times the slices.  It grows after a budget re-encode, and a large batch
 * that lowers its budget to make room in HBM (its first batch) lowers it. */
int64_t ffv1hip_max_packet_size(const ffv1hip_ctx *ctx);

/* AVCodec.encode2 over a batch (ffv1enc.c:1222 encode_frame, called once
 * per frame in order).  planes[np*i + p] / strides[np*i + p] describe plane
 * p of frame i in HOST memory (np = 4 for the YUVA formats, else 3).  Packets are written back to back into `out`;
 * sizes[i] and key_flags[i] describe packet i.  P-frame context state
 * carries across calls exactly as across encode_frame calls.  Frames go in
 * max_batch_frames at a time through pinned staging buffers; with HBM for
 * two batches, batch k+1 is copied in while batch k codes and batch k-1's
 * packets are copied out (ffv1hip_encode2_delay). */
int ffv1hip_encode(ffv1hip_ctx *ctx, const void *const *planes,
                   const int *strides, int n_frames, uint8_t *out,
                   int64_t out_cap, int64_t *sizes, int *key_flags);

/* AVCodec.encode2 under AV_CODEC_CAP_DELAY, one frame per call the way
 * avcodec_encode_video2 drives it (libavcodec/utils.c:1922-1990; the
 * callback signature avcodec.h:3642-3643).  planes/strides: the frame's
 * planes in HOST memory (copied before the call returns), or planes == NULL
 * to flush (ffmpeg.c:1699-1776 passes NULL frames until no packet comes
 * back).  Frames queue up to the context's max_batch_frames and are encoded
 * together, on the GPU while the next batch queues: each call then hands
 * out at most one packet in input order, and the first packet comes with
 * frame ffv1hip_encode2_delay + 1.  Frames go to HBM through pinned staging
 * buffers (a few host threads copy into them, DMA on a transfer stream of
 * the context) and packets come back through a pinned buffer.  A returned
 * packet has pts = dts = its frame's pts and the key flag
 * (ffv1enc.c:1365-1370).  *got_packet = 1 when a packet was handed out.
 * With out == NULL the packet is handed out without a copy (size, pts and
 * key set) and ffv1hip_encode2_last_packet copies it: the flow for a
 * libavcodec shim, which allocates the AVPacket with the size it was given
 * (ff_alloc_packet2) and so never sees a packet larger than its buffer.
 * With a buffer, out should hold ffv1hip_max_packet_size bytes, which grows
 * after a slice byte budget re-encode: a packet larger than out_cap makes
 * the call return -ENOSPC with *size = the packet's size, having taken the
 * frame, and the packet stays pending: the next call, with a frame or with
 * planes == NULL, hands it out first (so planes == NULL is a flush only once
 * no packet is pending). */
int ffv1hip_encode2(ffv1hip_ctx *ctx, const void *const planes[4],
                    const int strides[4], int64_t pts, uint8_t *out,
                    int64_t out_cap, int64_t *size, int64_t *pts_out,
                    int *key, int *got_packet);

/* The packet the last ffv1hip_encode2 call handed out, copied into out
 * (cap bytes).  Returns its size, -ENOSPC (nothing copied) when cap is
 * smaller, -EINVAL when that call handed out no packet.  Valid until the
 * next ffv1hip_encode2 call. */
int64_t ffv1hip_encode2_last_packet(ffv1hip_ctx *ctx, uint8_t *out, int64_t cap);

/* Caller-pinned host memory for the host-frame paths: [ptr, ptr + bytes)
 * is page-locked (hipHostRegister) until ffv1hip_host_unregister or
 * ffv1hip_destroy, and a plane of ffv1hip_encode / ffv1hip_encode2 that lies
 * inside a registered range goes to HBM by DMA straight from it, without
 * the staging copy (ffv1hip_encode2 still returns only once the frame's
 * copy is done, so the caller may reuse the buffer as before).  For an
 * application's frame pool, whose buffers outlive the encoder calls: the
 * range must stay allocated while registered.  A range the process already
 * pinned itself is accepted and left pinned on unregister.  Returns 0,
 * -EINVAL (null, empty, or overlapping a registered range) or -ENOMEM (the
 * pages cannot be locked). */
int ffv1hip_host_register(ffv1hip_ctx *ctx, void *ptr, int64_t bytes);
/* Forget the range registered at ptr (its pages unlocked).  -EINVAL when
 * none starts there. */
int ffv1hip_host_unregister(ffv1hip_ctx *ctx, void *ptr);

/* The encoder's delay in frames (avctx->delay): 2 * max_batch_frames - 1
 * when two batches fit in HBM side by side (one codes while the next
 * queues), else max_batch_frames - 1.  Allocates the host-frame path's
 * buffers if they are not yet. */
int ffv1hip_encode2_delay(ffv1hip_ctx *ctx);

/* Device-resident variant: frames already in HBM at d_frames + i*frame_bytes
 * with plane p at byte offset plane_offset[p] and row stride plane_stride[p].
 * `stream` (a hipStream_t) is the stream the frames were written on: the
 * batch waits for the work queued on it so far, and for nothing else; NULL
 * when the frames are complete already.  The coding runs on the context's
 * internal streams, so that consecutive calls overlap.  Nothing is synchronised: the packets of
 * the LAST call are valid after ffv1hip_synchronize, ffv1hip_fetch or
 * ffv1hip_device_packets (each call's packets replace the previous call's).
 * Those three check the last call's slices against the slice byte budget: a
 * slice over it makes them encode that call again with a larger budget (its
 * input frames must still be in place), so no truncated slice is ever
 * handed out; if even that fails they return -ENOSPC. */
int ffv1hip_encode_device(ffv1hip_ctx *ctx, const void *d_frames,
                          int64_t frame_bytes, const int64_t plane_offset[4],
                          const int plane_stride[4], int n_frames,
                          void *stream);

/* Waits for all work of the context (every stream it uses), then settles
 * the last call's slice byte budget (see ffv1hip_encode_device). */
int ffv1hip_synchronize(ffv1hip_ctx *ctx);

/* Synchronises and copies the packets of the last encode_device call. */
int ffv1hip_fetch(ffv1hip_ctx *ctx, uint8_t *out, int64_t out_cap,
                  int64_t *sizes, int *key_flags);

/* Device pointers of the last call's packet slots: packet i starts at
 * (*d_packets + i * (*packet_stride)); sizes live in *d_sizes (int64).
 * Synchronises first (ffv1hip_synchronize): a budget re-encode may move the
 * slots. */
int ffv1hip_device_packets(ffv1hip_ctx *ctx, void **d_packets,
                           int64_t *packet_stride, void **d_sizes);

/* Next picture number (frames encoded so far) and a reset to a fresh
 * stream (next frame is a keyframe). */
int64_t ffv1hip_picture_number(const ffv1hip_ctx *ctx);
void ffv1hip_reset(ffv1hip_ctx *ctx);

/* Per-slice context-state snapshot (the P-frame carry) of the last frame of
 * the last call: [slice][plane_ctx 0..1][context][32] bytes.  Returns the
 * byte count written (or needed when buf is NULL). */
int64_t ffv1hip_get_slice_states(ffv1hip_ctx *ctx, uint8_t *buf, int64_t cap);
int     ffv1hip_set_slice_states(ffv1hip_ctx *ctx, const uint8_t *buf,
                                 int64_t size);
/* Resume a stream mid-GOP (the multi-GPU exchange step): the picture number
 * of the next frame, which places the keyframes (ffv1enc.c:1299).  With
 * ffv1hip_set_slice_states a second context continues another's P-frame
 * chain bit-exactly. */
int     ffv1hip_set_picture_number(ffv1hip_ctx *ctx, int64_t picture_number);
/* The same snapshot between device buffers (the exchange step over RCCL
 * with no host staging).  get: once the last call's batch is settled (its
 * slice budget checked), a device-to-device copy into d_buf is queued on
 * `stream` (a hipStream_t; NULL: the context's own), ordered after the
 * batch, and the context's later batches are ordered after that copy;
 * returns the byte count (or the size needed when d_buf is NULL).
 * set: the context's next frames start from the states at d_buf, copied on
 * the context's stream once the work queued so far on `stream` is done;
 * work queued on `stream` after the call runs after the copy (d_buf may be
 * rewritten there), and the context's next call sees the states. */
int64_t ffv1hip_get_slice_states_device(ffv1hip_ctx *ctx, void *d_buf,
                                        int64_t cap, void *stream);
int     ffv1hip_set_slice_states_device(ffv1hip_ctx *ctx, const void *d_buf,
                                        int64_t size, void *stream);

/* Kernel timing: when enabled, HIP events are recorded on the launch stream
 * around each kernel of every call; ffv1hip_last_kernel_ms synchronises and
 * returns, for the last call, the time from its first launch to the packet
 * assembly (every coding kernel) and that of the packet-assembly kernel
 * (ffv1_assemble_packets). */
int ffv1hip_set_profiling(ffv1hip_ctx *ctx, int enable);
int ffv1hip_last_kernel_ms(ffv1hip_ctx *ctx, float *encode_ms, float *assemble_ms);

/* Per-kernel totals of every call since profiling was (re)enabled: summed
 * HIP-event durations (events on each kernel's own stream) and launch counts
 * of ffv1_symbols (prediction/context), the states walk (ffv1_walk,
 * frame-parallel mode), the range coder (frame-parallel mode: ffv1_range,
 * the serial pass, in code_ms, then ffv1_dseg and ffv1_dfix; chained mode:
 * ffv1_code or ffv1_code_golomb), ffv1_assemble_packets, and in
 * frame-parallel mode the decision layout (ffv1_layout), the decision bits
 * (ffv1_bits) and the coder's byte writer (ffv1_sink).  Frame-parallel mode
 * launches each once per call; the chained mode launches symbols and code
 * once per frame index of the GOP. */
typedef struct ffv1hip_kernel_stats {
    float symbols_ms, code_ms, assemble_ms;
    int symbols_launches, code_launches, assemble_launches;
    int64_t frames_coded_per_launch_max;   /* slice streams per coder launch / nslices */
    float states_ms;                       /* context-state walk (frame-parallel mode) */
    int states_launches;
    float layout_ms, bits_ms;              /* frame-parallel mode */
    int layout_launches, bits_launches;
    float sink_ms;                         /* frame-parallel mode: the coder's byte writer (ffv1_sink) */
    int sink_launches;
    float dseg_ms, dfix_ms;                /* frame-parallel mode: the coder's segments (ffv1_dseg) and
                                              their join (ffv1_dfix); code_ms is then ffv1_range */
    int dseg_launches, dfix_launches;
} ffv1hip_kernel_stats;
int ffv1hip_last_kernel_stats(ffv1hip_ctx *ctx, ffv1hip_kernel_stats *out);

/* Decoder: the AVCodec callbacks of ff_ffv1_decoder (ffv1dec.c decode_init
 * :1007, decode_frame :896-1030, decode_end) for the streams this library
 * encodes: versions 0, 1, 2 (the slice layout in the keyframe header), 3 and
 * 4 (per-slice RCT coefficients, PCM slices),
 * range coder (default or custom table) or Golomb-Rice, context model 0 or
 * 1, YCbCr or RGB, with alpha (YUVA, YA8, RGB32).  ffv1hip_dec_create takes
 * the stream's parameters and its extradata, which must be the one those
 * parameters produce (what read_extradata, ffv1dec.c:509-631, would parse;
 * none below version 2, whose in-band keyframe header must agree with the
 * parameters, as must version 2's in-band slice layout); otherwise FFV1HIP_AVERROR_INVALIDDATA.  Unsupported
 * parameters give -ENOSYS. */
typedef struct ffv1hip_dec ffv1hip_dec;
ffv1hip_dec *ffv1hip_dec_create(const ffv1hip_params *params,
                                const uint8_t *extradata, int extradata_size,
                                int device, int *err);
void ffv1hip_dec_destroy(ffv1hip_dec *dec);
/* decode_frame over a batch: packets back to back in HOST memory (sizes[i]
 * bytes each); plane p of frame i goes to planes[np*i + p] with row stride
 * strides[np*i + p] (the encoder's input layout; np = FFV1HIP_PLANES_YUVA
 * for the YUVA formats, else FFV1HIP_PLANES).  The key bit and the slice
 * chain (3-byte sizes, CRC-32 when ec) are read on the host as in
 * ffv1dec.c:931-989; every (GOP segment, slice) chain decodes on the GPU.
 * Context states carry across calls like the encoder's.  key_flags may be
 * NULL. */
int ffv1hip_decode(ffv1hip_dec *dec, const uint8_t *packets,
                   const int64_t *sizes, int n_frames, void *const *planes,
                   const int *strides, int *key_flags);
/* Damaged slices are decoded on and concealed as the reference does
 * (ffv1dec.c:963-977, 410-414, 461-467, 998-1021): a slice failing its CRC
 * or its end position is decoded, then takes the previous picture's
 * rectangle; a slice failing its slice header is neither decoded nor copied
 * in that frame (ffv1dec.c:411-414 zeroes its size; the rectangle keeps
 * what the output buffer held, zeros here);
 * either way the slice is then concealed from the previous picture in every
 * later frame up to the next keyframe.  This is how many (frame, slice)
 * pairs of the last ffv1hip_decode call were damaged. */
int ffv1hip_dec_damaged_slices(const ffv1hip_dec *dec);
/* Forget the carried states and the previous picture: the next frame must
 * be a keyframe. */
void ffv1hip_dec_reset(ffv1hip_dec *dec);
/* Last error message (thread-local) and the ABI version. */
const char *ffv1hip_last_error(void);
int ffv1hip_abi_version(void);
/* 1 for the debug build (lib/libffv1hip_check.so, build.py --check): the
 * walk's and the coder's device writes are bounds-checked, and an encode
 * call whose batch wrote outside a buffer fails with -EFAULT naming the
 * kernel; 0 for the release build. */
int ffv1hip_debug_checks(void);
/* Test counters of a context (no reference counterpart): "guard_skips", the
 * batches the FFV1HIP_DEBUG=guard_skip hook launched so that their kernels
 * skip them, and "guard_reruns", the guarded batches encoded again at settle
 * because their decisions did not fit the decision set (status[3]); -1 for
 * an unknown name. */
int64_t ffv1hip_debug_counter(const ffv1hip_ctx *ctx, const char *name);

#ifdef __cplusplus
}
#endif
#endif
