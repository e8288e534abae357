#!/usr/bin/env python3
"""PCIe-inclusive rates: frames in HOST memory, the path an AVCodec shim takes.

1. ``ffv1hip_encode`` of many batches in one call (the frames copied into
   HBM while the previous batch codes, the packets of the one before copied
   back);
2. ``ffv1hip_encode2`` one frame per call, the way avcodec_encode_video2
   drives AVCodec.encode2 (utils.c:1922-1990), at AV_CODEC_CAP_DELAY batch 1,
   12, 48 and the clip's (20 GOPs: 240), flushed with NULL frames.

Each twice: frames in pageable memory (staged through pinned buffers by the
copy threads) and in one caller-pinned pool (ffv1hip_host_register, the
frames DMA'd straight from it; the one-time registration is reported apart).
Steady state: each rate covers `batches` batches (default 10) of the same
host frames (4K yuv420p10le, the bench clip), timed around the C calls only.
bench.py's `value` is the HBM-resident rate; these are the numbers DESIGN.md
quotes beside it.  Usage: python tools/bench_host.py [gops] [batches] [out.json]
"""
import ctypes
import json
import os
import sys
import time


import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd")]

from ffv1hip import HipEncoder, configure, synth  # noqa: E402
from ffv1hip.encoder import load_library  # noqa: E402

W, H, GOP = 3840, 2160, 12
gops = int(sys.argv[1]) if len(sys.argv) > 1 else 20
batches = int(sys.argv[2]) if len(sys.argv) > 2 else 10
out_json = sys.argv[3] if len(sys.argv) > 3 else None
B = gops * GOP
src = list(synth.videogen_frames(W, H, B, depth=10))
L = load_library()
res = {"config": "4K 3840x2160 yuv420p10le, coder=1, slices=64, keyint=12", "clip_frames": B,
       "copy_threads": os.environ.get("OMP_NUM_THREADS"),
       "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "4 (runtime default)"), "hooks": os.environ.get("FFV1HIP_DEBUG")}
# the pool: every frame's planes back to back in one buffer (an application's frame pool)
fbytes = sum(p.nbytes for p in src[0])
pool = np.empty(fbytes * B, np.uint8)
pooled = []
off = 0
for f in src:
    v = []
    for p in f:
        a = pool[off:off + p.nbytes].view(p.dtype).reshape(p.shape)
        a[...] = p
        v.append(a)
        off += p.nbytes
    pooled.append(v)


def plane_ptrs(frames, idx):
    """ctypes plane pointer / stride arrays for the frames frames[i] of idx."""
    n = len(idx)
    ptrs = (ctypes.c_void_p * (3 * n))()
    strides = (ctypes.c_int * (3 * n))()
    for j, i in enumerate(idx):
        for k in range(3):
            ptrs[3 * j + k] = frames[i][k].ctypes.data
            strides[3 * j + k] = frames[i][k].strides[0]
    return ptrs, strides


def register(enc):
    t0 = time.perf_counter()
    rc = L.ffv1hip_host_register(enc._h, pool.ctypes.data, pool.nbytes)
    assert rc == 0, L.ffv1hip_last_error()
    return time.perf_counter() - t0


params = configure(W, H, "yuv420p10", slices=64, coder=1, gop_size=GOP)

for mode in ("staged", "registered"):
    frames = src if mode == "staged" else pooled
    # 1. ffv1hip_encode: `batches` batches of B frames in one call
    enc = HipEncoder(params, 0, B)
    if mode == "registered":
        res["register_s"] = round(register(enc), 3)
        res["register_gb"] = round(pool.nbytes / 1e9, 2)
    n = B * batches
    ptrs, strides = plane_ptrs(frames, [i % B for i in range(n)])
    cap = enc.max_packet_size() * 2 + n * (6 << 20)  # the clip codes to ~3.4 MB per frame
    out = np.empty(cap, np.uint8)
    sizes = (ctypes.c_int64 * n)()
    keys = (ctypes.c_int * n)()
    wp, ws = plane_ptrs(frames, list(range(B)))
    rc = L.ffv1hip_encode(enc._h, wp, ws, B, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), cap, sizes, keys)
    assert rc == 0, rc  # warm-up: buffers, staging, threads
    t0 = time.perf_counter()
    rc = L.ffv1hip_encode(enc._h, ptrs, strides, n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), cap, sizes,
                          keys)
    dt = time.perf_counter() - t0
    assert rc == 0, rc
    pk_bytes = sum(sizes)
    enc.close()
    key = "encode" if mode == "staged" else "encode_registered"
    res[key] = {"frames": n, "batches": batches, "seconds": round(dt, 3), "mpix_s": round(n * W * H / dt / 1e6, 1),
                "input_gb_s": round(n * fbytes / dt / 1e9, 2), "packet_gb_s": round(pk_bytes / dt / 1e9, 2)}
    print(f"ffv1hip_encode ({mode}), {n} frames ({batches} batches of {B}) in one call: {dt:.3f}s = "
          f"{n * W * H / dt / 1e6:.1f} Mpix/s ({n * fbytes / dt / 1e9:.2f} GB/s of input in, "
          f"{pk_bytes / dt / 1e9:.2f} GB/s of packets out)", flush=True)
    del out

    # 2. ffv1hip_encode2: one frame per call
    for batch in (1, 12, 48, B):
        nb = batches if batch > 1 else 4
        n = max(2 * batch, batch * nb)
        enc = HipEncoder(params, 0, batch)
        if mode == "registered":
            register(enc)
        delay = L.ffv1hip_encode2_delay(enc._h)
        pbuf = np.empty(enc.max_packet_size(), np.uint8)
        pp = pbuf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        size, pts_out = ctypes.c_int64(), ctypes.c_int64()
        key, got = ctypes.c_int(), ctypes.c_int()
        fp = [plane_ptrs(frames, [i]) for i in range(B)]
        got_n = 0
        t0 = time.perf_counter()
        for i in range(n):
            p3, s3 = fp[i % B]
            rc = L.ffv1hip_encode2(enc._h, p3, s3, i, pp, pbuf.size, ctypes.byref(size), ctypes.byref(pts_out),
                                   ctypes.byref(key), ctypes.byref(got))
            assert rc == 0, rc
            got_n += got.value
        while True:
            rc = L.ffv1hip_encode2(enc._h, None, None, 0, pp, pbuf.size, ctypes.byref(size), ctypes.byref(pts_out),
                                   ctypes.byref(key), ctypes.byref(got))
            assert rc == 0, rc
            if not got.value:
                break
            got_n += 1
        dt = time.perf_counter() - t0
        enc.close()
        assert got_n == n, (got_n, n)
        k2 = f"encode2_batch{batch}" + ("" if mode == "staged" else "_registered")
        res[k2] = {"frames": n, "delay": delay, "seconds": round(dt, 3), "mpix_s": round(n * W * H / dt / 1e6, 1),
                   "ms_per_frame": round(dt / n * 1e3, 3)}
        print(f"ffv1hip_encode2 ({mode}), batch {batch} (delay {delay}): {n} frames in {dt:.3f}s = "
              f"{n * W * H / dt / 1e6:.1f} Mpix/s ({dt / n * 1e3:.2f} ms per frame)", flush=True)
if out_json:
    json.dump(res, open(out_json, "w"), indent=1)
