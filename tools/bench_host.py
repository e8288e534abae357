#!/usr/bin/env python3
"""PCIe-inclusive rates: frames in HOST memory, the path an AVCodec shim takes.

1. ``ffv1hip_encode`` of many batches in one call (the frames staged into
   HBM through pinned buffers while the previous batch codes, the packets of
   the one before copied back);
2. ``ffv1hip_encode2`` one frame per call, the way avcodec_encode_video2
   drives AVCodec.encode2 (utils.c:1922-1990), at AV_CODEC_CAP_DELAY batch 1,
   12 and 252 (21 GOPs), flushed with NULL frames.

Steady state: each rate covers `batches` batches (default 10) of the same 252
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
gops = int(sys.argv[1]) if len(sys.argv) > 1 else 21
batches = int(sys.argv[2]) if len(sys.argv) > 2 else 10
out_json = sys.argv[3] if len(sys.argv) > 3 else None
B = gops * GOP
frames = list(synth.videogen_frames(W, H, B, depth=10))
L = load_library()
res = {"config": "4K 3840x2160 yuv420p10le, coder=1, slices=64, keyint=12", "clip_frames": B,
       "copy_threads": os.environ.get("OMP_NUM_THREADS")}


def plane_ptrs(idx):
    """ctypes plane pointer / stride arrays for the frames frames[i] of idx."""
    n = len(idx)
    ptrs = (ctypes.c_void_p * (3 * n))()
    strides = (ctypes.c_int * (3 * n))()
    for j, i in enumerate(idx):
        for k in range(3):
            ptrs[3 * j + k] = frames[i][k].ctypes.data
            strides[3 * j + k] = frames[i][k].strides[0]
    return ptrs, strides


params = configure(W, H, "yuv420p10", slices=64, coder=1, gop_size=GOP)

# 1. ffv1hip_encode: `batches` batches of B frames in one call
enc = HipEncoder(params, 0, B)
n = B * batches
ptrs, strides = plane_ptrs([i % B for i in range(n)])
cap = enc.max_packet_size() * 2 + n * (6 << 20)  # the clip codes to ~3.4 MB per frame
out = np.empty(cap, np.uint8)
sizes = (ctypes.c_int64 * n)()
keys = (ctypes.c_int * n)()
wp, ws = plane_ptrs(list(range(B)))
rc = L.ffv1hip_encode(enc._h, wp, ws, B, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), cap, sizes, keys)
assert rc == 0, rc  # warm-up: buffers, staging, threads
t0 = time.perf_counter()
rc = L.ffv1hip_encode(enc._h, ptrs, strides, n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), cap, sizes, keys)
dt = time.perf_counter() - t0
assert rc == 0, rc
pk_bytes = sum(sizes)
enc.close()
res["encode"] = {"frames": n, "batches": batches, "seconds": round(dt, 3), "mpix_s": round(n * W * H / dt / 1e6, 1),
                 "input_gb_s": round(n * W * H * 3 / dt / 1e9, 2),
                 "packet_gb_s": round(pk_bytes / dt / 1e9, 2)}
print(f"ffv1hip_encode, {n} frames ({batches} batches of {B}) in one call: {dt:.3f}s = "
      f"{n * W * H / dt / 1e6:.1f} Mpix/s ({n * W * H * 3 / dt / 1e9:.2f} GB/s of input in, "
      f"{pk_bytes / dt / 1e9:.2f} GB/s of packets out)", flush=True)
del out

# 2. ffv1hip_encode2: one frame per call
for batch in (1, 12, B):
    nb = batches if batch > 1 else 4
    n = max(2 * batch, batch * nb)
    enc = HipEncoder(params, 0, batch)
    delay = L.ffv1hip_encode2_delay(enc._h)
    pbuf = np.empty(enc.max_packet_size(), np.uint8)
    pp = pbuf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
    size, pts_out = ctypes.c_int64(), ctypes.c_int64()
    key, got = ctypes.c_int(), ctypes.c_int()
    fp = [plane_ptrs([i]) for i in range(B)]
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
    res[f"encode2_batch{batch}"] = {"frames": n, "delay": delay, "seconds": round(dt, 3),
                                    "mpix_s": round(n * W * H / dt / 1e6, 1),
                                    "ms_per_frame": round(dt / n * 1e3, 3)}
    print(f"ffv1hip_encode2, batch {batch} (delay {delay}): {n} frames in {dt:.3f}s = "
          f"{n * W * H / dt / 1e6:.1f} Mpix/s ({dt / n * 1e3:.2f} ms per frame)", flush=True)
if out_json:
    json.dump(res, open(out_json, "w"), indent=1)
