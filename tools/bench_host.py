#!/usr/bin/env python3
"""PCIe-inclusive rates: frames in HOST memory, the path an AVCodec shim takes.

1. ``ffv1hip_encode`` of a whole batch (H2D of the planes, the encode, D2H of
   the packets);
2. ``ffv1hip_encode2`` one frame per call, the way avcodec_encode_video2
   drives AVCodec.encode2 (utils.c:1922-1990), at AV_CODEC_CAP_DELAY batch 1
   (no delay: every call encodes its frame) and 12 / 252 (one GOP / 21 GOPs
   in flight), flushed with NULL frames.

bench.py's `value` is the HBM-resident rate; these are the numbers DESIGN.md
quotes beside it.  Usage: python tools/bench_host.py [gops] [repeats] [out.json]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd")]

from ffv1hip import AVCodecContext, FFV1Encoder, HipEncoder, configure, synth  # noqa: E402

W, H, GOP = 3840, 2160, 12
gops = int(sys.argv[1]) if len(sys.argv) > 1 else 21
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
out_json = sys.argv[3] if len(sys.argv) > 3 else None
B = gops * GOP
frames = list(synth.videogen_frames(W, H, B, depth=10))
res = {"config": "4K 3840x2160 yuv420p10le, coder=1, slices=64, keyint=12", "frames": B}

enc = HipEncoder(configure(W, H, "yuv420p10", slices=64, coder=1, gop_size=GOP), 0, B)
enc.encode(frames[:GOP])  # warm-up
best = None
for _ in range(reps):
    t0 = time.perf_counter()
    pk = enc.encode(frames)
    dt = time.perf_counter() - t0
    best = dt if best is None else min(best, dt)
enc.close()
mb = sum(len(p) for p, _ in pk) / 1e6
res["encode_batch"] = {"mpix_s": round(B * W * H / best / 1e6, 1), "seconds": round(best, 3),
                       "input_gb_s": round(B * W * H * 3 / best / 1e9, 2), "packet_mb": round(mb)}
print(f"ffv1hip_encode, {B} frames per call: {best:.3f}s = {B * W * H / best / 1e6:.1f} Mpix/s "
      f"({B * W * H * 3 / best / 1e9:.2f} GB/s of input over PCIe, {mb:.0f} MB of packets back)", flush=True)

for batch in (1, 12, B):
    n = min(B, max(24, 2 * batch))
    best = None
    for _ in range(max(1, reps - 1)):
        e = FFV1Encoder(batch=batch)
        e.init(AVCodecContext(W, H, "yuv420p10", gop_size=GOP, slices=64, coder=1))
        got = 0
        t0 = time.perf_counter()
        for i, f in enumerate(frames[:n]):
            got += e.encode2(f, pts=i) is not None
        while e.encode2(None) is not None:
            got += 1
        dt = time.perf_counter() - t0
        e.close()
        assert got == n
        best = dt if best is None else min(best, dt)
    res[f"encode2_batch{batch}"] = {"frames": n, "mpix_s": round(n * W * H / best / 1e6, 1),
                                    "ms_per_frame": round(best / n * 1e3, 2)}
    print(f"ffv1hip_encode2, batch {batch}: {n} frames in {best:.3f}s = {n * W * H / best / 1e6:.1f} Mpix/s "
          f"({best / n * 1e3:.1f} ms per frame)", flush=True)
if out_json:
    json.dump(res, open(out_json, "w"), indent=1)
