#!/usr/bin/env python3
"""PCIe-inclusive rate: ffv1hip_encode with frames in HOST memory (H2D of the
planes, the encode, D2H of the packets), the path an AVCodec shim takes.
bench.py's `value` is the HBM-resident rate; this is the number DESIGN.md
quotes beside it.  Usage: python tools/bench_host.py [gops] [repeats]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd")]

from ffv1hip import HipEncoder, configure, synth  # noqa: E402

W, H, GOP = 3840, 2160, 12
gops = int(sys.argv[1]) if len(sys.argv) > 1 else 21
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
B = gops * GOP
frames = list(synth.videogen_frames(W, H, B, depth=10))
enc = HipEncoder(configure(W, H, "yuv420p10", slices=64, coder=1, gop_size=GOP), 0, B)
enc.encode(frames[:GOP])  # warm-up
best = None
for _ in range(reps):
    t0 = time.perf_counter()
    pk = enc.encode(frames)
    dt = time.perf_counter() - t0
    best = dt if best is None else min(best, dt)
mb = sum(len(p) for p, _ in pk) / 1e6
print(f"host-buffer encode: {B} frames in {best:.3f}s = {B * W * H / best / 1e6:.1f} Mpix/s "
      f"({B * W * H * 3 / best / 1e9:.2f} GB/s of input over PCIe, {mb:.0f} MB of packets back)")
