"""Decoder timing: one GOP (64 chains) vs 24 GOPs (1536 chains) of the 4K
D1 clip, wall time of HipDecoder.decode (packets in, frames out)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd")]
import torch  # noqa: F401  (HIP runtime first)
from ffv1hip import HipEncoder, HipDecoder, configure, synth
W, H = 3840, 2160
params = configure(W, H, "yuv420p10", slices=64, coder=1, gop_size=12)
frames = list(synth.videogen_frames(W, H, 24, depth=10))
enc = HipEncoder(params, 0, 24)
pk = [p for p, _ in enc.encode(frames)]
ex = enc.extradata()
enc.close()
for n in (12, 24):
    for rep in range(2):
        dec = HipDecoder(params, ex, 0)
        t = time.perf_counter()
        dec.decode(pk[:n])
        print(f"{n} frames ({n // 12 * 64} chains): {time.perf_counter() - t:.3f} s", flush=True)
        dec.close()
# 288 frames = 24 GOPs of the same 2 GOPs repeated
big = pk * 12
dec = HipDecoder(params, ex, 0)
t = time.perf_counter()
dec.decode(big)
print(f"288 frames (1536 chains): {time.perf_counter() - t:.3f} s", flush=True)
