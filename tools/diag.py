#!/usr/bin/env python3
"""Diagnostics: per-chain latency vs concurrency of ffv1_encode_slices."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd"))
import numpy as np
import torch
from ffv1hip import HipEncoder, configure, synth

def run(w, h, slices, nframes, gop, label, reps=2):
    p = configure(w, h, "yuv420p10", slices=slices, coder=1, gop_size=gop)
    shapes = p.plane_shapes()
    pb = [a * b * 2 for a, b in shapes]
    fb = (sum(pb) + 255) // 256 * 256
    frames = list(synth.videogen_frames(w, h, nframes, depth=10))
    host = np.zeros((nframes, fb), np.uint8)
    for i, f in enumerate(frames):
        flat = np.concatenate([x.reshape(-1).view(np.uint8) for x in f]); host[i, :flat.size] = flat
    d = torch.from_numpy(host).cuda()
    enc = HipEncoder(p, 0, nframes); enc.set_profiling(True)
    offs = [0, pb[0], pb[0] + pb[1]]; st = [shapes[0][1] * 2, shapes[1][1] * 2, shapes[2][1] * 2]
    best = 1e9
    for _ in range(reps):
        enc.encode_device(d.data_ptr(), fb, offs, st, nframes)
        e, a = enc.last_kernel_ms(); best = min(best, e)
    pk = enc.fetch(nframes)
    nsl = p.num_h_slices * p.num_v_slices
    samples = w * h * 1.5
    chains = nsl * ((nframes + gop - 1) // gop)
    per_chain_frames = min(gop, nframes)
    sym_per_chain = samples / nsl * per_chain_frames
    print(json.dumps({"label": label, "chains": chains, "kernel_ms": round(best, 3),
                      "ns_per_symbol_per_chain": round(best * 1e6 / sym_per_chain, 2),
                      "bytes": sum(len(x) for x, _ in pk)}), flush=True)
    enc.close()

if __name__ == "__main__":
  run(480, 270, 1, 1, 12, "1chain_480x270_1frame")
  run(480, 270, 1, 4, 12, "1chain_480x270_4frames")
  run(960, 540, 4, 1, 12, "4chains")
  run(3840, 2160, 64, 1, 12, "64chains_4k_1frame")
  run(3840, 2160, 64, 12, 12, "64chains_4k_12frames")
  run(3840, 2160, 64, 48, 12, "256chains_4k_48frames")
  run(3840, 2160, 64, 96, 12, "512chains_4k_96frames")
  run(3840, 2160, 64, 144, 12, "768chains_4k_144frames", reps=1)
