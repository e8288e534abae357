#!/usr/bin/env python3
"""Per-kernel timing of one batch (argv: width height slices frames gop [reps])."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd"))
import numpy as np
import torch
from ffv1hip import HipEncoder, configure, synth

w, h, sl, n, g = (int(x) for x in sys.argv[1:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 2
p = configure(w, h, "yuv420p10", slices=sl, coder=1, gop_size=g)
shapes = p.plane_shapes()
pb = [a * b * 2 for a, b in shapes]
fb = (sum(pb) + 255) // 256 * 256
uniq = min(n, 24)
frames = list(synth.videogen_frames(w, h, uniq, depth=10))
host = np.zeros((n, fb), np.uint8)
for i in range(n):
    f = frames[i % uniq]
    flat = np.concatenate([x.reshape(-1).view(np.uint8) for x in f]); host[i, :flat.size] = flat
d = torch.from_numpy(host).cuda()
enc = HipEncoder(p, 0, n); enc.set_profiling(True)
offs = [0, pb[0], pb[0] + pb[1]]; st = [shapes[0][1] * 2, shapes[1][1] * 2, shapes[2][1] * 2]
for r in range(reps):
    enc.encode_device(d.data_ptr(), fb, offs, st, n)
    s = enc.last_kernel_stats()
    e, a = enc.last_kernel_ms()
    print(json.dumps({"label": f"{w}x{h}_s{sl}_n{n}_g{g}", "rep": r, "total_ms": round(e + a, 3),
                      **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in s.items()},
                      "mpix_s": round(n * w * h / ((e + a) * 1e3), 1)}), flush=True)
pk = enc.fetch(n)
print(json.dumps({"bytes": sum(len(x) for x, _ in pk)}))
enc.close()
