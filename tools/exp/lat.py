"""Latency of small batches (device-resident 4K c3 frames): ms per batch
(encode_device + synchronize, one batch at a time) and the kernel times."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from ffv1hip import HipEncoder  # noqa: E402

params = bench.hip_configure()
shapes = params.plane_shapes()
pb = [h * w * params.sample_bytes for h, w in shapes]
fb = (sum(pb) + 255) // 256 * 256
offs = [0, pb[0], pb[0] + pb[1]]
strides = [shapes[k][1] * params.sample_bytes for k in range(3)]
frames = bench.make_frames(24, "d1", keep=lambda i: True)
d = torch.from_numpy(bench.pack_batch(frames, fb)).cuda()
torch.cuda.synchronize()
for b in [int(x) for x in (sys.argv[1:] or ["1", "12"])]:
    enc = HipEncoder(params, 0, b)
    for rep in range(2):
        enc.set_profiling(rep == 1)
        ts = []
        for i in range(0, 24, b):
            t0 = time.perf_counter()
            enc.encode_device(d.data_ptr() + i * fb, fb, offs, strides, b)
            enc.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        if rep == 1:
            st = enc.last_kernel_stats()
            ks = {k: round(v, 2) for k, v in st.items() if isinstance(v, float)}
            print(f"batch {b}: median {ts[len(ts) // 2] * 1e3:.2f} ms per batch (min {ts[0] * 1e3:.2f}), "
                  f"{ts[len(ts) // 2] * 1e3 / b:.2f} ms per frame; kernels {ks}", flush=True)
    enc.close()
