"""Full-GOP parity of the bench workloads in the driver's GPU run.

bench.py checks every GOP it times against the oracle's per-GOP digests
(tests/golden/bench_gops.json, tools/make_bench_golden.py), but only in the
bench line.  Here one whole 12-frame GOP (a keyframe and 11 P-frames: the
context-state carry over a full GOP) of each config the bench runs besides
the default is encoded at full size through the HBM-resident path the bench
times (ffv1hip_encode_device) and compared with the same digests:

  c4     4K yuv444p16 at 12 bit (u16 >> 4), D1 clip (parity unpinned: no
         reference vector, the oracle restatement's digests)
  c5     8K yuv420p10, 16x16 slice grid, D1 clip (not encodable
         by the reference; the oracle restatement's digests)
  c3_d2  4K yuv420p10, 64 slices, the LSB-active D2 clip
"""
import hashlib

import numpy as np
import pytest

import bench

pytestmark = pytest.mark.gpu

CASES = [("c4", "d1", 0), ("c5", "d1", 0), ("c3", "d2", 0), ("c3", "d2", 1)]


@pytest.mark.parametrize("config,data,gop", CASES, ids=[f"{c}_{d}_gop{g}" for c, d, g in CASES])
def test_full_gop_matches_oracle_digest(config, data, gop):
    import torch
    from ffv1hip import HipEncoder

    bench.select_config(config)
    golden = bench.load_bench_golden(config if data == "d1" else f"{config}_d2")
    assert golden and len(golden["gops"]) > gop
    G = bench.GOP
    params = bench.hip_configure()
    shapes = params.plane_shapes()
    plane_bytes = [h * w * params.sample_bytes for h, w in shapes]
    frame_bytes = (sum(plane_bytes) + 255) // 256 * 256
    offs = [0, plane_bytes[0], plane_bytes[0] + plane_bytes[1]]
    strides = [shapes[k][1] * params.sample_bytes for k in range(3)]
    host, _ = bench.pack_clip(bench.clip_frames((gop + 1) * G, data, keep=lambda i: i // G == gop), G, frame_bytes)
    d_frames = torch.from_numpy(host).to("cuda:0")
    torch.cuda.synchronize()
    enc = HipEncoder(params, 0, G)
    try:
        enc.encode_device(d_frames.data_ptr(), frame_bytes, offs, strides, G)
        pkts = enc.fetch(G)
    finally:
        enc.close()
    assert [k for _, k in pkts] == [1] + [0] * (G - 1)
    h = hashlib.md5()
    for p, _ in pkts:
        h.update(p)
    ref = golden["gops"][gop]
    assert (h.hexdigest(), sum(len(p) for p, _ in pkts)) == (ref["md5"], ref["bytes"])
    del d_frames
    torch.cuda.empty_cache()
