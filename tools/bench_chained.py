#!/usr/bin/env python3
"""Throughput of the chained coders, HBM-resident frames.

The frame-parallel range coder (bench.py) covers context model 0 YCbCr.
Everything else goes through the chained coders: ffv1_code (range coder:
context model 1, RGB, alpha, version 4) and ffv1_code_golomb (coder=0).  They
keep one lane per (GOP segment, slice) and code a GOP's frames one after the
other.  Per case:
  - `encode_device` of one batch resident in HBM, timed over `steps` calls
    after a warm-up (the same contract as bench.py's `value`);
  - the first GOP's packets against the oracle encoder (bit-exact);
  - the oracle on this host's cores (GOP-sharded threads) as the CPU
    baseline.

Cases: BASELINE configs[0] (CIF yuv420p Golomb, intra), Golomb at 1080p
(24 slices, intra), context model 1 at the c3 shape (4K yuv420p10, 64 slices,
g=12), and bgr0 at 1080p (24 slices, g=12, the reversible colour transform).
Usage: python tools/bench_chained.py [out.json] [steps] [case,case,...]
"""
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd")]

import bench  # noqa: E402  (cpu_threads)
from oracle import oracle  # noqa: E402

CASES = [
    # name, W, H, pix_fmt, slices, coder, context, gop, batch frames, source
    ("c1_cif_golomb_intra", 352, 288, "yuv420p", 0, 0, 0, 1, 600, "d1"),
    ("golomb_1080p_intra_s24", 1920, 1080, "yuv420p", 24, 0, 0, 1, 240, "d1"),
    ("ctx1_4k_p10_s64_g12", 3840, 2160, "yuv420p10", 64, 1, 1, 12, 240, "d1"),
    ("bgr0_1080p_s24_g12", 1920, 1080, "bgr0", 24, 1, 0, 12, 240, "d1"),
    # the same P-frame streams with more GOPs per call: a chain per (GOP,
    # slice) lane, so the lanes (and waves) grow with the batch
    ("ctx1_4k_p10_s64_g12_b960", 3840, 2160, "yuv420p10", 64, 1, 1, 12, 960, "d1"),
    ("bgr0_1080p_s24_g12_b2400", 1920, 1080, "bgr0", 24, 1, 0, 12, 2400, "d1"),
]


def frames_of(W, H, pix_fmt, n):
    from ffv1hip import synth
    if pix_fmt == "bgr0":
        return [synth.yuv420p_to_bgr0(f) for f in synth.videogen_frames(W, H, n)]
    depth = 10 if pix_fmt.endswith("p10") else 8
    return list(synth.videogen_frames(W, H, n, depth=depth))


def main():
    import torch
    from ffv1hip import HipEncoder, configure
    out_json = sys.argv[1] if len(sys.argv) > 1 else None
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    only = set(sys.argv[3].split(",")) if len(sys.argv) > 3 else None
    threads = bench.cpu_threads()
    res = {"cases": [], "cpu_threads": threads, "steps": steps}
    for name, W, H, pf, slices, coder, context, gop, B, data in CASES:
        if only and name not in only:
            continue
        t0 = time.perf_counter()
        frames = frames_of(W, H, pf, B)
        params = configure(W, H, pf, slices=slices, coder=coder, context=context, gop_size=gop)
        # the planes as the frames hold them (bgr0: one packed plane)
        plane_bytes = [q.nbytes for q in frames[0]]
        frame_bytes = (sum(plane_bytes) + 255) // 256 * 256
        offs = [int(sum(plane_bytes[:k])) for k in range(len(plane_bytes))]
        offs += [0] * (4 - len(offs))
        strides = [q.strides[0] for q in frames[0]] + [0] * (4 - len(frames[0]))
        host = np.zeros((B, frame_bytes), np.uint8)
        for i, f in enumerate(frames):
            flat = np.concatenate([p.reshape(-1).view(np.uint8) for p in f])
            host[i, :flat.size] = flat
        d = torch.from_numpy(host).to("cuda:0")
        torch.cuda.synchronize()
        enc = HipEncoder(params, 0, B)
        enc.encode_device(d.data_ptr(), frame_bytes, offs, strides, B)  # warm-up
        enc.synchronize()
        enc.set_profiling(True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(steps):
            enc.encode_device(d.data_ptr(), frame_bytes, offs, strides, B)
        enc.synchronize()
        el = time.perf_counter() - t1
        stats = enc.last_kernel_stats()
        pk = enc.fetch(B)
        enc.close()
        del d
        torch.cuda.empty_cache()
        mpix = steps * B * W * H / el / 1e6
        # the first GOP (or 12 intra frames) against the oracle
        n_chk = max(gop, 1) if gop > 1 else 12
        cfg = oracle.configure(W, H, pf, slices=slices, coder=coder, context=context, gop_size=gop)
        oe = oracle.Encoder(cfg)
        ref = [oe.encode(f)[0] for f in frames[:n_chk]]
        equal = [p for p, _ in pk[:n_chk]] == ref
        # CPU: GOP-sharded oracle threads over a bounded sample
        per = max(gop, 1)
        workers = threads
        sample = [frames[(g * per) % B:(g * per) % B + per] for g in range(workers)]

        def one(fr):
            e = oracle.Encoder(cfg)
            for f in fr:
                e.encode(f)
        th = [threading.Thread(target=one, args=(s,)) for s in sample]
        tc = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        cpu = sum(len(s) for s in sample) * W * H / (time.perf_counter() - tc) / 1e6
        case = {"name": name, "config": f"{W}x{H} {pf}, coder={coder}, context={context}, slices={slices}, g={gop}",
                "frames_per_call": B, "mpix_s": round(mpix, 2), "ms_per_call": round(el / steps * 1e3, 3),
                "kernel_ms_per_call": {"symbols": round(stats["symbols_ms"] / steps, 3),
                                       "code": round(stats["code_ms"] / steps, 3),
                                       "assemble": round(stats["assemble_ms"] / steps, 3)},
                "code_launches_per_call": stats["code_launches"] // steps,
                "bitexact_vs_oracle_first_frames": {"frames": n_chk, "equal": equal},
                "bits_per_pixel": round(sum(len(p) for p, _ in pk) * 8 / (B * W * H), 4),
                "cpu_baseline": {"value": round(cpu, 2), "unit": "Mpixels/s", "cores": workers, "kind": "port",
                                 "sample": f"{workers} oracle threads x {per} frame(s)"},
                "setup_s": round(time.perf_counter() - t0, 1)}
        print(json.dumps(case), flush=True)
        res["cases"].append(case)
    if out_json:
        json.dump(res, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main()
