#!/usr/bin/env python3
"""Per-GOP packet digests of every bench.py workload, from the CPU oracle.

bench.py encodes GOPs of one synthetic D1 clip (tests/videogen widened to the
config's depth); rank r of N encodes GOPs r, r+N, ...  This script encodes
the first `--gops` GOPs of each config's clip with the oracle
(oracle/ffv1_oracle.c, itself pinned to the reference's FATE vectors and
known-answer MD5s, tests/golden/) and writes tests/golden/bench_gops.json:
for every GOP its packets' MD5 (over the concatenated packets) and byte
count.  bench.py then checks every GOP it timed against this file, so every
frame of the timed region is compared with the oracle, not only the first
24 frames that the reference's own MD5 pins.

GOPs are independent (keyframes reset every context state,
ffv1enc.c:1171-1172), so each is encoded by its own oracle instance on a
worker thread (ctypes drops the GIL).

    python tools/make_bench_golden.py                 # all configs, 8 ranks' worth
    python tools/make_bench_golden.py --configs c3 --ranks 1
    python tools/make_bench_golden.py --configs c3 --data d2 --gops 40   # key c3_d2
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd"))

import bench  # noqa: E402  (CONFIGS: the bench's workloads)
from ffv1hip import synth  # noqa: E402
from oracle import oracle  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "bench_gops.json")


def oracle_cfg(c):
    if c["GRID"]:
        cfg = oracle.configure(c["W"], c["H"], c["PIX_FMT"], slices=0, coder=1, gop_size=c["GOP"])
        cfg.num_h_slices, cfg.num_v_slices = 16, 16
        return cfg
    return oracle.configure(c["W"], c["H"], c["PIX_FMT"], slices=c["SLICES"], coder=1,
                            gop_size=c["GOP"], bits_per_raw_sample=c["BPR"])


def encode_gop(cfg, frames):
    enc = oracle.Encoder(cfg)
    h, n = hashlib.md5(), 0
    for f in frames:
        p, _ = enc.encode(f)
        h.update(p)
        n += len(p)
    return h.hexdigest(), n


def run_config(name, ngops, threads, data="d1"):
    c = bench.CONFIGS[name]
    cfg = oracle_cfg(c)
    per = max(c["GOP"], 1)
    group = per  # intra configs (GOP 1): one frame per entry
    if data == "d1":
        gen = synth.videogen_frames(c["W"], c["H"], ngops * group, depth=c["DEPTH"], chroma444=c["C444"])
    else:  # the seeded LSB-active clip bench.py --data d2 encodes
        gen = synth.d2_frames(c["W"], c["H"], ngops * group, depth=c["DEPTH"], chroma444=c["C444"])
    res = [None] * ngops
    t0 = time.time()
    with cf.ThreadPoolExecutor(threads) as ex:
        pending = {}
        for g in range(ngops):
            frames = [next(gen) for _ in range(group)]
            pending[ex.submit(encode_gop, cfg, frames)] = g
            while len(pending) >= 2 * threads:  # bound the frames held in memory
                done, _ = cf.wait(pending, return_when=cf.FIRST_COMPLETED)
                for d in done:
                    res[pending.pop(d)] = d.result()
        for d in cf.as_completed(pending):
            res[pending[d]] = d.result()
    print(f"{name}: {ngops} GOPs of {group} frames in {time.time() - t0:.1f}s", flush=True)
    return {"workload": c["workload"], "frames_per_gop": group, "data": data,
            "gops": [{"md5": m, "bytes": b} for m, b in res]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c2,c4,c5")
    ap.add_argument("--ranks", type=int, default=8, help="GOPs for this many ranks at the default batch")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--data", choices=("d1", "d2"), default="d1",
                    help="clip: d1 (videogen, key <config>) or d2 (key <config>_d2)")
    ap.add_argument("--gops", type=int, default=0, help="GOPs per config (default: --ranks x the bench batch)")
    args = ap.parse_args()
    data = json.load(open(OUT)) if os.path.exists(OUT) else {}
    data["note"] = ("per-GOP oracle digests of bench.py's D1 clips (tools/make_bench_golden.py); "
                    "md5 over the GOP's packets in order")
    for name in args.configs.split(","):
        c = bench.CONFIGS[name]
        # intra 1080p: 2 ranks' worth of frames keeps the file small
        ranks = args.ranks if c["GOP"] > 1 else min(args.ranks, 2)
        key = name if args.data == "d1" else f"{name}_d2"
        data[key] = run_config(name, args.gops or c["GOPS"] * ranks, args.threads, args.data)
        with open(OUT, "w") as f:
            json.dump(data, f, indent=0)
            f.write("\n")


if __name__ == "__main__":
    main()
