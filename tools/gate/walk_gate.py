#!/usr/bin/env python3
"""The walk gate: dump (GOP, slice, plane group) chains
of a BASELINE config's clip from the oracle (ffv1o_slice_symbols: context and
folded residual per sample, coding order) and run walk_gate.c on each.

    python tools/gate/walk_gate.py --config c3 --data d1 --slices 0,27,63

Prints one JSON object per chain (the luma chain, and the chroma chain: Cb
and Cr share context set 1, ffv1enc.c:1194-1195).  A measurement tool; the
oracle is the checker here, as everywhere outside the product.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ffmpeg-ffv1-p-frames_amd"))

import bench  # noqa: E402  (config table and clip generators)
from oracle import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--data", default="d1")
    ap.add_argument("--slices", default="0,27,63")
    ap.add_argument("--gop", type=int, default=0, help="which GOP of the clip")
    args = ap.parse_args()
    bench.select_config(args.config)
    exe = os.path.join(ROOT, "tools", "gate", "walk_gate")
    if not os.path.exists(exe):
        subprocess.check_call(["gcc", "-O2", "-w", "-o", exe, exe + ".c", "-lm"])
    G = max(bench.GOP, 1)
    first = args.gop * G
    frames = bench.make_frames(first + G, args.data, keep=lambda i: i >= first)
    cfg = oracle.configure(bench.W, bench.H, bench.PIX_FMT, slices=bench.SLICES, coder=1, gop_size=bench.GOP,
                           bits_per_raw_sample=bench.BPR)
    out = []
    for s in [int(x) for x in args.slices.split(",")]:
        chains = {"luma": [], "chroma": []}
        counts = {"luma": [], "chroma": []}
        for f in frames:
            sym = oracle.slice_symbols(cfg, f, s)
            # plane 0's symbols first: the slice's luma rectangle
            x0, y0, x1, y1 = rect(cfg, s)
            nl = (x1 - x0) * (y1 - y0)
            chains["luma"].append(sym[:nl])
            chains["chroma"].append(sym[nl:])
            counts["luma"].append(nl)
            counts["chroma"].append(len(sym) - nl)
        for grp in ("luma", "chroma"):
            with tempfile.TemporaryDirectory() as td:
                cb = os.path.join(td, "chain.bin")
                np.concatenate(chains[grp]).astype(np.int32).tofile(cb)
                ft = os.path.join(td, "frames.txt")
                open(ft, "w").write("\n".join(map(str, counts[grp])) + "\n")
                r = json.loads(subprocess.check_output([exe, cb, ft]))
            r.update(config=args.config, data=args.data, slice=s, group=grp, gop=args.gop)
            print(json.dumps(r), flush=True)
            out.append(r)


def rect(cfg, i):
    from tests.helpers import slice_rect
    return slice_rect(cfg, i)


if __name__ == "__main__":
    main()
