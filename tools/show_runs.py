#!/usr/bin/env python3
"""Summary of a tools/gpu_run.sh output directory: each bench / serial line's
value, step time, checks and per-kernel HIP-event times.
Usage: python tools/show_runs.py gpurun_out/<tag>"""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.json")), key=lambda p: int("".join(c for c in os.path.basename(p) if c.isdigit()) or 0)):
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(os.path.basename(f), "unreadable", e)
        continue
    k = {a: round(b, 1) for a, b in j.get("kernel_ms_per_step", {}).items() if a != "launches"}
    ok = j.get("bitexact_vs_oracle", {}).get("equal")
    print(f"{os.path.basename(f):14s} {j['config'].get('workload', '')[:4]} frames/step={j['config'].get('frames_per_step', j.get('frames_per_step'))} "
          f"value={j['value']} ms={j['ms_per_step']} oracle={ok} {j.get('env', '')}")
    print("   ", k)
