#!/usr/bin/env python3
"""Per-step kernel timeline from a rocprofv3 kernel_trace.csv (tools/gpu_timeline.sh)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = []
for r in rows:
    n = r["Kernel_Name"]
    for k in ("ffv1_symbols", "ffv1_layout", "ffv1_bits", "ffv1_walk", "ffv1_range", "ffv1_dseg", "ffv1_dfix",
              "ffv1_sink", "ffv1_assemble", "ffv1_delay"):
        if k in n:
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
ks.sort()
t0 = ks[0][0]
for s, e, k in ks[-40:]:
    print(f"{k:22s} {(s - t0) / 1e6:10.2f} {(e - t0) / 1e6:10.2f}  {(e - s) / 1e6:8.2f} ms")
