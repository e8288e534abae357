#!/usr/bin/env python3
"""Per-kernel sums of SQ counters from tools/walk_pmc.sh output dirs."""
import csv, sys
from collections import defaultdict
NAMES = ("ffv1_walk", "ffv1_dcode", "ffv1_code_golomb", "ffv1_code", "ffv1_symbols", "ffv1_layout", "ffv1_assemble")
for path in sys.argv[1:]:
    d = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(path)):
        k = next((n for n in NAMES if n in r["Kernel_Name"]), r["Kernel_Name"][:30])
        d[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in d.items():
        if k in ("ffv1_walk", "ffv1_dcode"):
            print(k, " ".join(f"{a}={b:.3g}" for a, b in sorted(v.items())))
