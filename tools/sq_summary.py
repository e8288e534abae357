#!/usr/bin/env python3
"""Per-kernel SQ counter summary of tools/prof_sq.sh output (one dispatch
average per kernel).  Cycle counters are quad-cycles (MI355X_MICROARCH.md)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("ffv1hip::", "").split("(")[0]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    return acc, n


def main(d):
    a1, n1 = load(os.path.join(d, "p1"))
    a2, _ = load(os.path.join(d, "p2"))
    for k in sorted(a1, key=lambda k: -a1[k].get("SQ_WAVE_CYCLES", 0)):
        c = dict(a1[k], **a2.get(k, {}))
        w = c.get("SQ_WAVES", 0) or 1
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        per = lambda x: c.get(x, 0) / w
        print(f"{k[:34]:34s} disp {len(n1[k]):3d} waves/disp {w / max(len(n1[k]), 1):8.0f} "
              f"cyc/wave {4 * wc / w:10.0f} wait {c.get('SQ_WAIT_ANY', 0) / wc:5.2f} "
              f"stall {c.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} issue {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f} | "
              f"per wave: valu {per('SQ_INSTS_VALU'):9.0f} salu {per('SQ_INSTS_SALU'):8.0f} "
              f"vmem r/w {per('SQ_INSTS_VMEM_RD'):7.0f}/{per('SQ_INSTS_VMEM_WR'):7.0f} lds {per('SQ_INSTS_LDS'):8.0f} "
              f"ldsconf {c.get('SQ_LDS_BANK_CONFLICT', 0) / max(c.get('SQ_ACTIVE_INST_LDS', 1), 1):.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
