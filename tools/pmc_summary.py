#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run into profiles/.

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats
summary, copied) and profiles/pmc_traffic_rNN.json: per-kernel HBM bytes per
launch from the FETCH_SIZE / WRITE_SIZE passes.  FETCH_SIZE and WRITE_SIZE
are reported by rocprofv3 in KiB; per MI355X_MICROARCH.md (HBM section)
gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads, so it is
doubled; WRITE_SIZE is taken as is.
"""
import csv, json, os, shutil, statistics, sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    for k in ("ffv1_decode_slices", "ffv1_code_golomb", "ffv1_dcode", "ffv1_code", "ffv1_walk", "ffv1_bits", "ffv1_layout", "ffv1_symbols",
              "ffv1_sink", "ffv1_assemble_packets", "ffv1_range_dseg", "ffv1_range", "ffv1_dseg", "ffv1_dfix", "ffv1_compact_packets",
              "ffv1_sizes_out", "ffv1_ints_out", "ffv1_delay"):
        if k in name:
            return k
    return name


def per_kernel(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return {k: statistics.mean(v) for k, v in vals.items()}


def main(tag, frames_per_launch, config, out_name="pmc_traffic_rNN.json", data="d1"):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    fetch = per_kernel(os.path.join(src, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "write", "write_counter_collection.csv"), "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("ffv1_"):
            continue
        f2 = 2.0 * fetch.get(k, 0.0)
        w = write.get(k, 0.0)
        kernels[k] = {"fetch_bytes_x2": int(f2), "write_bytes": int(w), "hbm_bytes": int(f2 + w)}
    stats, calls = {}, {}
    for r in csv.DictReader(open(os.path.join(dst, f"{tag}_kernel_stats.csv"))):
        stats[short(r["Name"])] = float(r["AverageNs"]) / 1e6
        calls[short(r["Name"])] = int(r["Calls"])
    # launches per step: the split schedule launches the walk in two parts
    # (the range pass: one launch of ffv1_range and one of ffv1_range_dseg)
    per_step = calls.get("ffv1_range", calls.get("ffv1_dcode", 0))
    for k, v in kernels.items():
        n = max(1, round(calls.get(k, per_step) / per_step)) if per_step else 1
        v["launches_per_step"] = n
        v["hbm_bytes_per_step"] = v["hbm_bytes"] * n
    out = {
        "tag": tag, "config": config, "data": data, "frames_per_launch": frames_per_launch,
        "note": "per-launch means over the profiled bench run; FETCH_SIZE doubled (gfx950), WRITE_SIZE as is",
        "kernels": kernels,
        "rocprof_avg_ms": stats,
        "frames_per_step": frames_per_launch,
        "encode_hbm_bytes_per_step": sum(v["hbm_bytes_per_step"] for k, v in kernels.items()
                                         if k != "ffv1_decode_slices"),
    }
    json.dump(out, open(os.path.join(dst, out_name), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01", int(sys.argv[2]) if len(sys.argv) > 2 else 252,
         sys.argv[3] if len(sys.argv) > 3 else "3840x2160 yuv420p10",
         sys.argv[4] if len(sys.argv) > 4 else "pmc_traffic_rNN.json",
         sys.argv[5] if len(sys.argv) > 5 else "d1")
