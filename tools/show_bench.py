"""Prints value, ms/step and per-kernel ms of bench JSON lines (gpurun_out)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        j = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(f, "ERR", e)
        continue
    k = {n: round(v, 1) for n, v in j.get("kernel_ms_per_step", {}).items() if n != "launches"}
    print(f"{f:32s} {j['value']:9.1f} {j['ms_per_step']:7.1f} exact={j.get('bitexact_vs_oracle', {}).get('equal')} {k}")
