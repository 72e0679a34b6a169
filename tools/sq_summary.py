"""Per-kernel averages of the rocprofv3 SQ counter passes (pmc_sq1, pmc_sq2 under a gpurun_out dir) -> JSON.
usage: python tools/sq_summary.py <dir> <out.json> <workload text>"""
import csv
import json
import sys
from collections import defaultdict

d, out, wl = sys.argv[1], sys.argv[2], sys.argv[3]
acc = defaultdict(lambda: defaultdict(list))
for sub in ("pmc_sq1", "pmc_sq2", "pmc_sq3"):
    try:
        rows = csv.DictReader(open(f"{d}/{sub}/pmc_counter_collection.csv"))
    except OSError:
        continue
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")  # the build TUs' kernels
        if name.startswith(("kb::", "void kb::")):
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
json.dump({"workload": wl, "note": "per-dispatch averages; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* in quad-cycles, "
           "SQ_VALU_MFMA_BUSY_CYCLES in cycles", "kernels": res}, open(out, "w"), indent=1)
