"""Summarise the two rocprofv3 PMC passes of tools/gpu_pmc.sh into per-kernel HBM bytes per launch.

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  gfx950 correction (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE counts 64 B per 128-B request of a wide coalesced read, so it is doubled; WRITE_SIZE is exact for
16-B-per-lane stores.  traffic = 2 * FETCH_SIZE + WRITE_SIZE.
usage: python tools/pmc_traffic.py <gpurun_out dir> <out.json> [bench --config, default 4]"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:  # the build TUs' kernels sit in an anonymous namespace
            acc[r["Kernel_Name"].replace("(anonymous namespace)::", "")].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    out = sys.argv[2] if len(sys.argv) > 2 else None
    fetch, nf = per_kernel(f"{d}/pmc_fetch/pmc_counter_collection.csv", "FETCH_SIZE")
    write, nw = per_kernel(f"{d}/pmc_write/pmc_counter_collection.csv", "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith(("kb::", "void kb::", "ksp::", "void ksp::")):
            continue
        f_kib, w_kib = fetch.get(k, 0.0), write.get(k, 0.0)
        res[k] = {"dispatches": [nf.get(k, 0), nw.get(k, 0)], "FETCH_SIZE_KiB": f_kib, "WRITE_SIZE_KiB": w_kib,
                  "hbm_bytes_per_launch": (2.0 * f_kib + w_kib) * 1024.0}
    cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    names = {2: "configs[1] (2-cam pinhole-radtan, 500 frames)", 3: "configs[2] (4-cam omni-radtan + EUCM, 1000 frames)",
             4: "configs[3] (8-cam pinhole-radtan, 2000 frames)", 5: "configs[4] (2-cam + IMU B-spline, 1200 frames)"}
    doc = {"workload": f"bench.py --config {cfg}: {names[cfg]}, N=1", "bench_config": cfg,
           "correction": "traffic = 2*FETCH_SIZE + WRITE_SIZE (KiB), gfx950 FETCH_SIZE halves 16-B/lane reads",
           "kernels": res}
    s = json.dumps(doc, indent=1)
    if out:
        open(out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
