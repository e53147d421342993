#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/profile.sh <tag> pmc ...) into
per-kernel means, and write the HBM traffic of the count kernel K1a for
bench.py's roofline.traffic.

    python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<round>

FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 derived counters).  On gfx950
FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads
(/opt/skills/guides/MI355X_MICROARCH.md, HBM section), which is how K1a reads
its input, so hbm_bytes = 2 * FETCH + WRITE.  WRITE_SIZE is exact for the
16-B-per-lane stores K1a issues.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

COUNT_KERNEL = "k_part<true"  # K1a, canonical (any bucket capacity)


def main(src, dst):
    sums = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(int))
    dur = defaultdict(lambda: defaultdict(float))  # ns per dispatch, per counter pass
    for path in sorted(glob.glob(os.path.join(src, "pmc*", "*counter_collection.csv"))):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"]
                c = r["Counter_Name"]
                sums[k][c] += float(r["Counter_Value"])
                calls[k][c] += 1
                dur[k][c] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    means = {k: {c: sums[k][c] / calls[k][c] for c in sums[k]} for k in sums}
    os.makedirs(dst, exist_ok=True)
    with open(os.path.join(dst, "pmc_per_kernel_mean.json"), "w") as f:
        json.dump(means, f, indent=1, sort_keys=True)
    name = next((k for k in means if COUNT_KERNEL in k.replace(" ", "")), None)
    if name is None:
        print("count kernel not found in", src)
        return 1
    m = means[name]
    if "FETCH_SIZE" not in m or "WRITE_SIZE" not in m:
        print("no FETCH_SIZE / WRITE_SIZE in this pass (per-kernel means only):", sorted(m))
        return 0
    fetch = m["FETCH_SIZE"] * 1024.0
    write = m["WRITE_SIZE"] * 1024.0
    valu = {}
    if "SQ_INSTS_VALU" in m and "GRBM_GUI_ACTIVE" in m:
        # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles: per XCD / duration = SCLK
        ns = dur[name]["GRBM_GUI_ACTIVE"] / calls[name]["GRBM_GUI_ACTIVE"]
        valu = {
            "valu_instr_per_launch": m["SQ_INSTS_VALU"],
            "sclk_ghz": m["GRBM_GUI_ACTIVE"] / 8.0 / ns,
            "pmc_launch_ns": ns,
        }
    out = {
        "kernel": name,
        "fetch_size_bytes_raw": fetch,
        "write_size_bytes": write,
        "hbm_bytes_per_launch": 2.0 * fetch + write,
        "correction": "gfx950: FETCH_SIZE x2 for 16-B/lane streaming reads (MI355X_MICROARCH.md HBM)",
        **valu,
        "source": os.path.relpath(os.path.join(dst, "pmc_per_kernel_mean.json"),
                                  os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
    }
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "profiles", "pmc_count_kernel.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2]))
