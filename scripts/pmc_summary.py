"""Summarise rocprofv3 PMC passes into per-kernel HBM bytes per launch.

  python scripts/pmc_summary.py gpurun_out/TAG profiles/TAG_pmc.json

Reads TAG/fetch/*_counter_collection.csv (FETCH_SIZE) and
TAG/write/*_counter_collection.csv (WRITE_SIZE), one pass each (they cannot
share a pass on gfx950).  Corrections from MI355X_MICROARCH.md "HBM":
rocprofv3 reports both counters in KiB; on gfx950 FETCH_SIZE counts exactly half
the bytes of wide (16 B/lane) coalesced streaming reads, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Kernels whose loads
are narrower than 16 B/lane are flagged "uncalibrated" (the doubling may not
apply to them).
"""
import collections
import csv
import glob
import json
import os
import sys

# kernels whose global loads are 16 B/lane (dwordx4) streaming reads
WIDE_LOAD_KERNELS = ("k_masks", "k_step", "k_reset", "k_sample")


def short(name):
    base = name.split("(")[0]
    return base.replace("void ", "").replace("mrts::", "")


def read(pattern, counter):
    out = collections.defaultdict(list)
    for f in glob.glob(pattern):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                out[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return out


def main(src, dst):
    fetch = read(os.path.join(src, "fetch", "*_counter_collection.csv"), "FETCH_SIZE")
    write = read(os.path.join(src, "write", "*_counter_collection.csv"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("k_"):
            continue
        f = sum(fetch[k]) / len(fetch[k]) if fetch.get(k) else None
        w = sum(write[k]) / len(write[k]) if write.get(k) else None
        wide = k.split("<")[0] in WIDE_LOAD_KERNELS   # k_sample_src: 4-B loads, uncalibrated
        fc = None if f is None else (2.0 * f if wide else f)
        res[k] = {"fetch_bytes_raw": f, "fetch_bytes": fc, "write_bytes": w,
                  "hbm_bytes": None if fc is None or w is None else fc + w,
                  "launches": len(fetch.get(k, [])), "fetch_correction": "x2 (gfx950, 16B/lane)" if wide else "uncalibrated"}
    json.dump(res, open(dst, "w"), indent=1)
    for k, v in res.items():
        print(k, {a: (round(b / 1e6, 2) if isinstance(b, float) else b) for a, b in v.items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
