"""Summarise rocprofv3 PMC passes into per-kernel HBM bytes per launch.

  python scripts/pmc_summary.py gpurun_out/TAG/pmc_selfplay profiles/pmc_latest.json \
      --workload selfplay@8192 [--lib microrts-py_amd/gym_microrts/libmicrorts_amd.so]

Reads SRC/fetch/*_counter_collection.csv (FETCH_SIZE) and
SRC/write/*_counter_collection.csv (WRITE_SIZE), one pass each (they cannot
share a pass on gfx950).  Corrections from MI355X_MICROARCH.md "HBM":
rocprofv3 reports both counters in KiB; on gfx950 FETCH_SIZE counts exactly half
the bytes of wide (16 B/lane) coalesced streaming reads, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Kernels whose loads
are narrower than 16 B/lane are flagged "uncalibrated" (the doubling may not
apply to them).

The summary is stamped with the sha256 of the library the passes ran
(`_meta.lib_sha256`) and filed under the bench workload it measured
(`workloads[<workload>@<envs>]`); entries for other workloads of the same build
are kept, a different build starts the file afresh.  bench.py reports
`roofline.traffic` only when the stamp matches the library it runs.
"""
import argparse
import collections
import csv
import glob
import hashlib
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "microrts-py_amd", "gym_microrts", "libmicrorts_amd.so")

# kernels whose global loads are 16 B/lane (dwordx4) streaming reads
WIDE_LOAD_KERNELS = ("k_masks", "k_step", "k_reset", "k_sample")


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


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


def summarise(src):
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
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--workload", required=True, help="bench workload key, <workload>@<envs per gpu>")
    ap.add_argument("--lib", default=LIB)
    ap.add_argument("--command", default="")
    a = ap.parse_args()
    res = summarise(a.src)
    digest = sha256(a.lib)
    doc = {}
    if os.path.exists(a.dst):
        try:
            doc = json.load(open(a.dst))
        except ValueError:
            doc = {}
    if doc.get("_meta", {}).get("lib_sha256") != digest:
        doc = {}
    doc.setdefault("_meta", {"lib_sha256": digest, "lib": os.path.relpath(a.lib, REPO),
                             "counters": "FETCH_SIZE x2 (gfx950 16 B/lane) + WRITE_SIZE, KiB -> bytes, separate passes"})
    doc.setdefault("workloads", {})[a.workload] = {"command": a.command, "kernels": res}
    json.dump(doc, open(a.dst, "w"), indent=1)
    for k, v in res.items():
        print(a.workload, k, {x: (round(y / 1e6, 2) if isinstance(y, float) else y) for x, y in v.items()})


if __name__ == "__main__":
    main()
