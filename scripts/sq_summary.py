"""Per-kernel means of rocprofv3 --pmc counters over every launch, from one or more
pass directories (each SRC/<pass>/*_counter_collection.csv), plus derived figures
for the step kernel: mean resident waves (SQ_WAVE_CYCLES / SQ_BUSY_CYCLES, both in
the same cycle unit), the fraction of wave time spent waiting (SQ_WAIT_ANY /
SQ_WAVE_CYCLES) and LDS bank conflicts per LDS instruction.

  python scripts/sq_summary.py gpurun_out/TAG/sq profiles/TAG_sq.json "bench command"
"""
import collections
import csv
import glob
import json
import os
import sys


def main(src, dst, command=""):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, "*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mrts::", "")
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"source": f"rocprofv3 --pmc, separate passes, per-launch means: {command}", "kernels": {}}
    for k, cs in sorted(acc.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {}
        if m.get("SQ_BUSY_CYCLES") and m.get("SQ_WAVE_CYCLES"):
            d["mean_resident_waves_per_busy_cycle"] = m["SQ_WAVE_CYCLES"] / m["SQ_BUSY_CYCLES"]
        if m.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in m:
            d["wait_any_frac_of_wave_cycles"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
        if m.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in m:
            d["lds_bank_conflict_cycles_per_lds_inst"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_INSTS_LDS"]
        if m.get("SQ_WAVES") and "SQ_INSTS_VMEM_WR" in m:
            d["vmem_store_insts_per_wave"] = m["SQ_INSTS_VMEM_WR"] / m["SQ_WAVES"]
        out["kernels"][k] = {"counters": m, "derived": d, "launches": max(len(v) for v in cs.values())}
    json.dump(out, open(dst, "w"), indent=1)
    for k, v in out["kernels"].items():
        if k.startswith("k_step"):
            print(k, {a: round(b, 3) for a, b in v["derived"].items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
