"""Per-kernel launch statistics from a rocprofv3 --kernel-trace database (rocpd
sqlite, the default output format): one line per (kernel, grid, workgroup, LDS)
with launches, mean / median / min duration in microseconds.  Optional --skip N
drops each group's first N launches (pre-roll / warmup).
  python scripts/kt_summary.py gpurun_out/X/prof/*_results.db [--skip N] [--json out.json]"""
import argparse
import collections
import json
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--skip", type=int, default=0)
ap.add_argument("--last", type=int, default=0, help="keep only each group's last N launches")
ap.add_argument("--json", default=None)
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = c.execute("select name, grid_x, workgroup_x, lds_size, vgpr_count, sgpr_count, start, end from kernels order by start").fetchall()
d = collections.defaultdict(list)
meta = {}
for n, g, w, lds, vg, sg, s, e in rows:
    k = (n.split("(")[0][:90], g // max(w, 1), w, lds)
    d[k].append((e - s) / 1e3)
    meta[k] = (vg, sg)
out = []
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v = v[a.skip:]
    if a.last:
        v = v[-a.last:]
    if not v:
        continue
    sv = sorted(v)
    r = {"kernel": k[0], "workgroups": k[1], "workgroup_size": k[2], "lds": k[3], "vgpr": meta[k][0], "sgpr": meta[k][1],
         "launches": len(v), "mean_us": round(sum(v) / len(v), 2), "median_us": round(sv[len(v) // 2], 2), "min_us": round(sv[0], 2)}
    out.append(r)
    print(f"{r['kernel'][:70]:70s} wg {r['workgroups']:6d}x{r['workgroup_size']:4d} lds {r['lds']:6d} n {r['launches']:5d} "
          f"mean {r['mean_us']:8.2f} med {r['median_us']:8.2f} min {r['min_us']:8.2f}")
if a.json:
    json.dump(out, open(a.json, "w"), indent=1)
