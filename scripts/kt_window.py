"""Mean duration of a kernel's last N launches in a rocprofv3 --kernel-trace CSV
(`*_kernel_trace.csv`): the bench's roofline pass is its last --roofline-steps
step launches, so `--last 64` prices the same launches as the bench line's
roofline.avg_launch_ms (bench.py's timed window carries no events).
  python scripts/kt_window.py gpurun_out/TAG/kt/kt_kernel_trace.csv --kernel k_step --last 64"""
import argparse
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--kernel", default="k_step")
ap.add_argument("--last", type=int, default=64)
ap.add_argument("--per-step", type=int, default=1, help="launches of the kernel per bench step (summed per step)")
a = ap.parse_args()
rows = [r for r in csv.DictReader(open(a.csv)) if a.kernel in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
all_mean = sum(d) / len(d)
tail = d[-a.last * a.per_step:]
per_step = [sum(tail[i:i + a.per_step]) for i in range(0, len(tail), a.per_step)]
print(json.dumps({"kernel": a.kernel, "launches": len(d), "mean_us_all_launches": round(all_mean, 2),
                  "last_steps": len(per_step), "mean_us_per_step_last": round(sum(per_step) / len(per_step), 2)}))
