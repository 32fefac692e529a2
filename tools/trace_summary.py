"""Summarise the last plan_run in a rocprofv3 kernel trace: per-kernel totals + tiled timeline."""
import collections
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_c3/run_kernel_trace.csv"
show = int(sys.argv[2]) if len(sys.argv) > 2 else 12
t = list(csv.DictReader(open(path)))
idx = [i for i, r in enumerate(t) if r["Kernel_Name"].startswith("dbslmm_unpack")]
last = t[idx[-1]:]
t0 = int(last[0]["Start_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0])
for r in last:
    n = r["Kernel_Name"].split("(")[0]
    agg[n][0] += 1
    agg[n][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, v in agg.items():
    print(f"{k:34s} n={v[0]:4d} total={v[1] / 1e3:9.1f} us avg={v[1] / v[0] / 1e3:8.1f} us")
tc = [r for r in last if "tchol" in r["Kernel_Name"]]
for r in tc[:show] + tc[-show:]:
    s = int(r["Start_Timestamp"]) - t0
    e = int(r["End_Timestamp"]) - t0
    print(f"{r['Kernel_Name'].split('(')[0][13:]:10s} wg={int(r['Grid_Size_X']) // 256:6d} "
          f"start={s / 1e3:9.1f} dur={(e - s) / 1e3:7.1f} q={r['Queue_Id']}")
print("run span us", (max(int(r["End_Timestamp"]) for r in last) - t0) / 1e3)
