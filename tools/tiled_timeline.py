"""Timeline of the last tiled sequence in a rocprofv3 kernel trace: per launch kind, grid size,
duration, gap to the previous launch; plus totals per kind and the busy fraction of the stream.
    python tools/tiled_timeline.py gpurun_out/prof_c5/run_kernel_trace.csv [every]"""
import collections
import csv
import sys

path = sys.argv[1]
every = int(sys.argv[2]) if len(sys.argv) > 2 else 0
t = list(csv.DictReader(open(path)))
t.sort(key=lambda r: int(r["Start_Timestamp"]))
# last solve: from the last dbslmm_set_scalar
idx = [i for i, r in enumerate(t) if r["Kernel_Name"].startswith("dbslmm_set_scalar")]
last = [r for r in t[idx[-1]:] if "tchol" in r["Kernel_Name"]]
t0 = int(last[0]["Start_Timestamp"])
prev_end = t0
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
rows = []
for r in last:
    k = r["Kernel_Name"].split("(")[0].replace("dbslmm_tchol_", "")
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    wg = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
    gap = s - prev_end
    prev_end = max(prev_end, e)
    agg[k][0] += 1
    agg[k][1] += (e - s) / 1e3
    agg[k][2] += gap / 1e3
    rows.append((k, wg, (s - t0) / 1e3, (e - s) / 1e3, gap / 1e3))
span = (prev_end - t0) / 1e3
print(f"tiled sequence span {span:.1f} us, launches {len(last)}")
for k, (n, d, g) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {k:10s} n={n:5d} busy={d:9.1f} us  gaps-before={g:8.1f} us  avg={d / n:7.1f} us")
if every:
    for i, (k, wg, s, d, g) in enumerate(rows):
        if i % every == 0 or i > len(rows) - 12:
            print(f"{i:5d} {k:10s} wg={wg:6d} start={s:9.1f} dur={d:8.1f} gap={g:6.1f}")
