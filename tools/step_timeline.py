"""Kernel classes of the last step in a rocprofv3 kernel trace: first start / last end / busy time
per class, relative to the step's unpack.  python tools/step_timeline.py gpurun_out/c4t/run_kernel_trace.csv"""
import collections
import csv
import sys

t = list(csv.DictReader(open(sys.argv[1])))
t.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(t) if r["Kernel_Name"].startswith("dbslmm_unpack")]
# a plan with a lead group unpacks in two launches per step (its slots first)
st = lambda i: int(t[i]["Start_Timestamp"])
first = idx[-2] if len(idx) > 1 and st(idx[-1]) - st(idx[-2]) < 5_000_000 else idx[-1]
last = t[first:]
t0 = int(last[0]["Start_Timestamp"])
agg = collections.OrderedDict()
for r in last:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    a = agg.setdefault(k, [s, e, 0.0, 0])
    a[0], a[1], a[2], a[3] = min(a[0], s), max(a[1], e), a[2] + e - s, a[3] + 1
for k, (s, e, b, n) in agg.items():
    print(f"{k:32s} n={n:5d} first={s:9.1f} last_end={e:9.1f} busy={b:9.1f} us")
