"""Per-stream phase timeline of the last step in a rocprofv3 kernel trace: for every (stream,
kernel) pair its first start, last end (ms from its unpack), launch count and busy
time -- where each group's factorisation and substitutions begin and end in the step.
    python tools/step_timeline.py gpurun_out/c4t/run_kernel_trace.csv"""
import collections
import csv
import sys

t = list(csv.DictReader(open(sys.argv[1])))
t.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last step starts at its unpack; a plan with a lead group unpacks in two launches per step
# (its slots first)
idx = [i for i, r in enumerate(t) if r["Kernel_Name"].startswith("dbslmm_unpack")]
st = lambda i: int(t[i]["Start_Timestamp"])
first = idx[-2] if len(idx) > 1 and st(idx[-1]) - st(idx[-2]) < 5_000_000 else idx[-1]
name = lambda r: r["Kernel_Name"].replace("void ", "").split("(")[0]
run = [r for r in t[first:] if name(r).startswith("dbslmm_")]
t0 = int(run[0]["Start_Timestamp"])
g = collections.OrderedDict()
for r in run:
    key = (r["Stream_Id"], name(r).replace("dbslmm_", ""))
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
    if key not in g:
        g[key] = [s, e, 0, 0.0]
    v = g[key]
    v[0], v[1], v[2], v[3] = min(v[0], s), max(v[1], e), v[2] + 1, v[3] + e - s
end = max(v[1] for v in g.values())
print(f"step span {end:.2f} ms ({len(run)} launches)")
print(f"{'stream':>6s} {'kernel':24s} {'first':>8s} {'last end':>8s} {'n':>5s} {'busy ms':>8s}")
for (st, k), (s, e, n, b) in sorted(g.items(), key=lambda x: (x[1][0], x[0][0])):
    print(f"{st:>6s} {k:24s} {s:8.2f} {e:8.2f} {n:5d} {b:8.2f}")
