"""Per super step of the lead chain in a kernel trace (tools/trace_opts.sh): regions + panels (P),
the wait before the chain's near-trailing launch, near, and the bulk stream's far launch of the
previous step.  python tools/chain_steps.py gpurun_out/tr0/run_kernel_trace.csv"""
import collections
import csv
import sys

t = list(csv.DictReader(open(sys.argv[1])))
t.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(t) if r["Kernel_Name"].startswith("dbslmm_unpack")]
last = t[idx[-2]:]
t0 = int(last[0]["Start_Timestamp"])
by = collections.defaultdict(list)
for r in last:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
    by[r["Queue_Id"]].append((k, (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3))
# the lead chain = the queue whose first tiled kernel starts first
q_chain = min((q for q in by if any(k.startswith("dbslmm_tchol_region") for k, _, _ in by[q])),
              key=lambda q: min(s for k, s, _ in by[q] if k.startswith("dbslmm_tchol")))
chain = [x for x in by[q_chain] if x[0].startswith("dbslmm_tchol")]
print("chain queue", q_chain, "tchol kernels", len(chain), "end %.0f us" % max(e for _, _, e in chain))
for q, v in by.items():
    ks = collections.Counter(k for k, _, _ in v)
    print("  queue", q, dict(ks), "%.0f-%.0f" % (min(s for _, s, _ in v), max(e for _, _, e in v)))
step, acc, prev, t_step = 0, collections.Counter(), None, chain[0][1]
for k, s, e in chain:
    kind = k.split("_")[-1]
    if kind.startswith("trailing") and prev is not None and acc["panel"] > 0 and acc.get("cnt_p", 0) >= 0:
        pass
    if kind.startswith("trailing"):
        acc["trail_n"] += 1
        acc["trail"] += e - s
    else:
        if acc["trail_n"] and kind == "region" and acc["region_n"] == 0:
            pass
        acc[kind] += e - s
        acc[kind + "_n"] += 1
    acc["gap"] += max(0.0, s - prev) if prev is not None else 0.0
    prev = e
tot = {k: round(v) for k, v in acc.items()}
print("chain totals (us):", tot)
