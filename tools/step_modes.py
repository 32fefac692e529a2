"""Per-step timelines of a multi-step kernel trace (diagnostic, round 4): for every step (two
unpack launches each: lead slots, then the rest) the step length and the start / end of the
unpack, Gram, lead-chain and substitution launches, to tell the slow mode (unpack span ~2.7 ms,
Gram span ~12.8 ms) from the usual one.  python tools/step_modes.py run_kernel_trace.csv"""
import csv
import sys

t = list(csv.DictReader(open(sys.argv[1])))
t.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(t) if r["Kernel_Name"].startswith("dbslmm_unpack")][::2]
for n, i0 in enumerate(starts):
    i1 = starts[n + 1] if n + 1 < len(starts) else len(t)
    seg = t[i0:i1]
    t0 = int(seg[0]["Start_Timestamp"])
    def span(pfx, q=None):
        v = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0) for r in seg
             if r["Kernel_Name"].replace("void ", "").startswith(pfx) and (q is None or r["Queue_Id"] == q)]
        return (min(a for a, _ in v) / 1e6, max(b for _, b in v) / 1e6) if v else (0, 0)
    un = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Queue_Id"]) for r in seg
          if r["Kernel_Name"].startswith("dbslmm_unpack")]
    gh = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Queue_Id"]) for r in seg
          if r["Kernel_Name"].startswith("dbslmm_gram_huge")]
    end = max(int(r["End_Timestamp"]) for r in seg) - t0
    print(f"step {n:2d} len {end / 1e6:6.2f} ms  unpack {[(round(a / 1e6, 2), round(b / 1e6, 2), q) for a, b, q in un]}"
          f"  gram_huge {[(round(a / 1e6, 2), round(b / 1e6, 2), q) for a, b, q in gh]}"
          f"  region {span('dbslmm_tchol_region')}  trsv {span('dbslmm_trsv')}")
