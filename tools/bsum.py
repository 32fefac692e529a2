"""One-line summaries of bench JSON files (round-6 A/B helper): value, ms/step, phase spans."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads([l for l in open(f).read().splitlines() if l.startswith("{")][-1])
    except Exception as e:   # noqa: BLE001
        print(f, "ERR", e)
        continue
    ks = " ".join("%s=%.3f" % (k["kernel"].replace("dbslmm_", ""), k["ms"]) for k in d["kernels"] if k["ms"] > 0)
    extra = ""
    for k in d["kernels"]:
        if k["kernel"] == "dbslmm_pcg" and k["ms"] > 0:
            extra = " pcg_it=%d pcg_frac=%.3f" % (k.get("iterations", 0), k["frac"])
    print("%-40s %.4g SNPs/s  %.3f ms/step  %s%s  st=%d" % (f, d["value"], d["ms_per_step"], ks, extra,
                                                            d.get("status_nonzero_blocks", -1)))
