"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE counter CSVs into per-kernel HBM bytes per launch.

FETCH_SIZE and WRITE_SIZE are in KB.  On gfx950 FETCH_SIZE reports half of the bytes of a wide
coalesced streaming read (MI355X_MICROARCH.md, HBM section): the read side is doubled here.
    python tools/pmc_traffic.py gpurun_out/pmc profiles/r01/pmc_traffic_c4.json [bench args]

Also records launches per kernel and, for the composite phases the bench times as one slot --
the tiled Cholesky (dbslmm_tchol_* launches plus the persistent backward substitution
dbslmm_trsv_bwd<1>) and the h2f substitutions (dbslmm_trsv_fwd/bwd<2>) -- the summed
HBM bytes per run (= per bench step; runs = launches of dbslmm_pcg_init on the PCG route, else of
dbslmm_gram_i8, one per run -- the unpack is two launches per run with a lead group) under
"dbslmm_tchol" and "dbslmm_trsv", and likewise the Gram launches under "dbslmm_gram" and the
chip-wide PCG launches under "dbslmm_pcg" (key "hbm_bytes_per_step").
"""
import collections
import csv
import json
import os
import sys


def per_kernel(path):
    agg = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        # one row per (dispatch, counter instance) -> sum the instances of a dispatch
        d = agg[r["Kernel_Name"]]
        d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in agg.items()}


def main(src, dst, bench_args=""):
    f = per_kernel(os.path.join(src, "fetch_counter_collection.csv"))
    w = per_kernel(os.path.join(src, "write_counter_collection.csv"))
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over "
                     f"`python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline {bench_args}`".rstrip(),
           "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch",
           "kernels": {}}
    # runs: one dbslmm_pcg_init per run on the PCG route, else one dbslmm_gram_i8
    runs = f.get("dbslmm_pcg_init", (0, 0))[1] or f.get("dbslmm_gram_i8", (0, 0))[1]
    seq = trsv = gram = pcg = 0.0
    for k in sorted(set(f) | set(w)):
        name = k[5:] if k.startswith("void ") else k
        if not name.startswith("dbslmm_"):
            continue
        (fk, n), (wk, _) = f.get(k, (0.0, 0)), w.get(k, (0.0, 0))
        out["kernels"][name] = dict(fetch_kb=fk, write_kb=wk, hbm_bytes=(2 * fk + wk) * 1024.0, launches=n)
        if name.startswith("dbslmm_tchol_") or name.startswith("dbslmm_trsv_bwd<1>"):
            seq += (2 * fk + wk) * 1024.0 * n
        elif name.startswith("dbslmm_trsv_"):
            trsv += (2 * fk + wk) * 1024.0 * n
        if name.startswith("dbslmm_gram_"):
            gram += (2 * fk + wk) * 1024.0 * n
        elif name.startswith("dbslmm_pcg_") and name != "dbslmm_pcg_block":
            pcg += (2 * fk + wk) * 1024.0 * n
    if runs and seq:
        out["kernels"]["dbslmm_tchol"] = dict(hbm_bytes_per_step=seq / runs, runs=runs,
                                              note="dbslmm_tchol_* + persistent backward, per run")
    if runs and trsv:
        out["kernels"]["dbslmm_trsv"] = dict(hbm_bytes_per_step=trsv / runs, runs=runs,
                                             note="h2f substitutions (CG by default), per run")
    if runs and gram:
        out["kernels"]["dbslmm_gram"] = dict(hbm_bytes_per_step=gram / runs, runs=runs,
                                             note="dbslmm_gram_huge / _big / _i8 launches, per run")
    if runs and pcg:
        out["kernels"]["dbslmm_pcg"] = dict(hbm_bytes_per_step=pcg / runs, runs=runs,
                                            note="chip-wide PCG launches (init, symv, rows, update, final), per run")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], " ".join(sys.argv[3:]))
