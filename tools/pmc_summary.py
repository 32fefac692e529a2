"""Aggregate rocprofv3 --pmc csv passes (gpurun_out/pmc_c<N>/p*_counter_collection.csv) per kernel."""
import collections
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_c5"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in sorted(glob.glob(f"{d}/p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((f, r["Dispatch_Id"]))
for k, v in agg.items():
    if not k.startswith("dbslmm"):
        continue
    line = f"{k:26s}"
    g = v.get("GRBM_GUI_ACTIVE", 0) / 8
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in v:
        line += f" mfma_busy/SIMD={v['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / g:6.1%}"
    if "SQ_WAVE_CYCLES" in v and v["SQ_WAVE_CYCLES"]:
        line += f" wait={v['SQ_WAIT_INST_ANY'] / v['SQ_WAVE_CYCLES']:5.1%}"
    h, mi = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
    if h + mi:
        line += f" L2hit={h / (h + mi):5.1%}"
    if "FETCH_SIZE" in v:
        line += f" fetch={2 * v['FETCH_SIZE'] / 1e6:7.2f}GB"
    if v.get("SQ_LDS_IDX_ACTIVE"):
        line += f" lds_conflict={v['SQ_LDS_BANK_CONFLICT'] / v['SQ_LDS_IDX_ACTIVE']:5.1%}"
    if g:
        line += f" gui_cycles/XCD={g:.3g}"
    print(line)
