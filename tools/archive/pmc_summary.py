"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/*) for one kernel; optionally write the
per-launch HBM traffic JSON bench.py reads (FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM)."""
import csv, glob, json, os, sys
from collections import defaultdict

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
pat = sys.argv[2] if len(sys.argv) > 2 else "k_est_all_h2"
vals = defaultdict(list)
dur = []
for f in glob.glob(os.path.join(base, "*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "FETCH_SIZE":
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
for k, v in sorted(vals.items()):
    print(f"{k:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
    fetch_kb = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
    write_kb = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
    hbm = (2 * fetch_kb + write_kb) * 1024  # gfx950: FETCH_SIZE reports half of a wide streaming read
    print(f"HBM bytes/launch (2*FETCH+WRITE) = {hbm/1e6:.1f} MB; raw FETCH {fetch_kb*1024/1e6:.1f} MB WRITE {write_kb*1024/1e6:.1f} MB")
    if len(sys.argv) > 3:
        json.dump({"config": sys.argv[3], "B": int(sys.argv[4]), "kernel": sys.argv[5], "hbm_bytes_per_launch": hbm,
                   "fetch_size_kb": fetch_kb, "write_size_kb": write_kb,
                   "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, FETCH doubled (gfx950)"},
                  open(sys.argv[6], "w"), indent=1)
if "TCC_HIT_sum" in vals:
    h, m = sum(vals["TCC_HIT_sum"]), sum(vals["TCC_MISS_sum"])
    print(f"L2 hit rate {h/(h+m):.3f}")
if "SQ_VALU_MFMA_BUSY_CYCLES" in vals and "GRBM_GUI_ACTIVE" in vals:
    busy = sum(vals["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(vals["SQ_VALU_MFMA_BUSY_CYCLES"])
    gui = sum(vals["GRBM_GUI_ACTIVE"]) / len(vals["GRBM_GUI_ACTIVE"])
    print(f"MFMA busy per SIMD ~ {busy/(256*4)/ (gui/8):.3f} (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * GRBM_GUI_ACTIVE/8))")
