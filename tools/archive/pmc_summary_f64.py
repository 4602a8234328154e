"""Summarise the PMC passes of tools/pmc_f64.sh (gpurun_out/pmc64/<pass>/run_counter_collection.csv) for
the FP64 fused kernel; write the per-launch traffic JSON bench.py reads.

Derived numbers (MI355X_MICROARCH.md):
  * effective clock = GRBM_GUI_ACTIVE / 8 / dispatch time (GRBM sums the 8 XCDs);
  * MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8);
  * HBM-side traffic = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half of a wide streaming
    read); the K=1 passes (calibration: y in + h out, the tables negligible) check that factor on this
    kernel's own y-load / h-store pattern against the known byte count 32 N B.
"""
import csv
import json
import os
import sys

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc64"
pat = sys.argv[2] if len(sys.argv) > 2 else "k_est_all_f64"
B, N = 100000, 64


def load(name):
    f = os.path.join(base, name, "run_counter_collection.csv")
    out, dur = {}, []
    if not os.path.exists(f):
        return out, dur
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return {k: sum(v) / len(v) for k, v in out.items()}, dur


res = {}
for p in ("sq", "fetch", "write", "lds", "tcc", "cfetch", "cwrite"):
    v, d = load(p)
    res[p] = (v, d)
    for k, x in sorted(v.items()):
        print(f"[{p:6s}] {k:28s} {x:.6g}")
sq, dsq = res["sq"]
if sq:
    t = sum(dsq) / len(dsq)
    clk = sq["GRBM_GUI_ACTIVE"] / 8 / t
    busy = sq["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * sq["GRBM_GUI_ACTIVE"] / 8)
    print(f"dispatch {t * 1e3:.3f} ms, effective clock {clk / 1e9:.3f} GHz, MFMA busy {busy:.3f}")
    print(f"wave time split: wait {sq['SQ_WAIT_ANY'] / sq['SQ_WAVE_CYCLES']:.3f}, issue-stall "
          f"{sq['SQ_WAIT_INST_ANY'] / sq['SQ_WAVE_CYCLES']:.3f}, active {sq['SQ_ACTIVE_INST_ANY'] / sq['SQ_WAVE_CYCLES']:.3f}")
f, w = res["fetch"][0].get("FETCH_SIZE"), res["write"][0].get("WRITE_SIZE")
cf, cw = res["cfetch"][0].get("FETCH_SIZE"), res["cwrite"][0].get("WRITE_SIZE")
if f and w:
    hbm = (2 * f + w) * 1024
    print(f"metric launch: FETCH {f * 1024 / 1e6:.1f} MB (x2 = {2 * f * 1024 / 1e6:.1f}), WRITE {w * 1024 / 1e6:.1f} MB, "
          f"traffic {hbm / 1e6:.1f} MB vs algorithmic y+h {32 * N * B / 1e6:.1f} MB")
    cal = None
    if cf and cw:
        cal = dict(read_ratio=2 * cf * 1024 / (16 * N * B), write_ratio=cw * 1024 / (16 * N * B))
        print(f"K=1 calibration: 2*FETCH / y bytes = {cal['read_ratio']:.3f}, WRITE / h bytes = {cal['write_ratio']:.3f}")
    if len(sys.argv) > 3:
        json.dump({"config": "metric", "B": B, "kernel": "f64", "hbm_bytes_per_launch": hbm, "fetch_size_kb": f,
                   "write_size_kb": w, "calibration_k1": cal,
                   "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, FETCH doubled (gfx950); "
                           "K=1 passes calibrate the y-load / h-store pattern"},
                  open(sys.argv[3], "w"), indent=1)
tcc = res["tcc"][0]
if tcc:
    h, m = tcc["TCC_HIT_sum"], tcc["TCC_MISS_sum"]
    print(f"L2 hit rate {h / (h + m):.3f}")
lds = res["lds"][0]
if lds:
    print(f"LDS bank conflicts / LDS active {lds['SQ_LDS_BANK_CONFLICT'] / max(lds['SQ_LDS_IDX_ACTIVE'], 1):.4f}")
