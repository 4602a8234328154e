"""Summary of tools/pmc_kernel.sh's passes (<out>/<pass>/run_counter_collection.csv) for one kernel, and the
traffic JSON bench.py reads (<out>/traffic_<cfg>.json, stamped with the library's build id).

Derived numbers (MI355X_MICROARCH.md):
  * cycle base = GRBM_GUI_ACTIVE / 8 of the kernel's own dispatches (GRBM sums the 8 XCDs), checked against the
    dispatch's wall time: the effective clock must be <= 2.4 GHz (it reads high on dispatches < ~0.3 ms -- then
    the cycle ratios are flagged unreliable; rerun with a larger BCYC);
  * MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycle base);
  * HBM-side traffic = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half of a wide streaming read),
    per launch at the config's B; optional K=1 calibration passes check that factor on the kernel's y / h pattern.
usage: pmc_report.py OUT KPAT CFG BUILD_ID [TRAFFIC_NAME]   (default traffic_<CFG>; traffic_<CFG>_mean for --mean runs)
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
base, pat, cfg, bid = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
tname = sys.argv[5] if len(sys.argv) > 5 and sys.argv[5] else f"traffic_{cfg}"
import bench  # noqa: E402

C = bench.CONFIGS[cfg]
B, N = C["B"], C["N"]


def load(name):
    f = os.path.join(base, name, "run_counter_collection.csv")
    out, dur = {}, {}
    if not os.path.exists(f):
        return {}, 0.0
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        dur[r.get("Dispatch_Id", len(dur))] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    t = sum(dur.values()) / max(len(dur), 1)
    return {k: sum(v) / len(v) for k, v in out.items()}, t


res = {p: load(p) for p in ("sq", "inst", "lds", "fetch", "write", "tcc", "dram", "cfetch", "cwrite", "cdram")}
print(f"kernel pattern {pat!r}, config {cfg} (B={B}, N={N}), library build {bid}")
for p, (v, t) in res.items():
    for k, x in sorted(v.items()):
        print(f"[{p:6s}] {k:28s} {x:.6g}")
sq, tsq = res["sq"]
if sq:
    cyc = sq["GRBM_GUI_ACTIVE"] / 8
    clk = cyc / tsq
    ok = clk <= 2.45e9 and tsq >= 3e-4
    print(f"sq pass: dispatch {tsq * 1e3:.4f} ms, cycle base {cyc:.4g}, effective clock {clk / 1e9:.3f} GHz"
          + ("" if ok else "  ** UNRELIABLE cycle base (dispatch < 0.3 ms or clock > 2.4 GHz): rerun with larger BCYC"))
    print(f"MFMA busy {sq['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * cyc):.3f}; mean resident waves per SIMD "
          f"{sq['SQ_WAVE_CYCLES'] * 4 / (1024 * cyc):.2f}")
    print(f"wave time split: wait {sq['SQ_WAIT_ANY'] / sq['SQ_WAVE_CYCLES']:.3f}, issue-stall "
          f"{sq['SQ_WAIT_INST_ANY'] / sq['SQ_WAVE_CYCLES']:.3f}, active {sq['SQ_ACTIVE_INST_ANY'] / sq['SQ_WAVE_CYCLES']:.3f}")
ins, _ = res["inst"]
if ins:
    nw = ins["SQ_WAVES"]
    print("per wave: " + ", ".join(f"{k[9:]} {ins[k] / nw:.0f}" for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA",
                                                                         "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                                                                         "SQ_INSTS_SALU") if k in ins))
lds, _ = res["lds"]
if lds:
    print(f"LDS bank conflicts / LDS active cycles {lds['SQ_LDS_BANK_CONFLICT'] / max(lds['SQ_LDS_IDX_ACTIVE'], 1):.4f}")
tcc, _ = res["tcc"]
if tcc:
    h, m = tcc["TCC_HIT_sum"], tcc["TCC_MISS_sum"]
    print(f"L2 hit rate {h / (h + m):.3f}")
f, tf = res["fetch"]
w, _ = res["write"]
if f and w:
    f, w = f["FETCH_SIZE"], w["WRITE_SIZE"]
    hbm = (2 * f + w) * 1024
    alg = 32.0 * N * B
    print(f"launch at B={B}: FETCH {f * 1024 / 1e6:.1f} MB (x2 = {2 * f * 1024 / 1e6:.1f}), WRITE {w * 1024 / 1e6:.1f} MB, "
          f"traffic {hbm / 1e6:.1f} MB = {hbm / alg:.2f}x the algorithmic y+h {alg / 1e6:.1f} MB; "
          f"{hbm / tf / 1e9:.0f} GB/s over the dispatch")
    cal = None
    cf, cw = res["cfetch"][0].get("FETCH_SIZE"), res["cwrite"][0].get("WRITE_SIZE")
    if cf and cw:
        cal = dict(read_ratio=2 * cf * 1024 / (16 * N * B), write_ratio=cw * 1024 / (16 * N * B))
        print(f"K=1 calibration: 2*FETCH / y bytes = {cal['read_ratio']:.3f}, WRITE / h bytes = {cal['write_ratio']:.3f}")
    kern = "fft" if pat.startswith("k_fft") else "f64"
    # DRAM-side requests (TCC_EA0_{RD,WR}REQ_DRAM: L2 misses that went to HBM, not the Infinity Cache); bytes per
    # request from the K=1 calibration of the kernel's own y / h pattern when present, else 64 B
    dram = None
    dr, _ = res["dram"]
    if dr:
        rq, wq = dr.get("TCC_EA0_RDREQ_DRAM_sum", 0.0), dr.get("TCC_EA0_WRREQ_DRAM_sum", 0.0)
        cd, _ = res["cdram"]
        rb = wb = 64.0
        basis = "64 B per request (no calibration pass)"
        if cd and cd.get("TCC_EA0_RDREQ_DRAM_sum") and cd.get("TCC_EA0_WRREQ_DRAM_sum"):
            rb = 16.0 * N * B / cd["TCC_EA0_RDREQ_DRAM_sum"]
            wb = 16.0 * N * B / cd["TCC_EA0_WRREQ_DRAM_sum"]
            basis = f"bytes per request calibrated on the K=1 run (read {rb:.1f} B, write {wb:.1f} B)"
        dram = dict(bytes_per_launch=rq * rb + wq * wb, read_requests=rq, write_requests=wq, basis=basis)
        print(f"DRAM (HBM) side: {rq:.4g} read + {wq:.4g} write requests -> {dram['bytes_per_launch'] / 1e6:.1f} MB "
              f"= {dram['bytes_per_launch'] / alg:.2f}x algorithmic ({basis})")
    json.dump({"config": cfg, "B": B, "kernel": kern, "kernel_name": pat, "build_id": bid,
               "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": alg, "dram": dram,
               "fetch_size_kb": f, "write_size_kb": w, "calibration_k1": cal,
               "note": "hbm_bytes_per_launch: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, FETCH "
                       "doubled (gfx950), as MI355X_MICROARCH.md prescribes -- it counts L2 misses served by the "
                       "Infinity Cache too; dram: the requests that reached HBM; tools/pmc_kernel.sh + pmc_report.py"},
              open(os.path.join(base, f"{tname}.json"), "w"), indent=1)
