"""Audit of the inline-asm sites' hazards in the gfx950 ISA: compiles the sources that use
lds_dma16 / inline ds_read to assembly and checks, at every global_load_lds_dwordx4, that M0 was written by the
asm block's own s_mov_b32 and followed by >= 1 wait state before the DMA (CDNA3/4 hazard: SALU write of M0 ->
LDS-DMA read of M0 needs 1 wait state), and that the DMA's address operand is a VGPR pair ("off": no SGPR base, so
the SALU-write -> VMEM-SGPR-read hazard of the reverted saddr form cannot occur).  Prints one line per source and
exits non-zero on a violation.  python tools/asm_hazard_audit.py [sources...]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "quantized_channel_estimation_amd", "csrc")
DEFAULT = ["qce_f64g_m64.hip", "qce_f64_m64.hip", "qce_f64_m128.hip", "qce_wsum_f64.hip", "qce_estimate_h2.hip",
           "qce_h2x_s128x128.hip"]


def audit(src):
    asm = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                          "--cuda-device-only", "-S", src, "-o", "-", "-I" + os.path.join(ROOT, "include")],
                         capture_output=True, text=True, check=True).stdout
    lines = [ln.strip() for ln in asm.splitlines()]
    ins = [ln for ln in lines if ln and not ln.startswith((";", ".", "//")) and not ln.endswith(":")]
    n_dma, bad = 0, []
    for i, ln in enumerate(ins):
        if not ln.startswith("global_load_lds"):
            continue
        n_dma += 1
        prev = ins[i - 1] if i >= 1 else ""
        prev2 = ins[i - 2] if i >= 2 else ""
        ok = prev.startswith("s_nop") and prev2.startswith("s_mov_b32 m0")
        ok = ok and re.search(r"global_load_lds_dwordx4 v\[\d+:\d+\], off", ln) is not None
        if not ok:
            bad.append((prev2, prev, ln))
    return n_dma, bad


def main():
    srcs = sys.argv[1:] or [os.path.join(CSRC, s) for s in DEFAULT]
    rc = 0
    for s in srcs:
        n, bad = audit(s)
        print(f"{os.path.basename(s)}: {n} LDS-DMA sites, {len(bad)} violations", flush=True)
        for b in bad[:5]:
            print("   ", " | ".join(b))
        rc |= bool(bad)
    return rc


if __name__ == "__main__":
    sys.exit(main())
