"""Register / spill / occupancy summary of every kernel in one HIP source (hipcc -Rpass-analysis=kernel-resource-usage).
python tools/regs.py quantized_channel_estimation_amd/csrc/qce_f64g_m64.hip [-DNAME=V ...]"""
import re
import subprocess
import sys

src, defs = sys.argv[1], sys.argv[2:]
p = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o",
                    "/tmp/regs_probe.o", "-Rpass-analysis=kernel-resource-usage"] + defs,
                   capture_output=True, text=True)
cur = None
rows = []
for line in p.stderr.splitlines():
    m = re.search(r"remark:\s+(.*?)\s+\[-Rpass", line)
    if not m:
        if "error" in line:
            print(line)
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    n = re.sub(r"EvxiiiixPK.*", "", r["name"])
    print(f"{n:60s} VGPR {r.get('VGPRs','?'):>4} AGPR {r.get('AGPRs','?'):>3} spillV {r.get('VGPRs Spill','?'):>3} "
          f"spillS {r.get('SGPRs Spill','?'):>3} occ {r.get('Occupancy [waves/SIMD]','?')} LDS {r.get('LDS Size [bytes/block]','?')}")
