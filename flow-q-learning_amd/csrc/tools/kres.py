"""Per-kernel VGPR / scratch / LDS / occupancy from hipcc -Rpass-analysis=kernel-resource-usage
(developer helper): python kres.py [filter]"""
import re
import subprocess
import sys

out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-x", "hip", "-c",
                      (sys.argv[2] if len(sys.argv) > 2 else "kernels.hip"), "-I", ".", "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: (.*)\[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.strip()
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for name, r in rows.items():
    if flt in name:
        print(f"{r.get('VGPRs','?'):>4} vgpr {r.get('ScratchSize [bytes/lane]','?'):>4} scr "
              f"{r.get('LDS Size [bytes/block]','?'):>6} lds occ {r.get('Occupancy [waves/SIMD]','?'):>2}  {name[:90]}")
