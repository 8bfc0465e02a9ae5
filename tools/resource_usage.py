"""Print per-kernel VGPR/AGPR/spill/occupancy from hipcc -Rpass-analysis=kernel-resource-usage."""
import re
import subprocess
import sys

src = sys.argv[1]
extra = sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", src, "-o", "/tmp/_ru.o",
       "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    nm = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
    print(f"{nm[:70]:70s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} spill={r.get('VGPRs Spill')} "
          f"occ={r.get('Occupancy [waves/SIMD]')} lds={r.get('LDS Size [bytes/block]')} sgpr={r.get('SGPRs')}")
