"""Per-kernel resource usage of one gfx950 source (VGPRs, spills, LDS, occupancy)
from hipcc's -Rpass-analysis=kernel-resource-usage remarks.

    python tools/kres.py gsvc_amd/csrc/raster_sum.hip [name-filter] [-DGSVC_DIAG]
"""
import re
import subprocess
import sys

import os
src = os.path.abspath(sys.argv[1])
filt = [a for a in sys.argv[2:] if not a.startswith("-")]
defs = [a for a in sys.argv[2:] if a.startswith("-")]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-ffp-contract=off", "-std=c++17",
       "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage", *defs]
r = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp")
rows, cur = [], None
for line in r.stderr.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        name = t.split(":", 1)[1].strip()
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        cur = {"name": name}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
if r.returncode != 0:
    print(r.stderr[-3000:])
for c in rows:
    if filt and not any(f in c["name"] for f in filt):
        continue
    print(f'{c.get("VGPRs","?"):>4} v {c.get("VGPRs Spill","?"):>3} vs {c.get("SGPRs Spill","?"):>3} ss '
          f'{c.get("LDS Size [bytes/block]","?"):>6} lds occ {c.get("Occupancy [waves/SIMD]","?"):>2}  '
          f'{c["name"][:150]}')
