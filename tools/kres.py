#!/usr/bin/env python3
"""tools/kres.py FILE.hip [more hipcc args] — per-kernel VGPRs / SGPRs / scratch / spills /
occupancy from hipcc's kernel-resource-usage remarks (gfx950), one line per kernel."""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
       "-I../include", "-Iinclude", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in err.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
filt = re.compile(sys.argv[2]) if False else None
for r in rows:
    d = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    d = re.sub(r"\(.*", "", d)
    print(f"{d:70s} V{r.get('VGPRs','?'):>4} A{r.get('AGPRs','?'):>3} S{r.get('SGPRs','?'):>4} "
          f"scr{r.get('ScratchSize [bytes/lane]','?'):>4} vsp{r.get('VGPRs Spill','?'):>3} "
          f"ssp{r.get('SGPRs Spill','?'):>3} occ{r.get('Occupancy [waves/SIMD]','?'):>3} "
          f"lds{r.get('LDS Size [bytes/block]','?'):>6}")
