"""Print per-kernel VGPRs / scratch / occupancy from hipcc -Rpass-analysis output (stdin)."""
import re
import sys

cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split(" ")[0].replace("\\", "")] = int(m.group(1))
for r in rows:
    n = r["name"]
    m = re.match(r"_ZN2zk\d+(\w+?)I", n) or re.match(r"_ZN2zk\d+(\w+?)E", n)
    short = n[:70]
    print(f"{short:72s} v{r.get('VGPRs')} a{r.get('AGPRs')} scr{r.get('ScratchSize')} occ{r.get('Occupancy')} lds{r.get('LDS')}")
