"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin):
one line per kernel with VGPRs, AGPRs, scratch bytes, occupancy and LDS.
    hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kres.py [filter]"""
import re
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                  r"LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = int(m.group(2))
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:90]:90s} v{r.get('VGPRs', '?'):>4} a{r.get('AGPRs', '?'):>3} "
              f"scr{r.get('ScratchSize', '?'):>4} occ{r.get('Occupancy', '?'):>2} "
              f"lds{r.get('LDS', '?'):>7}")
