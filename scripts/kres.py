#!/usr/bin/env python3
"""Per-kernel register / spill / LDS summary of a hipcc -Rpass-analysis=kernel-resource-usage log.
Usage: hipcc ... -Rpass-analysis=kernel-resource-usage -c X.hip 2> log; python scripts/kres.py log [filter]"""
import re, subprocess, sys
txt = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ''
cur = None
rows = {}
for line in txt.splitlines():
    m = re.search(r'remark: Function Name: (\S+)', line)
    if m:
        cur = m.group(1); rows[cur] = {}
        continue
    m = re.search(r'remark:\s+([A-Za-z \[\]/]+?):\s+(\d+)', line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
names = list(rows)
dem = subprocess.run(['c++filt'], input='\n'.join(names), capture_output=True, text=True).stdout.split('\n')
for n, d in zip(names, dem):
    if flt not in d:
        continue
    r = rows[n]
    print(f"{d[:90]:90s} V{r.get('VGPRs')} A{r.get('AGPRs','-')} S{r.get('TotalSGPRs')} "
          f"vsp{r.get('VGPRs Spill')} ssp{r.get('SGPRs Spill')} scr{r.get('ScratchSize [bytes/lane]')} "
          f"occ{r.get('Occupancy [waves/SIMD]')} lds{r.get('LDS Size [bytes/block]')}")
