#!/usr/bin/env python3
"""Summarise build/asm/resource.txt (make asm): VGPRs, spills, scratch and
occupancy of each render_tiles<STATS, F, PCW, COST> instance."""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "real-time-ray-tracing-engine_amd/build/asm/resource.txt"
cur, rows = None, {}
for line in open(path):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        k = re.search(r"render_tilesILb(\d)ELj(\d+)ELi(\d+)ELb(\d)E", m.group(1))
        cur = tuple(int(x) for x in k.groups()) if k else None
        if cur:
            rows[cur] = {}
        continue
    if cur:
        m = re.search(r"(VGPRs|VGPRs Spill|SGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
        if m:
            rows[cur][m.group(1).split(" [")[0]] = int(m.group(2))
only = [int(x) for x in sys.argv[2:]]
for (st, f, pc, cost), r in sorted(rows.items()):
    if st == 0 and (not only or f in only):
        print("F=%2d PC=%2d COST=%d  VGPRs %3d  spill %3d  sgpr-spill %3d  scratch %4d  waves %d" % (
            f, pc, cost, r.get("VGPRs", 0), r.get("VGPRs Spill", 0), r.get("SGPRs Spill", 0),
            r.get("ScratchSize", 0), r.get("Occupancy", 0)))
