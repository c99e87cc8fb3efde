#!/usr/bin/env python3
"""Static instruction histogram of one kernel in a device .s built with
-gline-tables-only, attributed to source lines (.loc) — where the VALU code of
a kernel instance comes from.

    hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -gline-tables-only \
          --cuda-device-only -S csrc/rt_kernel.hip -o k.s
    python tools/isa_lines.py k.s 'render_tilesILb0ELj0E' [--top 40]
"""
import argparse
import collections
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel", help="substring of the kernel symbol")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    files = {}
    cur = None
    inside = False
    per_line = collections.Counter()
    per_kind = collections.defaultdict(collections.Counter)
    total = collections.Counter()
    for raw in open(a.asm):
        s = raw.strip()
        m = re.match(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
            continue
        if not inside:
            lab = s.split(";")[0].strip()
            if lab.endswith(":") and a.kernel in lab and not lab.startswith("."):
                inside = True
            continue
        if s.startswith(".Lfunc_end"):
            break
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            cur = "%s:%s" % (files.get(m.group(1), m.group(1)), m.group(2))
            continue
        m = re.match(r"(v_|s_|ds_|global_|scratch_|buffer_|flat_)(\w+)", s)
        if not m:
            continue
        cls = m.group(1)
        total[cls] += 1
        if cls == "v_":
            per_line[cur] += 1
            per_kind[cur][m.group(1) + m.group(2)] += 1
    print("totals:", dict(total))
    for ln, n in per_line.most_common(a.top):
        kinds = ", ".join("%s %d" % kv for kv in per_kind[ln].most_common(4))
        print("%6d  %-22s %s" % (n, ln, kinds))


if __name__ == "__main__":
    main()
