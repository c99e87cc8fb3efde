#!/usr/bin/env python3
"""Basic blocks of one render_tiles<STATS, F> instance in the gfx950 asm
(make asm): instruction counts by class for the blocks that look like the BVH
walk (fp32 FMAs / LDS reads).   python tools/asm_blocks.py F [--pc (the 16-wave persistent instance)] [--all] [--dump BB]"""
import re
import sys

ASM = __import__("os").environ.get("ASM", "real-time-ray-tracing-engine_amd/build/asm/rt_kernel-hip-amdgcn-amd-amdhsa-gfx950.s")


def blocks(F, stats=0, pc=0, cost=0):
    s = open(ASM).read()
    # render_tiles<STATS, F, PCW, COST> (COST: the flat world's cost-measuring instance)
    name = "_ZN12_GLOBAL__N_112render_tilesILb%dELj%dELi%dELb%dEEEv6DScene7DCamera7DLaunchPdPy" % (stats, F, pc, cost)
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    out, cur = [], ["entry", []]
    out.append(cur)
    for line in s[i:j].split("\n"):
        m = re.match(r"^(\.LBB\d+_\d+):", line)
        if m:
            cur = [m.group(1), []]
            out.append(cur)
            continue
        t = line.strip()
        if line.startswith("\t") and t and not t.startswith(";") and not t.startswith("."):
            cur[1].append(t)
    return out


def classify(ins):
    c = {}
    for x in ins:
        op = x.split()[0]
        k = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") and not op.startswith(("s_load", "s_buffer")) else
             "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else "smem")
        c[k] = c.get(k, 0) + 1
    return c


if __name__ == "__main__":
    F = int(sys.argv[1])
    bl = blocks(F, pc=16 if "--pc" in sys.argv else 0)
    if "--dump" in sys.argv:
        want = sys.argv[sys.argv.index("--dump") + 1]
        for b, ins in bl:
            if b == want:
                print("\n".join(ins))
        sys.exit()
    for b, ins in bl:
        nf = sum(1 for x in ins if "_f32" in x.split()[0])
        nds = sum(1 for x in ins if x.startswith("ds_read"))
        if "--all" in sys.argv or nf >= 6 or nds >= 2:
            br = [x for x in ins if x.startswith(("s_cbranch", "s_branch"))]
            print(b, len(ins), classify(ins), "f32", nf, br)
