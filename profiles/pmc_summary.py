#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into HBM bytes per render-kernel launch.

    python profiles/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> \
        --config C2 [--valu <valu_counter_collection.csv>] [--out profiles/pmc_C2.json]

FETCH_SIZE and WRITE_SIZE are collected in separate passes (TCC slots, see
MI355X_MICROARCH.md "rocprofv3 PMC slots"); both are in KiB.  Per that guide's
HBM section, gfx950's FETCH_SIZE reports half the bytes of a wide coalesced read,
so it is doubled; WRITE_SIZE is taken as is.  Only steady-state launches of the
non-instrumented render kernel (render_tiles<false, F>) are averaged.

The optional VALU pass (SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, the four
SQ_INSTS_VALU_*_F64 counters, GRBM_GUI_ACTIVE) gives the kernel's compute side:
fp64 FLOP per launch (64 per ADD/MUL/TRANS wave-instruction, 128 per FMA) and the
VALU issue occupancy SQ_ACTIVE_INST_VALU x 4 (quad-cycles) / (GRBM_GUI_ACTIVE / 8
XCDs x 1024 SIMDs).
"""
import argparse
import csv
import json


def per_launch(path, counter):
    vals = []
    for r in csv.DictReader(open(path)):
        if "render_tiles<false" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit("no render_tiles<false, F> rows for %s in %s" % (counter, path))
    return sum(vals) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--config", required=True)
    ap.add_argument("--out")
    ap.add_argument("--valu")
    a = ap.parse_args()
    f_kib, nf = per_launch(a.fetch_csv, "FETCH_SIZE")
    w_kib, nw = per_launch(a.write_csv, "WRITE_SIZE")
    fetch = 2.0 * f_kib * 1024
    write = w_kib * 1024
    res = {"config": a.config, "launches": [nf, nw], "fetch_size_kib_raw": f_kib,
           "write_size_kib": w_kib, "hbm_read_bytes_per_launch": int(fetch),
           "hbm_write_bytes_per_launch": int(write), "hbm_bytes_per_launch": int(fetch + write),
           "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section)"}
    if a.valu:
        c = {k: per_launch(a.valu, k)[0] for k in (
            "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
            "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64", "GRBM_GUI_ACTIVE")}
        f64 = (c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_ADD_F64"]
               + c["SQ_INSTS_VALU_TRANS_F64"])
        res.update({
            "valu_insts_per_launch": int(c["SQ_INSTS_VALU"]),
            "f64_insts_per_launch": int(f64),
            "f64_flops_per_launch": int(64 * (f64 - c["SQ_INSTS_VALU_FMA_F64"])
                                        + 128 * c["SQ_INSTS_VALU_FMA_F64"]),
            # rocprofv3's VALUBusy; may exceed 1 (gfx950 dual issue): bench.py
            # reports valu_busy from SQ_ACTIVE_INST_VALU2 as well (valu_figures)
            "valu_issue_ratio": round(4 * c["SQ_ACTIVE_INST_VALU"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024), 4),
            "valu_counters": {k: int(v) for k, v in c.items()}})
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
