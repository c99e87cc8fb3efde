#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into HBM bytes per render-kernel launch.

    python profiles/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> \
        --config C2 [--out profiles/pmc_C2.json]

FETCH_SIZE and WRITE_SIZE are collected in separate passes (TCC slots, see
MI355X_MICROARCH.md "rocprofv3 PMC slots"); both are in KiB.  Per that guide's
HBM section, gfx950's FETCH_SIZE reports half the bytes of a wide coalesced read,
so it is doubled; WRITE_SIZE is taken as is.  Only steady-state launches of the
non-instrumented render kernel (render_tiles<false, F>) are averaged.
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
    a = ap.parse_args()
    f_kib, nf = per_launch(a.fetch_csv, "FETCH_SIZE")
    w_kib, nw = per_launch(a.write_csv, "WRITE_SIZE")
    fetch = 2.0 * f_kib * 1024
    write = w_kib * 1024
    res = {"config": a.config, "launches": [nf, nw], "fetch_size_kib_raw": f_kib,
           "write_size_kib": w_kib, "hbm_read_bytes_per_launch": int(fetch),
           "hbm_write_bytes_per_launch": int(write), "hbm_bytes_per_launch": int(fetch + write),
           "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section)"}
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
