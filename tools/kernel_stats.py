#!/usr/bin/env python3
"""Steady-state kernel statistics from a rocprofv3 --kernel-trace CSV.

rocprofv3 --stats averages every launch of a kernel, warm-up launches
included (C2's render average 5.856 ms over 6 launches,
max 6.54 ms, against a 5.619 ms step).  This reads the per-dispatch rows of
the same run's *_kernel_trace.csv, drops each kernel's first --skip launches
(the bench's warm-up steps) and reports, per kernel: the steady launches,
mean, median, min, max and standard deviation in ns, and the share of the
summed steady time.  It also prints the per-step time of the steady launches
(the summed durations of every kernel the timed steps launch, divided by the
steps) for comparison with the bench line's ms_per_step.

    python tools/kernel_stats.py TRACE.csv --skip W --steps K [--out steady.csv]"""
import argparse
import csv
import statistics
import sys


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        if r.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
            continue
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def summarise(rows, skip, steps):
    by = {}
    for t0, t1, name in rows:
        by.setdefault(name, []).append(t1 - t0)
    out = []
    for name, ds in by.items():
        # kernels launched once per step: drop the warm-up launches, keep the
        # timed steps' (kernels launched a different number of times -- the
        # STATS instance, copies -- are listed whole)
        steady = ds[skip:skip + steps] if len(ds) >= skip + steps and steps > 0 else ds
        out.append({"Name": name, "Calls": len(ds), "SteadyCalls": len(steady),
                    "MeanNs": statistics.fmean(steady), "MedianNs": statistics.median(steady),
                    "MinNs": min(steady), "MaxNs": max(steady),
                    "StdDevNs": statistics.pstdev(steady) if len(steady) > 1 else 0.0,
                    "per_step": len(ds) >= skip + steps and steps > 0})
    total = sum(o["MeanNs"] * o["SteadyCalls"] for o in out)
    for o in out:
        o["Percentage"] = 100.0 * o["MeanNs"] * o["SteadyCalls"] / max(1.0, total)
    out.sort(key=lambda o: -o["MeanNs"] * o["SteadyCalls"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=1, help="warm-up launches per kernel to drop")
    ap.add_argument("--steps", type=int, default=0, help="timed steps (launches kept per kernel)")
    ap.add_argument("--match", default="", help="kernels whose name contains this only")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = [r for r in load(a.trace) if a.match in r[2]]
    st = summarise(rows, a.skip, a.steps)
    keys = ["Name", "Calls", "SteadyCalls", "MeanNs", "MedianNs", "MinNs", "MaxNs", "StdDevNs",
            "Percentage"]
    w = csv.DictWriter(open(a.out, "w") if a.out else sys.stdout, fieldnames=keys,
                       extrasaction="ignore", quoting=csv.QUOTE_NONNUMERIC)
    w.writeheader()
    for o in st:
        w.writerow(o)
    if a.steps:
        per_step = sum(o["MeanNs"] for o in st if o["per_step"] and o["SteadyCalls"] == a.steps)
        print("steady per-step kernel time: %.4f ms (%d timed steps, first %d launches dropped)"
              % (per_step / 1e6, a.steps, a.skip), file=sys.stderr)


if __name__ == "__main__":
    main()
