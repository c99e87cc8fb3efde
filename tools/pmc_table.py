#!/usr/bin/env python3
"""Average PMC counters of the render kernel (render_tiles<false, F>) from
rocprofv3 counter_collection.csv files: python tools/pmc_table.py <csv>..."""
import collections
import csv
import sys

for path in sys.argv[1:]:
    tot, n = collections.defaultdict(float), collections.Counter()
    for r in csv.DictReader(open(path)):
        if "render_tiles<false" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
    for k in sorted(tot):
        print("%-32s %14.4g" % (k, tot[k] / n[k]))
