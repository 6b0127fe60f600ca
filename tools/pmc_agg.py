"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel: mean value of
each counter per dispatch.  usage: python tools/pmc_agg.py CSV [CSV ...]"""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "at::" not in k:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((path, r["Dispatch_Id"]))
for k in sorted(acc):
    nd = len(disp[k]) / max(1, len(sys.argv) - 1)
    print(k, "dispatches=%d" % nd)
    for c, v in sorted(acc[k].items()):
        print("   %-24s %14.0f" % (c, v / nd))
