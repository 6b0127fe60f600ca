"""Aggregate rocprofv3 --pmc counter_collection.csv files per kernel: the mean value
of each counter per dispatch (over the dispatches that report that counter, so a
counter collected in several passes -- GRBM_GUI_ACTIVE -- is not summed across them).
usage: python tools/pmc_agg.py CSV [CSV ...]"""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(set))
disp = collections.defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "at::" not in k:
            continue
        c = r["Counter_Name"]
        acc[k][c] += float(r["Counter_Value"])
        cnt[k][c].add((path, r["Dispatch_Id"]))
        disp[k].add((path, r["Dispatch_Id"]))
for k in sorted(acc):
    nd = len(disp[k]) / max(1, len(sys.argv) - 1)
    print(k, "dispatches=%d" % nd)
    for c, v in sorted(acc[k].items()):
        print("   %-24s %14.0f" % (c, v / max(1, len(cnt[k][c]))))
