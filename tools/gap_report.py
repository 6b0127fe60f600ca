"""Per-frame kernel chain of a B=1 kernel trace (rocprofv3 --kernel-trace CSV):
median duration of each kernel and median idle gap before it.  Usage:
python tools/gap_report.py run_kernel_trace.csv"""
import collections
import csv
import sys

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "at::k_" in r["Kernel_Name"]]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].split("(")[0].replace("void ", "").replace("at::", "")) for r in rows)
chains, cur = [], []
for s, e, n in ev:
    if (n.startswith("k_pre") or n.startswith("k_thr_ccl")) and cur and not cur[-1][2].startswith("k_pre"):
        chains.append(cur)
        cur = []
    cur.append((s, e, n))
chains = chains[len(chains) // 4:]  # steady state
dur, gap = collections.defaultdict(list), collections.defaultdict(list)
span = []
for c in chains:
    span.append((max(e for _, e, _ in c) - c[0][0]) / 1e3)
    for k, (s, e, n) in enumerate(c):
        dur[n].append((e - s) / 1e3)
        if k:
            gap[n].append((s - max(ee for _, ee, _ in c[:k])) / 1e3)
print("frames %d  first kernel start -> last kernel end: median %.1f us" % (len(chains), np.median(span)))
for n in dur:
    print("  %-26s dur %6.1f us  gap before %5.1f us" % (n[:26], np.median(dur[n]), np.median(gap[n]) if gap[n] else 0))
