"""Summarize an interleaved A/B stages.txt (tools/ab_stages.sh): per library the
concurrent frames/s of every round, their mean, and the mean serialized stage times.
usage: python tools/ab_summary.py stages.txt [kernel ...]"""
import collections
import sys

d = collections.defaultdict(list)
st = collections.defaultdict(lambda: collections.defaultdict(list))
for line in open(sys.argv[1]):
    p = line.split()
    lib = p[1].split("/")[-1]
    d[lib].append(float(p[2]))
    for kv in p[4:]:
        k, v = kv.split("=")
        st[lib][k].append(float(v))
ks = sys.argv[2:]
for lib in d:
    print(lib, " ".join("%.1f" % (x / 1e3) for x in d[lib]), "| mean %.2f k" % (sum(d[lib]) / len(d[lib]) / 1e3), "|",
          " ".join("%s=%.4f" % (k, sum(v) / len(v)) for k, v in st[lib].items() if not ks or k in ks))
