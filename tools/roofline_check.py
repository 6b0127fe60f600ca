"""Recompute the bench line's roofline fractions from a rocprofv3 kernel_stats.csv.

usage: roofline_check.py kernel_stats.csv bench_line.json [isolated_traced.json]

The line's headline `roofline` is the longest kernel of the launch sequence measured
in isolation (one batch in flight, bench.py isolated_kernel_times).  The profile round
runs `bench.py --isolated-only` under `rocprofv3 --kernel-trace --stats`: every launch
in that process is serialized, so each kernel's rocprof average is its isolated
duration.  This prints, per kernel of the line's `isolated` table, the rocprof average,
the line's device-clock span, and the fraction of the 8 TB/s HBM peak recomputed from
the rocprof average and the line's algorithmic bytes per launch, with the ratio to the
line's own fraction (the check: within 5 %).
"""
import csv
import json
import sys


def stats_by_kernel(path):
    out = {}
    for r in csv.DictReader(open(path)):
        name = r["Name"].split("(")[0].replace("void ", "").strip()
        base = name.split("<")[0].split("::")[-1]
        calls, avg = int(r["Calls"]), float(r["AverageNs"]) / 1e6
        # several template variants of one kernel (e.g. the 1080p split blob launches):
        # the call-weighted mean
        c0, a0 = out.get(base, (0, 0.0))
        out[base] = (c0 + calls, (a0 * c0 + avg * calls) / (c0 + calls))
    return out


def main(stats_csv, line_json, traced_json=None):
    line = json.load(open(line_json))
    rf = line.get("roofline") or {}
    rows = rf.get("isolated") or line.get("isolated") or []
    peak = rf.get("peak", 8000.0)
    st = stats_by_kernel(stats_csv)
    traced = {}
    if traced_json:
        traced = {r["kernel"]: r for r in json.load(open(traced_json)).get("isolated", [])}
    res = []
    for r in rows:
        k = r["kernel"]
        if k not in st or not r.get("algorithmic_bytes_per_launch"):
            continue
        calls, avg = st[k]
        frac = r["algorithmic_bytes_per_launch"] / (avg * 1e-3) / 1e9 / peak
        e = {"kernel": k, "rocprof_calls": calls, "rocprof_avg_ms": round(avg, 5),
             "line_avg_launch_ms_device_clock": r["avg_launch_ms_device_clock"],
             "line_frac": r["frac"], "frac_from_rocprof": round(frac, 6),
             "ratio_line_to_rocprof": round(r["frac"] / frac, 4) if r.get("frac") else None}
        if k in traced:
            e["traced_run_avg_launch_ms_device_clock"] = traced[k]["avg_launch_ms_device_clock"]
        res.append(e)
    head = rf.get("kernel") or (rows[0]["kernel"] if rows else None)
    hv = next((e for e in res if e["kernel"] == head), None)
    print(json.dumps({"headline_kernel": head, "headline_line_frac": rf.get("frac"),
                      "headline_frac_from_rocprof": hv["frac_from_rocprof"] if hv else None,
                      "headline_within_5pct": (abs(hv["ratio_line_to_rocprof"] - 1) <= 0.05) if hv else None,
                      "kernels": res}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
