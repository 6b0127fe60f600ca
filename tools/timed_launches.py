"""rocprofv3 kernel trace of the bench's traced run vs the bench line's live timer.

usage: timed_launches.py run_kernel_trace.csv trace_timed_bench.json

The traced run (tools/profile_round.sh) is bench.py with the timed loop only:
W warmup steps, one step that resets the timer, then the K timed steps, all
with batch B.  Its line names the timed kernel and K.  This prints, for that
kernel, the rocprofv3 durations of every launch and of the last K (the timed
steps), next to the line's device-clock span and HIP-event averages, as JSON.
"""
import csv
import json
import statistics
import sys


def main(trace_csv, bench_json):
    line = json.load(open(bench_json))
    rf = line.get("roofline_concurrent") or line["roofline"]  # (the timed loop's live timer)
    kern, k = rf["kernel"], line["steps"]
    rows = [r for r in csv.DictReader(open(trace_csv)) if r["Kernel_Name"].split("(")[0].split("<")[0].endswith(kern)]
    # the bench's batch size is in its grid (k_* kernels of other batch sizes are
    # other legs): keep the launches of the most frequent grid
    grids = {}
    for r in rows:
        grids.setdefault((r["Kernel_Name"], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"]), []).append(r)
    rows = max(grids.values(), key=len)  # (the traced run holds the timed loop's launches only)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    timed = dur[-k:]
    out = {
        "kernel": kern, "variant": rows[0]["Kernel_Name"].split("(")[0], "launches_traced": len(dur),
        "timed_launches": len(timed), "groups": {"%s grid %s" % (g[0].split("(")[0], g[1:]): len(v) for g, v in grids.items()},
        "rocprof_avg_ms_all": round(statistics.mean(dur), 5),
        "rocprof_avg_ms_timed": round(statistics.mean(timed), 5),
        "bench_avg_launch_ms_device_clock": rf.get("avg_launch_ms_device_clock"),
        "bench_avg_launch_ms_hip_events": rf.get("avg_launch_ms_hip_events"),
        "device_clock_vs_rocprof": round(rf.get("avg_launch_ms_device_clock", 0) / statistics.mean(timed), 4),
        "algorithmic_bytes_per_launch": rf.get("algorithmic_bytes_per_launch"),
        "frac_rocprof_timed": round(rf["algorithmic_bytes_per_launch"] / (statistics.mean(timed) * 1e-3) / 1e9 /
                                    rf["peak"], 6) if rf.get("algorithmic_bytes_per_launch") else None,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
