"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of
`bench.py --batch B` into HBM bytes per frame -> profiles/pmc_traffic.json.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (TCC_EA0_RDREQ/WRREQ based).
Calibration on known byte counts (tools/pmc_calib.hip, profiles/r02/pmc_calibration.json):
streaming reads of 4/8/16 B per lane report exactly 1/2 of their bytes, stores
report their bytes, a scattered 4/8-B read on its own line reports 64 B (its true
DRAM cost is 64-128 B).  Per kernel we store the raw counters, the read side x2
(exact for streaming reads, an upper bound for scattered ones) as "corrected",
and read x1 as the lower bound.
"""
import csv
import json
import sys
from collections import defaultdict


def load(path, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name", r.get("Counter_Name".lower(), "")) != counter:
            continue
        name = r.get("Kernel_Name", "")
        per[name].append(float(r["Counter_Value"]))
    return per


def main(fetch_csv, write_csv, batch, width, height, out):
    f = load(fetch_csv, "FETCH_SIZE")
    w = load(write_csv, "WRITE_SIZE")
    kernels = {}
    tot_f = tot_w = 0.0
    for name in sorted(set(f) | set(w)):
        if not name.startswith(("at::k_", "k_", "void at::k_")) and "k_" not in name:
            continue
        fk = sum(f.get(name, [0])) / max(1, len(f.get(name, [1]))) * 1024 / batch
        wk = sum(w.get(name, [0])) / max(1, len(w.get(name, [1]))) * 1024 / batch
        short = name.split("(")[0].split("::")[-1]
        kernels[short] = {"fetch_bytes_per_frame": round(fk), "write_bytes_per_frame": round(wk),
                          "raw_per_frame": round(fk + wk), "corrected_per_frame": round(2 * fk + wk)}
        tot_f += fk
        tot_w += wk
    res = {"width": width, "height": height, "batch": batch,
           "hbm_bytes_per_frame": round(2 * tot_f + tot_w),
           "raw_fetch_plus_write_per_frame": round(tot_f + tot_w),
           "lower_bound_per_frame": round(tot_f + tot_w),
           "algorithmic_bytes_per_frame": 3 * width * height,
           "correction": "read side x2: exact for streaming reads (gfx950 FETCH_SIZE counts 64 B per 128 B request, "
                         "MI355X_MICROARCH.md HBM, calibrated in pmc_calibration.json), upper bound for scattered "
                         "4/8-B reads (64 B reported per access); write side as counted",
           "kernels": kernels}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6])
