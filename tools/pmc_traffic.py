"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of
`bench.py --batch B` into HBM bytes per frame -> profiles/pmc_traffic.json.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (TCC_EA0_RDREQ/WRREQ based).
MI355X_MICROARCH.md: FETCH_SIZE reports 1/2 of the bytes of wide (16 B/lane)
coalesced streaming reads on gfx950; other widths are uncalibrated.  We report
the raw sum and the x2-corrected read side, per frame, per kernel.
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
        kernels[short] = {"fetch_bytes_per_frame": round(fk), "write_bytes_per_frame": round(wk)}
        tot_f += fk
        tot_w += wk
    res = {"width": width, "height": height, "batch": batch,
           "hbm_bytes_per_frame": round(2 * tot_f + tot_w),
           "raw_fetch_plus_write_per_frame": round(tot_f + tot_w),
           "algorithmic_bytes_per_frame": 3 * width * height,
           "correction": "read side x2 (gfx950 FETCH_SIZE counts 64 B per 128 B request, MI355X_MICROARCH.md HBM)",
           "kernels": kernels}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6])
