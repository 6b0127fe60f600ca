"""FETCH_SIZE / WRITE_SIZE calibration from tools/pmc_calib (one rocprofv3 --pmc pass each).

Each calibration kernel moves a known byte count with one access pattern
(tools/pmc_calib.hip); the counters (KiB per dispatch) divided by those bytes
give the factor to apply per pattern.  The 1-byte streaming read is skipped:
its loads are folded away (XOR of bytes into a word compared with a constant
whose high bytes are nonzero).

usage: python tools/pmc_calib.py DIR   (DIR = gpurun_out/<tag> of tools/profile_round.sh)
writes DIR/pmc_calibration.json
"""
import csv
import json
import os
import sys

NAMES = {  # rocprof kernel name prefix -> calibration row
    "void stream_rd<unsigned int>": "stream_rd4", "void stream_rd<unsigned long>": "stream_rd8",
    "void stream_rd<HIP_vector_type<unsigned int, 4u> >": "stream_rd16",
    "void stream_wr<unsigned char>": "stream_wr1", "void stream_wr<unsigned int>": "stream_wr4",
    "void stream_wr<unsigned long>": "stream_wr8", "void stream_wr<HIP_vector_type<unsigned int, 4u> >": "stream_wr16",
    "void gather_rd<unsigned int>": "gather_rd4", "void gather_rd<unsigned long>": "gather_rd8",
    "scatter_wr4": "scatter_wr4", "scatter_atomic4": "scatter_atomic4",
}


def counters(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0]
        for pre, row in NAMES.items():
            if name == pre:
                out[row] = float(r["Counter_Value"]) * 1024
    return out


def main(d):
    known = {r["kernel"]: r for r in csv.DictReader(open(os.path.join(d, "calib_bytes.csv")))}
    fetch = counters(os.path.join(d, "calib_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counters(os.path.join(d, "calib_write", "run_counter_collection.csv"), "WRITE_SIZE")
    rows = {}
    for k, r in known.items():
        if k not in fetch and k not in write:
            continue
        nbytes, acc = int(r["bytes_moved"]), int(r["accesses"])
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        # the index array of the gathers / scatters is itself a 4-B streaming read (FETCH x1/2)
        idx = 4 * acc / 2 if k.startswith(("gather", "scatter")) else 0.0
        rows[k] = {"bytes": nbytes, "accesses": acc, "fetch_size_bytes": round(f), "write_size_bytes": round(w),
                   "fetch_per_byte": round((f - idx) / nbytes, 4) if "rd" in k else None,
                   "write_per_byte": round(w / nbytes, 4) if ("wr" in k or "atomic" in k) else None,
                   "fetch_per_access": round((f - idx) / acc, 2), "write_per_access": round(w / acc, 2)}
    res = {"rows": rows,
           "summary": "streaming reads (4/8/16 B per lane): FETCH_SIZE = 1/2 of the bytes (x2 correction exact); "
                      "streaming stores (1-16 B): WRITE_SIZE = the bytes; a scattered 4/8-B read on its own 128-B "
                      "line: FETCH_SIZE 64 B (the true DRAM cost is 64-128 B, so x2 is an upper bound); a scattered "
                      "4-B store or atomic: WRITE_SIZE 32 B, no FETCH_SIZE for the atomic's line read"}
    json.dump(res, open(os.path.join(d, "pmc_calibration.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
