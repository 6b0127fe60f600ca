"""Issue-rate ceiling of the pipeline's kernels from per-class VALU counters.

usage: valu_ceiling.py valu_rates.jsonl pmc_sq_c.csv pmc_sq_d.csv pmc_sq_e.csv [--frames B] [--step-ms T]

rocprofv3 --pmc serializes the dispatches it counts, so every dispatch's counters and
its Start/End timestamps describe the kernel alone on the chip.  Per kernel (mean per
dispatch):
  * VALU issue cycles = sum over instruction classes of count x the class's measured
    issue cost (cycles per wave64 instruction per SIMD, tools/valu_rates on the same box,
    8 waves per SIMD); unclassified VALU instructions (moves, logic, compares, DPP,
    lane ops) at the cost of v_add_f32;
  * VALU issue utilisation = issue cycles / (SIMDs x duration x clock), at the peak
    clock 2.4 GHz (--kernel-clock-ghz): a lower bound -- the chip runs 1.9-2.4 GHz
    under load, and GRBM_GUI_ACTIVE / 8 / duration reads high on dispatches under
    ~0.3 ms (MI355X_MICROARCH.md, DVFS), so it is reported but not used;
  * the wave-cycle shares: SQ_WAIT_ANY (parked on s_waitcnt / barrier), SQ_WAIT_INST_ANY
    (ready but not issued: dependency or pipe), SQ_ACTIVE_INST_ANY (issuing), of
    SQ_WAVE_CYCLES; SQ_WAIT_INST_LDS (a part of WAIT_INST_ANY) and the LDS bank conflicts
    per LDS instruction.
Then the pipeline: the sum of issue cycles over a step's kernels against the step time
(--step-ms, the bench line's ms_per_step at --frames per step) on the whole chip.
"""
import collections
import csv
import json
import sys

SIMDS = 1024  # 256 CUs x 4 SIMD-32


def load_rates(path):
    r = {}
    for line in open(path):
        line = line.strip()
        if line.startswith("{"):
            j = json.loads(line)
            r[j["class"]] = j["cycles_per_wave_instr_per_simd"]
    base = r["add_f32"]
    f64 = r.get("fma_f64", 2 * base)
    cost = {
        "SQ_INSTS_VALU_ADD_F32": r.get("add_f32", base), "SQ_INSTS_VALU_MUL_F32": r.get("fma_f32", base),
        "SQ_INSTS_VALU_FMA_F32": r.get("fma_f32", base), "SQ_INSTS_VALU_INT32": base,
        "SQ_INSTS_VALU_ADD_F64": r.get("add_f64", f64), "SQ_INSTS_VALU_MUL_F64": f64, "SQ_INSTS_VALU_FMA_F64": f64,
        # the rate kernels pair each transcendental with one add: subtract it
        "SQ_INSTS_VALU_TRANS_F32": max(base, r.get("sqrt_f32", 2 * base) - base),
        "SQ_INSTS_VALU_TRANS_F64": max(f64, r.get("sqrt_f64", 4 * base) - r.get("add_f64", f64)),
        # 64-bit integer ops counted once per instruction (shifts, 64-bit adds are two
        # 32-bit instructions counted as INT32): at the f64 rate
        "SQ_INSTS_VALU_INT64": f64,
        "SQ_INSTS_VALU_CVT": base,
    }
    return cost, base, r


def per_kernel(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(lambda: collections.defaultdict(int))
    dur = collections.defaultdict(list)
    for p in paths:
        seen = set()
        for row in csv.DictReader(open(p)):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "")
            if "at::" not in k or "at::native" in k:  # (torch's own kernels: the pool set-up copy)
                continue
            c = row["Counter_Name"]
            acc[k][c] += float(row["Counter_Value"])
            n[k][c] += 1
            key = (p, row["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    out = {}
    for k in acc:
        out[k] = {c: acc[k][c] / n[k][c] for c in acc[k]}
        out[k]["_dur_s"] = sum(dur[k]) / len(dur[k])
        out[k]["_dispatches"] = len(dur[k]) / len(paths)
    return out


def main(argv):
    args = [a for a in argv if not a.startswith("--")]
    opts = dict(a[2:].split("=", 1) for a in argv if a.startswith("--") and "=" in a)
    cost, base, rates = load_rates(args[0])
    K = per_kernel(args[1:])
    rows = []
    tot_cyc = 0.0
    for k, c in sorted(K.items(), key=lambda kv: -kv[1]["_dur_s"]):
        if "SQ_INSTS_VALU" not in c:
            continue
        classified = 0.0
        cyc = 0.0
        for cls, w in cost.items():
            v = c.get(cls, 0.0)
            classified += v
            cyc += v * w
        other = max(0.0, c["SQ_INSTS_VALU"] - classified)
        cyc += other * base
        tot_cyc += cyc
        grbm_clk = c.get("GRBM_GUI_ACTIVE", 0.0) / 8 / c["_dur_s"] if c["_dur_s"] > 0 else 0.0
        clk = float(opts.get("kernel-clock-ghz", "2.4")) * 1e9
        util = cyc / (SIMDS * c["_dur_s"] * clk)
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        row = {"kernel": k, "dur_ms": round(c["_dur_s"] * 1e3, 4), "grbm_clock_ghz": round(grbm_clk / 1e9, 3),
               "valu_instr_M": round(c["SQ_INSTS_VALU"] / 1e6, 2),
               "valu_issue_cycles_M": round(cyc / 1e6, 2),
               "valu_issue_util": round(util, 3) if util else None,
               "f64_share_of_issue": round(sum(c.get(x, 0) * cost[x] for x in cost if "F64" in x) / cyc, 3) if cyc else None,
               "trans_share_of_issue": round(sum(c.get(x, 0) * cost[x] for x in cost if "TRANS" in x) / cyc, 3) if cyc else None}
        if wc:
            row.update({"wait_any": round(c.get("SQ_WAIT_ANY", 0) / wc, 3),
                        "wait_inst_any": round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
                        "active_inst_any": round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3)})
        if c.get("SQ_WAIT_INST_LDS") is not None and wc:
            row["wait_inst_lds"] = round(c["SQ_WAIT_INST_LDS"] / wc, 4)
        if c.get("SQ_INSTS_LDS"):
            row["lds_conflicts_per_op"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_INSTS_LDS"], 3)
        rows.append(row)
    out = {"issue_costs_cycles_per_wave_instr": {k: round(v, 3) for k, v in rates.items()}, "kernels": rows,
           "step_valu_issue_cycles_M": round(tot_cyc / 1e6, 1)}
    if "step-ms" in opts:
        step_s = float(opts["step-ms"]) * 1e-3
        clk = float(opts.get("clock-ghz", "2.4")) * 1e9
        out["pipeline_valu_issue_util"] = round(tot_cyc / (SIMDS * step_s * clk), 3)
        out["pipeline_note"] = ("sum of the kernels' issue cycles of one step (counters at batch %s) over %d SIMDs x "
                                "the step time %s ms x %s GHz" % (opts.get("frames", "?"), SIMDS, opts["step-ms"],
                                                                   opts.get("clock-ghz", "2.4")))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
