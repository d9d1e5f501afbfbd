#!/usr/bin/env python3
"""Summarise a profile_round.sh run into profiles/.

- <tag>_kernel_stats.csv          rocprofv3 --kernel-trace --stats of the default bench command
- <tag>_kernel_stats_serial.csv   the same with --inflight 1 (averages = bench's kernel_ms)
- <tag>_pmc_traffic.json          HBM bytes per launch per kernel from the two PMC passes,
                                  bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md
                                  HBM section: gfx950 FETCH_SIZE counts half of wide streaming reads)
usage: tools/pmc_summary.py <tag> [gpurun_out/prof_<tag>]
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter or not row["Kernel_Name"].startswith("k_"):
                continue
            vals.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    shutil.copy(os.path.join(src, "trace_serial", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats_serial.csv"))
    for name in ("bench_under_trace.json", "bench_under_trace_serial.json"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(prof, f"{tag}_{name}"))
    out = traffic_summary(src, "", tag, prof)
    vpath = os.path.join(src, "pmc_valu", "run_counter_collection.csv")
    if os.path.exists(vpath):
        valu_summary(vpath, tag, prof)
    print(json.dumps({k: v for k, v in out.items() if not k.endswith("_KiB")}, indent=1))
    # the C3 circuit's passes (profile_round.sh step 5), when present: <tag>_c3_*
    if os.path.exists(os.path.join(src, "c3_pmc_fetch")):
        shutil.copy(os.path.join(src, "c3_trace_serial", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_c3_kernel_stats_serial.csv"))
        traffic_summary(src, "c3_", tag + "_c3", prof)
        valu_summary(os.path.join(src, "c3_pmc_valu", "run_counter_collection.csv"), tag + "_c3", prof)


def traffic_summary(src, pre, tag, prof):
    """<tag>_pmc_traffic.json from the <pre>pmc_fetch / <pre>pmc_write passes."""
    fetch = per_kernel(os.path.join(src, pre + "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, pre + "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    out = {"_note": "HBM bytes per launch (median over launches) from rocprofv3 PMC, separate FETCH_SIZE / WRITE_SIZE "
                    "passes of bench.py --steps 3 --inflight 1, corrected per MI355X_MICROARCH.md HBM section: "
                    "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024; batch = 4096 "
                    + ("C3 (live lookup) proofs" if pre else "std proofs") + "; round " + tag}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        out[k] = int(round((2 * f + w) * 1024))
        out[k + "_raw_KiB"] = {"FETCH_SIZE": f, "WRITE_SIZE": w}
    json.dump(out, open(os.path.join(prof, f"{tag}_pmc_traffic.json"), "w"), indent=1)
    return out


VALU_COUNTERS = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU2", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_WAVES",
                 "SQ_INSTS_SALU", "SQ_ACTIVE_INST_VALU", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")


def durations(path):
    """Median dispatch duration (s) per kernel from the PMC csv's timestamps."""
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != "SQ_INSTS_VALU" or not row["Kernel_Name"].startswith("k_"):
                continue
            vals.setdefault(row["Kernel_Name"], []).append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return {k: statistics.median(v) for k, v in vals.items()}


def valu_summary(vpath, tag, prof):
    """<tag>_pmc_valu.json: VALU instruction counters per kernel launch (median).  The VALU issue
    model (measured, profiles/r02_valu_rates.txt + r02_valu_rates_pmc.json): a SIMD issues one
    VALU instruction per 4-cycle quad, or two in one quad when both are dual-issuable (VOP1/VOP2
    32-bit ops; SQ_ACTIVE_INST_VALU2 counts those quads), so a launch's VALU issue cycles are
    4 * (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2); bench.py divides them by 1024 SIMDs x 2.4 GHz x time."""
    valu = {c: per_kernel(vpath, c) for c in VALU_COUNTERS}
    valu = {c: v for c, v in valu.items() if v}
    tot = sum(valu["SQ_INSTS_VALU"].values())
    vout = {"_note": "rocprofv3 PMC SQ counters per launch (median), bench.py --steps 3 --inflight 1, batch = 4096 std "
                     "proofs; SQ_INSTS_VALU = wave-level VALU instructions, SQ_ACTIVE_INST_VALU2 = quad-cycles in which "
                     "two VALU instructions issued; issue_cycles = 4 * (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2); "
                     "share = fraction of all VALU instructions of one verification step; round " + tag}
    dur = durations(vpath)
    for k in sorted(valu["SQ_INSTS_VALU"]):
        vout[k] = {c: valu[c].get(k) for c in valu}
        vout[k]["issue_cycles"] = 4 * (valu["SQ_INSTS_VALU"][k] - valu.get("SQ_ACTIVE_INST_VALU2", {}).get(k, 0.0))
        vout[k]["valu_share"] = round(valu["SQ_INSTS_VALU"][k] / tot, 4)
        g = valu.get("GRBM_GUI_ACTIVE", {}).get(k)
        if g and dur.get(k):
            # the guide's effective clock: GRBM_GUI_ACTIVE summed over the 8 XCDs / 8 / wall time
            # (reads high on dispatches shorter than ~0.3 ms)
            vout[k]["duration_s"] = dur[k]
            vout[k]["effective_clock_ghz"] = round(g / 8 / dur[k] / 1e9, 3)
            vout[k]["issue_frac_at_effective_clock"] = round(vout[k]["issue_cycles"] / (1024 * g / 8), 3)
    json.dump(vout, open(os.path.join(prof, f"{tag}_pmc_valu.json"), "w"), indent=1)
    print(json.dumps({k: v["valu_share"] for k, v in vout.items() if not k.startswith("_")}, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--valu-only":   # tools/pmc_summary.py --valu-only <tag> <csv>
        valu_summary(sys.argv[3], sys.argv[2], os.path.join(ROOT, "profiles"))
    else:
        main()
