#!/usr/bin/env python3
"""tools/pmc_report.py — turn the rocprofv3 PMC CSVs of tools/profile.sh into per-launch metrics
of the render kernel and (with --write-traffic) profiles/pmc_traffic.json, which bench.py reports
as roofline.traffic.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KB; on gfx950
FETCH_SIZE counts half of a wide coalesced read stream, so it is doubled; WRITE_SIZE is exact for
16-B-per-lane stores (the framebuffer stores here are 4 B per lane: uncalibrated, reported as is).
"""
import argparse
import collections
import csv
import json
import os
import re
import sys


def load(path, kernel_filter):
    per = collections.defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        if kernel_filter not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[d] = (r["Kernel_Name"], int(r["VGPR_Count"]), int(r["LDS_Block_Size"]),
                   int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return per, meta


def is_count_variant(name):
    """True for the RTG_RENDER_COUNT instantiation: COUNT is template argument 3 of
    render_kernel / render_kernel_lds <STACK, SPILL, COUNT, ...> and argument 2 of the A/B kernels
    render_kernel_v0 / render_kernel_segment <STACK, COUNT>."""
    m = re.search(r"(render_kernel\w*)<([^>]*)>", name)
    if not m:
        return False
    args = [x.strip() for x in m.group(2).split(",")]
    idx = 1 if m.group(1) in ("render_kernel_v0", "render_kernel_segment") else 2
    return len(args) > idx and args[idx] == "true"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir", nargs="?", default="gpurun_out/prof")
    ap.add_argument("--kernel", default="render_kernel")
    ap.add_argument("--timed-only", action="store_true", default=True,
                    help="use the non-counting dispatches only")
    ap.add_argument("--workload", default=None)
    ap.add_argument("--write-traffic", default=None)
    ap.add_argument("--write-binding", default=None,
                    help="write the binding-resource summary bench.py attaches (profiles/pmc_binding.json)")
    ap.add_argument("--simds", type=int, default=1024, help="SIMDs of the chip (256 CUs x 4)")
    ap.add_argument("--counted-launch", default="the render kernel's single launch",
                    help="which launch the counters saw (config 2: the 16-wave launch alone, RTG_DUAL=0)")
    a = ap.parse_args()
    counters, info = {}, {}
    for sub in sorted(os.listdir(a.prof_dir)):
        p = os.path.join(a.prof_dir, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        per, meta = load(p, a.kernel)
        # the render kernel that did the frame's work: the longest non-COUNT dispatch name (a dual
        # launch's 4-wave partner, serialised by counter collection, finds the work done and ends in
        # microseconds; tools/profile.sh takes the PMC passes with RTG_DUAL=0 for that reason)
        durs = {}
        for d in per:
            if not (a.timed_only and is_count_variant(meta[d][0])):
                durs.setdefault(meta[d][0], []).append(meta[d][3])
        if not durs:
            continue
        main = max(durs, key=lambda n: sum(durs[n]) / len(durs[n]))
        for d, vals in per.items():
            name = meta[d][0]
            if name != main:
                continue
            for k, v in vals.items():
                counters.setdefault(k, []).append(v)
            info[sub] = meta[d]
    avg = {k: sum(v) / len(v) for k, v in counters.items()}
    out = {"per_launch": {k: avg[k] for k in sorted(avg)}}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        out["hbm_read_bytes"] = 2 * avg["FETCH_SIZE"] * 1024
        out["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = out["hbm_read_bytes"] + out["hbm_write_bytes"]
    if "SQ_THREAD_CYCLES_VALU" in avg and "SQ_ACTIVE_INST_VALU" in avg:
        out["valu_lane_utilization"] = avg["SQ_THREAD_CYCLES_VALU"] / (64 * avg["SQ_ACTIVE_INST_VALU"])
    if "SQ_WAVE_CYCLES" in avg:
        w = avg["SQ_WAVE_CYCLES"]
        out["wave_cycle_split"] = {k: avg[k] / w for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                          "SQ_ACTIVE_INST_ANY") if k in avg}
    if "TCC_HIT_sum" in avg:
        out["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    if "TCP_TOTAL_CACHE_ACCESSES_sum" in avg and "TCP_TCC_READ_REQ_sum" in avg:
        out["l1_to_l2_read_fraction"] = avg["TCP_TCC_READ_REQ_sum"] / avg["TCP_TOTAL_CACHE_ACCESSES_sum"]
    if "GRBM_GUI_ACTIVE" in avg:
        ns = [m[3] for m in info.values()]
        out["effective_clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / (sum(ns) / len(ns))
    out["dispatch"] = {k: {"vgpr": v[1], "lds": v[2], "ns": v[3]} for k, v in info.items()}
    ns_avg = sum(m[3] for m in info.values()) / max(1, len(info))
    if "SQ_INSTS_VALU" in avg and "GRBM_GUI_ACTIVE" in avg:
        # wave64 VALU issue takes 2 cycles of a SIMD-32 (MI355X_MICROARCH.md constants table);
        # kernel cycles per SIMD = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs)
        cycles = avg["GRBM_GUI_ACTIVE"] / 8
        out["valu_issue_frac"] = 2 * avg["SQ_INSTS_VALU"] / (a.simds * cycles)
        if "valu_lane_utilization" in out:
            out["useful_valu_frac"] = out["valu_issue_frac"] * out["valu_lane_utilization"]
    if "TA_BUSY_avr" in avg and "GRBM_GUI_ACTIVE" in avg:
        out["ta_busy_frac"] = avg["TA_BUSY_avr"] / (avg["GRBM_GUI_ACTIVE"] / 8)
    if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_ACTIVE_INST_LDS" in avg:
        out["lds_bank_conflict_per_lds_cycle"] = avg["SQ_LDS_BANK_CONFLICT"] / max(1.0, avg["SQ_ACTIVE_INST_LDS"])
    print(json.dumps(out, indent=1))
    if a.write_traffic and "hbm_bytes_per_launch" in out:
        merge_record(a.write_traffic, {
            "workload": a.workload, "hbm_bytes_per_launch": int(out["hbm_bytes_per_launch"]),
            "hbm_read_bytes": int(out["hbm_read_bytes"]), "hbm_write_bytes": int(out["hbm_write_bytes"]),
            "counted_launch": a.counted_launch, "profile_dir": a.prof_dir,
            "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                      "FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM"})
    if a.write_binding:
        keys = ("valu_issue_frac", "valu_lane_utilization", "useful_valu_frac", "wave_cycle_split",
                "lds_bank_conflict_per_lds_cycle", "l2_hit_rate", "effective_clock_ghz", "ta_busy_frac")
        rec = {"workload": a.workload, "kernel_ns": round(ns_avg),
               **{k: out[k] for k in keys if k in out},
               "sq_insts_valu_per_launch": avg.get("SQ_INSTS_VALU"),
               "counted_launch": a.counted_launch, "profile_dir": a.prof_dir,
               "source": "rocprofv3 --pmc passes of tools/profile.sh (SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU, "
                         "SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, "
                         "SQ_LDS_BANK_CONFLICT, SQ_ACTIVE_INST_LDS, GRBM_GUI_ACTIVE, TCC_HIT/MISS, TA_BUSY)",
               "reading": "valu_issue_frac = 2 cycles x SQ_INSTS_VALU / (1024 SIMDs x kernel cycles of the counted "
                          "launch); useful_valu_frac = that x lane utilisation: the fraction of the chip's fp32 "
                          "lane-issue slots doing path-tracing work (DESIGN.md §6). bench.py re-derives both for "
                          "the timed launch (valu_issue_frac_timed) from the counted instructions"}
        merge_record(a.write_binding, rec)
    return 0


def merge_record(path, rec):
    """Add or replace rec (keyed by workload) in a {"records": [...]} file."""
    try:
        with open(path) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        doc = {}
    recs = [r for r in doc.get("records", [doc] if doc.get("workload") else []) if r.get("workload") != rec["workload"]]
    recs.append(rec)
    with open(path, "w") as f:
        json.dump({"records": recs}, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())
