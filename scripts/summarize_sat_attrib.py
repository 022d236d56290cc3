#!/usr/bin/env python3
"""scripts/summarize_sat_attrib.py -- summary of scripts/r05_sat_attrib.sh
(VERDICT r04 item 5): splits the coalesced kernel's loss at 131072 x 64 KiB
against 131072 x 256 KiB into clock, per-chain instructions, and the part of
the dispatch in which waves are not alive (ramp + tail).

Inputs: gpurun_out/r05_sat/{satsweep.jsonl, trace/, pmc_sat64_[ab]/, pmc_sat256_[ab]/}.
Output: profiles/r05_sat_attribution.json (+ the raw CSVs copied beside it).

Units (MI355X_MICROARCH.md): GRBM_GUI_ACTIVE is summed over the 8 XCDs, so
GRBM_GUI_ACTIVE / 8 = the dispatch's busy cycles; SQ_WAVE_CYCLES and
SQ_ACTIVE_INST_VALU count quad-cycles (x4 = cycles); SQ_INSTS_* count
wave-instructions.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RAW = os.path.join(ROOT, "gpurun_out", "r05_sat")
TAG = sys.argv[1] if len(sys.argv) > 1 else ""  # suffix of the profiles/ names (e.g. "_warm")
PROF = os.path.join(ROOT, "profiles")
KERNEL = "qsmd5_batch_coal_kernel"
N = 131072
LAUNCHES = 11  # bench_configs.saturation: max(reps, 10) + 1 launches per size


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def one(pattern):
    hits = sorted(glob.glob(os.path.join(RAW, pattern), recursive=True))
    if not hits:
        raise SystemExit("missing: " + pattern)
    return hits[0]


def pmc(name):
    """Per-dispatch counters of the coalesced kernel: {dispatch: {counter: value, 'ns': wall}}."""
    out = {}
    for r in rows(one("pmc_%s/**/pmc_counter_collection.csv" % name)):
        if not r["Kernel_Name"].startswith(KERNEL):
            continue
        d = out.setdefault(int(r["Dispatch_Id"]), {})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    disp = [out[k] for k in sorted(out)][-(LAUNCHES - 1):]  # the timed launches (warm-up ones first)
    return disp


def med(disp, key):
    return statistics.median(d[key] for d in disp)


def size_line(cfg, L):
    a, b = pmc(cfg + "_a"), pmc(cfg + "_b")
    waves = N // 64
    blocks = waves * (L // 64)  # wave-blocks: one 64-B block in each of a wave's 64 chains
    busy = med(a, "GRBM_GUI_ACTIVE") / 8.0
    ns_a = statistics.median(d["ns"] for d in a)
    life = 4.0 * med(a, "SQ_WAVE_CYCLES") / med(a, "SQ_WAVES")
    valu = med(b, "SQ_INSTS_VALU")
    salu = med(b, "SQ_INSTS_SALU")
    return {
        "chunk_KiB": L // 1024,
        "dispatches": len(a),
        "wall_ms_pmc_pass": round(ns_a / 1e6, 4),
        "clock_GHz": round(busy / ns_a, 4),
        "busy_cycles": round(busy),
        "waves": med(a, "SQ_WAVES"),
        "mean_wave_life_cycles": round(life),
        "wave_life_over_dispatch": round(life / busy, 4),
        "valu_per_wave_block": round(valu / blocks, 2),
        "salu_per_wave_block": round(salu / blocks, 2),
        "valu_active_over_wave_cycles": round(med(b, "SQ_ACTIVE_INST_VALU") / med(a, "SQ_WAVE_CYCLES"), 4),
        "wait_inst_any_over_wave_cycles": round(med(b, "SQ_WAIT_INST_ANY") / med(a, "SQ_WAVE_CYCLES"), 4),
        "sq_busy_cycles": med(a, "SQ_BUSY_CYCLES"),
    }


def main():
    sweep = [json.loads(l) for l in open(os.path.join(RAW, "satsweep.jsonl")) if l.strip()]
    pts = []
    for r in sweep:
        L = int(r["workload"].split(" x ")[1].split(" KiB")[0]) * 1024
        pts.append((L, r["kernel_ms_median"], r["frac_of_hbm_peak"]))
    # least squares t = a + b * L over the sweep
    xs, ys = [p[0] / 1024 for p in pts], [p[1] for p in pts]
    mx, my = statistics.mean(xs), statistics.mean(ys)
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    a = my - b * mx
    trace = rows(one("trace/**/sat_kernel_trace.csv"))
    # each size fills its chunks (qsmd5_lcg_fill_kernel) before its launches:
    # the fills separate the sizes' runs; the last LAUNCHES - 1 of a run are
    # the timed launches (warm-up ones come first)
    runs, cur = [], []
    for r in sorted(trace, key=lambda r: int(r["Start_Timestamp"])):
        if r["Kernel_Name"].startswith("qsmd5_lcg_fill"):
            if cur:
                runs.append(cur)
            cur = []
        elif r["Kernel_Name"].startswith(KERNEL):
            cur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    if cur:
        runs.append(cur)
    trace_ms = [round(statistics.median(r[-(LAUNCHES - 1):]), 4) for r in runs]
    s64, s256 = size_line("sat64", 64 * 1024), size_line("sat256", 256 * 1024)
    # The 64 KiB dispatch against 1/4 of the 256 KiB one (same bytes per chain
    # ratio): how many of its cycles each mechanism explains.
    t64 = s64["busy_cycles"] / s64["clock_GHz"]  # ns
    t256q = s256["busy_cycles"] / s256["clock_GHz"] / 4.0
    deficit_ns = t64 - t256q
    clock_ns = s64["busy_cycles"] / s64["clock_GHz"] - s64["busy_cycles"] / s256["clock_GHz"]
    dead = lambda s: 1.0 - s["wave_life_over_dispatch"]
    ramp_tail_ns = (dead(s64) - dead(s256)) * t64
    insts_ns = (s64["valu_per_wave_block"] / s256["valu_per_wave_block"] - 1.0) * t64 * s64["wave_life_over_dispatch"]
    out = {
        "what": "coalesced kernel, 131072 chains, device-resident: where 64 KiB chunks lose against 256 KiB",
        "sweep_hip_events": [{"chunk_KiB": p[0] // 1024, "kernel_ms_median": p[1], "frac_of_8TBps": p[2]} for p in pts],
        "fit_ms": {"a_per_launch": round(a, 4), "b_per_KiB": round(b, 6),
                   "note": "t(L) = a + b * L over the sweep's HIP-event medians"},
        "trace_ms_median_by_size": dict(zip([p[0] // 1024 for p in pts], trace_ms)),
        "pmc": {"64KiB": s64, "256KiB": s256},
        "attribution_ns": {
            "deficit": round(deficit_ns), "clock": round(clock_ns), "ramp_and_tail": round(ramp_tail_ns),
            "per_chain_instructions": round(insts_ns),
            "rest": round(deficit_ns - clock_ns - ramp_tail_ns - insts_ns),
            "note": "64 KiB dispatch time minus 1/4 of the 256 KiB one; clock = its cycles at 256 KiB's clock; "
                    "ramp_and_tail = the extra share of the dispatch with no wave alive (1 - mean wave life / "
                    "busy cycles); per_chain_instructions = extra VALU per wave-block (prologue, finish) at "
                    "the 64 KiB VALU rate",
        },
    }
    json.dump(out, open(os.path.join(PROF, "r05_sat_attribution%s.json" % TAG), "w"), indent=1)
    for name in ("sat64_a", "sat64_b", "sat256_a", "sat256_b"):
        shutil.copy(one("pmc_%s/**/pmc_counter_collection.csv" % name),
                    os.path.join(PROF, "r05_sat_pmc_%s%s.csv" % (name, TAG)))
    shutil.copy(one("trace/**/sat_kernel_stats.csv"), os.path.join(PROF, "r05_sat_kernel_stats%s.csv" % TAG))
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
