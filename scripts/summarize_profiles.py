#!/usr/bin/env python3
"""scripts/summarize_profiles.py -- turn scripts/profile_round.sh's raw rocprofv3
output (gpurun_out/prof/) into the committed summaries under profiles/:

  profiles/<round>_bench_kernel_stats.csv        kernel stats of `python3 bench.py`
  profiles/<round>_bench_under_rocprof.json      that run's bench JSON line
  profiles/<round>_pmc_fetch_size_bench.csv      raw FETCH_SIZE pass of bench.py
  profiles/<round>_pmc_fetch_size.csv            raw FETCH_SIZE calibration pass
  profiles/<round>_traffic.json                  HBM bytes per launch, latency kernel
                                                 (bench.py reads it for roofline.traffic)
  profiles/<round>_saturation_kernel_stats.csv   kernel stats of the saturation lines
  profiles/<round>_saturation_traffic.json       HBM bytes per launch, coalesced kernel

FETCH_SIZE is corrected as MI355X_MICROARCH.md's HBM section prescribes: on
gfx950 it tallies 128-B requests at 64 B, so the factor is calibrated in the
same session on a 4 GiB coalesced read (ubench k_stream_read) and applied.
Runs in the build container (no GPU).
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RAW = os.path.join(ROOT, "gpurun_out", "prof")
PROF = os.path.join(ROOT, "profiles")


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def fetch_kib(path, kernel_prefix):
    return [float(r["Counter_Value"]) for r in rows(path)
            if r["Kernel_Name"].startswith(kernel_prefix) and r["Counter_Name"] == "FETCH_SIZE"]


def main(rnd):
    cal_path = os.path.join(RAW, "pmc_calib", "pmc_counter_collection.csv")
    cal_kib = fetch_kib(cal_path, "k_stream_read")
    cal_bytes = 4 << 30
    factor = cal_bytes / (statistics.median(cal_kib) * 1024.0)

    bench_pmc = os.path.join(RAW, "pmc_bench", "pmc_counter_collection.csv")
    pc_kib = fetch_kib(bench_pmc, "qsmd5_batch_pc64_kernel")
    alg = 512 * 10485760
    hbm = statistics.median(pc_kib) * 1024.0 * factor
    traffic = {
        "workload": "batch512x10MiB", "kernel": "qsmd5_batch_pc64_kernel",
        "source": "rocprofv3 --pmc FETCH_SIZE -- python3 bench.py --no-cpu-baseline --no-config5 "
                  "--steps 2 --warmup 1 (own pass, no trace domains); raw: profiles/%s_pmc_fetch_size_bench.csv" % rnd,
        "fetch_size_kib_raw_per_launch": statistics.median(pc_kib), "launches": len(pc_kib),
        "calibration": {"kernel": "k_stream_read (ubench/ubench_md5 calib): coalesced 16 B/lane "
                                  "dwordx4 read of 4 GiB",
                        "fetch_size_kib_raw": statistics.median(cal_kib), "bytes_read": cal_bytes,
                        "factor": round(factor, 5), "raw": "profiles/%s_pmc_fetch_size.csv" % rnd},
        "hbm_read_bytes_per_launch": int(round(hbm)), "algorithmic_bytes_per_launch": alg,
        "ratio_traffic_to_algorithmic": round(hbm / alg, 5),
    }
    json.dump(traffic, open(os.path.join(PROF, "%s_traffic.json" % rnd), "w"), indent=1)

    # saturation: the coalesced kernel, 131072 x 64 KiB launches then 131072 x 256 KiB
    sat_pmc = os.path.join(RAW, "pmc_sat", "pmc_counter_collection.csv")
    co_kib = fetch_kib(sat_pmc, "qsmd5_batch_coal_kernel")
    trace = [r for r in rows(os.path.join(RAW, "sat", "sat_kernel_trace.csv"))
             if r["Kernel_Name"].startswith("qsmd5_batch_coal_kernel")]
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in trace]
    # Since round 5 each size runs untimed warm-up launches first (a time
    # budget, so their count varies): split the two sizes by magnitude (4x
    # apart) and keep each size's last 11 dispatches, the timed ones.
    def split(vals, keep=11):
        cut = (min(vals) * max(vals)) ** 0.5
        return [v for v in vals if v < cut][-keep:], [v for v in vals if v >= cut][-keep:]
    kib64, kib256 = split(co_kib)
    d64, d256 = split(durs)
    out = []
    for label, L, kib, d in (("131072x64KiB", 65536, kib64, d64),
                             ("131072x256KiB", 262144, kib256, d256)):
        a = 131072 * L
        b = statistics.median(kib) * 1024.0 * factor
        med = statistics.median(d)
        out.append({"workload": label, "kernel": "qsmd5_batch_coal_kernel", "launches": len(d),
                    "rocprof_ms_median": round(med, 4), "rocprof_ms_mean": round(statistics.mean(d), 4),
                    "algorithmic_bytes_per_launch": a, "hbm_read_bytes_per_launch": int(round(b)),
                    "ratio_traffic_to_algorithmic": round(b / a, 5),
                    "achieved_GBps_median": round(a / (med * 1e-3) / 1e9, 1),
                    "frac_of_8TBps": round(a / (med * 1e-3) / 8e12, 4)})
    json.dump({"calibration_factor": round(factor, 5), "lines": out},
              open(os.path.join(PROF, "%s_saturation_traffic.json" % rnd), "w"), indent=1)

    shutil.copy(os.path.join(RAW, "bench", "bench_kernel_stats.csv"),
                os.path.join(PROF, "%s_bench_kernel_stats.csv" % rnd))
    shutil.copy(os.path.join(RAW, "sat", "sat_kernel_stats.csv"),
                os.path.join(PROF, "%s_saturation_kernel_stats.csv" % rnd))
    shutil.copy(bench_pmc, os.path.join(PROF, "%s_pmc_fetch_size_bench.csv" % rnd))
    shutil.copy(cal_path, os.path.join(PROF, "%s_pmc_fetch_size.csv" % rnd))
    line = [l for l in open(os.path.join(RAW, "bench.json")) if l.startswith("{")][-1]
    open(os.path.join(PROF, "%s_bench_under_rocprof.json" % rnd), "w").write(line)
    print(json.dumps(traffic["ratio_traffic_to_algorithmic"]), json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
