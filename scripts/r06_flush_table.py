"""Markdown tables for INTEGRATION.md §3 from a flush sweep
(scripts/r06_flush_sweep.sh output): the reference's own flush loop beside
the staged binding, at qsfs's default -n 5.  Wall = the best pass; uploader
wait, host CPU-s and the loop's own split are from that pass where the
harness reports them per pass (wall, CPU) and from the last pass otherwise.

usage: python3 scripts/r06_flush_table.py profiles/r06_flush_sweep_final.jsonl
"""
import json
import sys


def main():
    rows = {}
    for line in open(sys.argv[1]):
        r = json.loads(line)
        rows[r["case"]] = r

    def cell(case):
        r = rows.get(case)
        if not r:
            return None
        i = r["wall_s_runs"].index(min(r["wall_s_runs"]))
        return r, r["wall_s_runs"][i], r["cpu_s_runs"][i]

    flows = [("reference_sync", "reference loop, sync (qsfs's `File::Flush`)"),
             ("reference_async5", "reference loop on a 5-thread executor (`-M` would-be)"),
             ("staged_whole", "staged binding, whole file in one pre-hash"),
             ("staged_ramp_noahead", "staged binding, ramp 4…64, no read-ahead"),
             ("staged_ramp", "**staged binding, ramp 4…64 (the default)**")]
    print("| 10 MiB parts | uploads | flow | wall | vs reference | uploader waited | loop reads | host CPU-s | waves GPU / CPU |")
    print("|---|---|---|---|---|---|---|---|---|")
    for P in (128, 512):
        for U in (0, 10):
            ref = cell("reference_sync_u%d_P%d" % (U, P))
            for key, label in flows:
                c = cell("%s_u%d_P%d" % (key, U, P))
                if not c:
                    continue
                r, wall, cpu = c
                vs = "—" if key == "reference_sync" else "%.1f× faster" % (ref[1] / wall) if ref else "?"
                waves = "%d / %d" % (r["gpu_waves"], r["cpu_waves"]) if not key.startswith("reference") else \
                    "0 / %d (md5 per part)" % r["parts"]
                print("| %d | %s | %s | %.3f s | %s | %.3f s | %.3f s | %.2f | %s |" % (
                    P, "return at once" if U == 0 else "10 ms each (%.2f s)" % (P * 0.01), label, wall, vs,
                    r["wait_s"], r["loop_read_s"], cpu, waves))
    print()
    for case in ("staged_whole_auto_P128", "staged_whole_gpu_P128", "staged_whole_auto_P512", "staged_whole_gpu_P512",
                 "staged_4files_ramp_u0_P128", "staged_4files_whole_u0_P128", "reference_sync_4files_u0_P128"):
        c = cell(case)
        if c:
            r, wall, cpu = c
            print("- %s: %.3f s, %.2f CPU-s, golden %s, traces %s" % (case, wall, cpu, r["golden_ok"],
                  [(t["backend"], round(t["total_ms"])) for t in r["traces"]][:6]))


if __name__ == "__main__":
    main()
