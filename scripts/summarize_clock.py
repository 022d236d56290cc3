"""Effective shader clock per dispatch from a rocprofv3 --pmc GRBM_GUI_ACTIVE
pass (counter_collection CSV): GRBM_GUI_ACTIVE is summed over the 8 XCDs, so
busy cycles = value / 8, and clock = busy cycles / the dispatch's wall time
(MI355X_MICROARCH.md, 'DVFS give-back'; within ~3% of the in-kernel clock on
dispatches of 10 ms or more; dispatches under 1 ms are skipped: the counter's
granularity makes their figure meaningless).

usage: python3 summarize_clock.py <counter_collection.csv> [title]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    rows = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
                continue
            d = int(r["Dispatch_Id"])
            rows[d] = (r["Kernel_Name"], float(r["Counter_Value"]),
                       (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    print(title)
    for d in sorted(rows):
        name, active, wall = rows[d]
        if wall < 1e-3:
            continue
        print("  dispatch %3d %-32s %8.3f ms  GRBM_GUI_ACTIVE %.4g  -> %.3f GHz"
              % (d, name[:32], wall * 1e3, active, active / 8.0 / wall / 1e9))


if __name__ == "__main__":
    main()
