"""Per-kernel median durations from a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv),
grouped by kernel name and grid size (so the 4096-state act forward is not mixed with the
32,768-state configs[3] launches of the same kernel).
usage: python tools/kmedians.py <prof dir> [name substring ...]"""
import collections
import csv
import glob
import os
import statistics
import sys


def main():
    d, keys = sys.argv[1], sys.argv[2:]
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if keys and not any(k in name for k in keys):
            continue
        grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
        g[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (name, grid), v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        print(f"{statistics.median(v):10.2f} us median  {len(v):6d} launches  grid {grid:>9}  {name[:90]}")


if __name__ == "__main__":
    main()
