"""Per-kernel duration summary of a rocprofv3 run: either the --stats CSV
(<dir>/*kernel_stats.csv) or the SQLite run_results.db rocprofv3 writes by default.
usage: python tools/kstats.py <prof dir> [name substring ...]"""
import csv
import glob
import os
import sqlite3
import sys


def rows(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if f:
        for r in csv.DictReader(open(f[0])):
            yield r["Name"], int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3
        return
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    q = ("select name, count(*), avg(end - start), sum(end - start) from kernels group by name "
         "order by sum(end - start) desc")
    for name, n, avg, tot in c.execute(q):
        yield name, n, avg / 1e3, tot / 1e3


def main():
    d, keys = sys.argv[1], sys.argv[2:]
    for name, n, avg, tot in rows(d):
        if keys and not any(k in name for k in keys):
            continue
        print(f"{avg:9.2f} us x {n:6d} = {tot / 1e3:9.2f} ms  {name[:100]}")


if __name__ == "__main__":
    main()
