"""HBM traffic per launch of one kernel from counter-only rocprofv3 passes.

usage: python tools/traffic.py <pmc dir> <kernel substring> <out.json> [algorithmic bytes]
<pmc dir> holds p2/run_counter_collection.csv (FETCH_SIZE) and
p3/run_counter_collection.csv (WRITE_SIZE), as tools/pmc_h3.sh writes them.
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes
of 16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM section), so it is
doubled; WRITE_SIZE is taken as is.
"""
import csv
import json
import sys


def avg(path, counter, kern):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
         if r["Counter_Name"] == counter and kern in r["Kernel_Name"]]
    if not v:
        raise SystemExit(f"no {counter} rows for {kern} in {path}")
    name = next(r["Kernel_Name"] for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"])
    return sum(v) / len(v), len(v), name


def main():
    d, kern, out = sys.argv[1:4]
    alg = float(sys.argv[4]) if len(sys.argv) > 4 else None
    f, nf, name = avg(f"{d}/p2/run_counter_collection.csv", "FETCH_SIZE", kern)
    w, nw, _ = avg(f"{d}/p3/run_counter_collection.csv", "WRITE_SIZE", kern)
    res = {"kernel": name.replace("void ", "").replace("snk::", ""), "fetch_kib": f, "write_kib": w, "launches": [nf, nw],
           "bytes_per_launch": (2.0 * f + w) * 1024.0, "algorithmic_bytes_per_launch": alg,
           "how": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes), per-launch mean; "
                  "FETCH_SIZE x2 (gfx950 wide-read tally), KiB -> bytes"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
