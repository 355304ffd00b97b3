"""Per-kernel counter summary of the counter-only passes tools/pmc_h3.sh /
tools/pmc_syrk.sh write (p1: SQ cycles, p2: FETCH_SIZE + GRBM_GUI_ACTIVE,
p3: WRITE_SIZE + TCC hit/miss, p4: instruction counts).

usage: python tools/pmc_summary.py <pmc dir> <out.json> [kernel substrings...]

mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x 2.4 GHz x the dispatch's
duration in the same pass (End - Start timestamps)): the fraction of the
nominal dense MFMA peak; clock_ghz = GRBM_GUI_ACTIVE / 8 XCDs / the duration of
the dispatch in the SAME pass (p2; round 5 divided by p1's duration, which gave
clocks up to 7 GHz for microsecond kernels), and mfma_busy_at_clock the same
fraction at that clock. The GRBM quotient reads high on dispatches shorter than
~0.3 ms (MI355X_MICROARCH.md 'DVFS give-back'): below that, or above the part's
2.4 GHz, no clock is reported (clock_note says why); wait_*_frac = the SQ wait
counters over SQ_WAVE_CYCLES;
hbm_bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB; FETCH_SIZE doubled per
MI355X_MICROARCH.md's gfx950 note); all per launch (mean over launches).
"""
import collections
import csv
import json
import os
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in ("p1", "p2", "p3", "p4"):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        seen = set()
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Dispatch_Id"] not in seen:   # one duration per dispatch, per pass
                seen.add(r["Dispatch_Id"])
                agg[r["Kernel_Name"]]["duration_ns_" + p].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main():
    d, out = sys.argv[1], sys.argv[2]
    keys = sys.argv[3:]
    res = {}
    for k, c in load(d).items():
        if keys and not any(s in k for s in keys):
            continue
        row = {"counters": c}
        c["duration_ns"] = c.get("duration_ns_p1", 0.0)
        cyc = c["duration_ns"] * 2.4
        if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            row["mfma_busy"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc)
        d2 = c.get("duration_ns_p2", 0.0)
        if d2 and "GRBM_GUI_ACTIVE" in c:   # summed over the 8 XCDs; pass p2's own duration
            clk = c["GRBM_GUI_ACTIVE"] / 8.0 / d2
            if d2 < 3e5:
                row["clock_note"] = f"no clock: dispatch {d2 / 1e3:.1f} us < 0.3 ms (GRBM quotient reads high)"
            elif clk > 2.4:
                row["clock_note"] = f"no clock: GRBM quotient {clk:.2f} GHz above the part's 2.4 GHz"
            else:
                row["clock_ghz"] = clk
                if "mfma_busy" in row:
                    row["mfma_busy_at_clock"] = row["mfma_busy"] * 2.4 / clk
        if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
            row["wait_inst_any_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
            row["wait_lds_frac"] = c.get("SQ_WAIT_INST_LDS", 0) / c["SQ_WAVE_CYCLES"]
            row["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            row["hbm_bytes"] = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
        if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c and c["SQ_LDS_IDX_ACTIVE"]:
            row["lds_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
        if "TCC_HIT" in c and "TCC_MISS" in c and (c["TCC_HIT"] + c["TCC_MISS"]):
            row["l2_hit"] = c["TCC_HIT"] / (c["TCC_HIT"] + c["TCC_MISS"])
        res[k.replace("void snk::", "").replace("snk::", "")[:90]] = row
    json.dump(res, open(out, "w"), indent=1)
    for k, r in res.items():
        print(k[:60], {x: round(y, 3) for x, y in r.items() if x != "counters" and isinstance(y, float)})


if __name__ == "__main__":
    main()
