#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs for one kernel: mean counter value per
dispatch, plus derived HBM bytes (FETCH_SIZE x2 per the gfx950 correction in
MI355X_MICROARCH.md, WRITE_SIZE as is; both in KiB)."""
import csv
import glob
import json
import sys
from collections import defaultdict


def summarize(root, pattern):
    vals = defaultdict(lambda: defaultdict(float))
    durs = {}
    for path in glob.glob(f"{root}/run_counter_collection.csv") + glob.glob(f"{root}/*/run_counter_collection.csv"):
        for row in csv.DictReader(open(path)):
            if pattern not in row["Kernel_Name"]:
                continue
            key = (path, row["Dispatch_Id"])
            vals[key][row["Counter_Name"]] += float(row["Counter_Value"])
            durs[key] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    per = defaultdict(list)
    for key, cs in vals.items():
        for c, v in cs.items():
            per[c].append(v)
    out = {c: sum(v) / len(v) for c, v in per.items()}
    out["_dispatches"] = len(vals)
    out["_mean_dispatch_s"] = sum(durs.values()) / max(1, len(durs))
    if "FETCH_SIZE" in out:
        out["hbm_read_bytes_corrected"] = out["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in out:
        out["hbm_write_bytes"] = out["WRITE_SIZE"] * 1024
    # L2 -> fabric reads by request size (tools/probes/fetch_calib: the sized
    # sum is the calibrated byte count for every access shape of the kernels)
    sized = [out.get(f"TCC_EA0_RDREQ_{s}_sum") for s in ("32B", "64B", "128B")]
    if None not in sized:
        out["hbm_read_bytes_sized"] = 32 * sized[0] + 64 * sized[1] + 128 * sized[2]
    return out


if __name__ == "__main__":
    print(json.dumps(summarize(sys.argv[1], sys.argv[2]), indent=1))
