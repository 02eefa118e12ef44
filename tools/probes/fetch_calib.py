#!/usr/bin/env python3
"""Combine tools/probes/fetch_calib's known line bytes with the counters of
rocprofv3 --pmc passes over it: per kernel shape, the factor by which the
counted bytes must be multiplied to give the bytes of the lines touched.

    python tools/probes/fetch_calib.py <expected.json> <pmc_dir> [<pmc_dir> ...]

A pmc dir holds run_counter_collection.csv of one pass (FETCH_SIZE, WRITE_SIZE,
or raw TCC_EA0_* counters).  FETCH_SIZE / WRITE_SIZE are in KiB."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def counters(d):
    vals = defaultdict(lambda: defaultdict(float))
    for path in glob.glob(os.path.join(d, "run_counter_collection.csv")) + \
            glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for row in csv.DictReader(open(path)):
            vals[(row["Kernel_Name"].split("(")[0], row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
    per = defaultdict(lambda: defaultdict(list))
    for (k, _), cs in vals.items():
        for c, v in cs.items():
            per[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}


def main():
    exp = json.load(open(sys.argv[1]))["kernels"]
    got = defaultdict(dict)
    for d in sys.argv[2:]:
        for k, cs in counters(d).items():
            got[k].update(cs)
    out = {}
    for k, e in exp.items():
        c = got.get(k, {})
        row = {"line_bytes": e["line_bytes"], "result_write_bytes": e["result_write_bytes"]}
        if "FETCH_SIZE" in c:
            fb = c["FETCH_SIZE"] * 1024
            row["FETCH_SIZE_bytes"] = fb
            if not k.startswith("calib_w_"):
                row["fetch_factor"] = round(e["line_bytes"] / fb, 4) if fb else None
        if "WRITE_SIZE" in c:
            wb = c["WRITE_SIZE"] * 1024
            row["WRITE_SIZE_bytes"] = wb
            want = e["line_bytes"] if k.startswith("calib_w_") else e["result_write_bytes"]
            row["write_factor"] = round(want / wb, 4) if wb else None
        for name, v in c.items():
            if name.startswith("TCC_"):
                row[name] = v
        n32, n64, n128 = (c.get(f"TCC_EA0_RDREQ_{s}_sum") for s in ("32B", "64B", "128B"))
        if None not in (n32, n64, n128):
            sized = 32 * n32 + 64 * n64 + 128 * n128
            row["rdreq_sized_bytes"] = sized
            if not k.startswith("calib_w_") and sized:
                row["rdreq_sized_factor"] = round(e["line_bytes"] / sized, 4)
        out[k] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
