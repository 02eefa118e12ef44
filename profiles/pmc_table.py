#!/usr/bin/env python3
"""Summarise tools/prof_pmc.sh output: per counter, the mean over the
dispatches of the named kernel (substring), one JSON object per tag.
    python profiles/pmc_table.py gpurun_out/pmc_<tag> <kernel-substring>"""
import csv, glob, json, os, sys
from collections import defaultdict

def load(d, kern):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for row in csv.DictReader(open(f)):
            if kern not in row.get("Kernel_Name", ""):
                continue
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (disp, name), v in per.items():
            vals[name].append(v)
    return {k: sum(v) / len(v) for k, v in sorted(vals.items())}

if __name__ == "__main__":
    out = {}
    for d in sorted(glob.glob(os.path.join(sys.argv[1], "*"))):
        if os.path.isdir(d):
            out.update(load(d, sys.argv[2]))
    print(json.dumps(out, indent=1))
