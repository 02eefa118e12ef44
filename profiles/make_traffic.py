#!/usr/bin/env python3
"""Turn a run_profile.sh output directory into profiles/traffic_<config>.json:
per-record HBM bytes of the dominant kernel = (FETCH_SIZE x 2 + WRITE_SIZE)
per dispatch / records per dispatch (MI355X_MICROARCH.md: FETCH_SIZE counts
half the bytes of 16 B/lane streaming reads on gfx950, WRITE_SIZE is exact).
    python profiles/make_traffic.py gpurun_out/prof_<tag> <kernel-substring> <config> <records> <direction> <inner>
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_pmc import summarize  # noqa: E402

root, kern, config, records, direction, inner = sys.argv[1:7]
records, inner = int(records), int(inner)
f = summarize(os.path.join(root, "pmc_fetch"), kern)
w = summarize(os.path.join(root, "pmc_write"), kern)
rd = f["hbm_read_bytes_corrected"]
wr = w["hbm_write_bytes"]
# the sized L2->fabric read counters when the profile has them (calibrated
# per access shape by tools/probes/fetch_calib; FETCH_SIZE x 2 kept beside)
sized = None
if os.path.isdir(os.path.join(root, "pmc_rdreq")):
    sized = summarize(os.path.join(root, "pmc_rdreq"), kern).get("hbm_read_bytes_sized")
out = {"config": config, "direction": direction, "record_inner_bytes": inner, "kernel": kern,
       "records_per_dispatch": records, "hbm_read_bytes_per_dispatch": sized if sized else rd, "hbm_write_bytes_per_dispatch": wr,
       "hbm_bytes_per_record": ((sized if sized else rd) + wr) / records,
       "hbm_read_bytes_per_dispatch_fetch_x2": rd,
       "read_counters": ("TCC_EA0_RDREQ_{32B,64B,128B}_sum x size" if sized else "FETCH_SIZE x 2"),
       "source": os.path.basename(root.rstrip("/"))}
path = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"traffic_{config}.json")
with open(path, "w") as fh:
    json.dump(out, fh, indent=1)
print(json.dumps(out, indent=1))
