#!/usr/bin/env python3
"""profiles/traffic_<config>.json for a run whose step is several kernels
(c4 / c4s: the GCM kernel over the AES records, the ChaCha20-Poly1305 kernel
over the others, plus the bucket pass): HBM bytes per record = the sum over
the step's kernels of (FETCH_SIZE x 2 + WRITE_SIZE) per dispatch (gfx950
correction, MI355X_MICROARCH.md) / records per step.
    python profiles/make_mix_traffic.py gpurun_out/prof_<tag> <config> <records> <direction> <inner> <kernel-substr>...
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_pmc import summarize  # noqa: E402

root, config, records, direction, inner = sys.argv[1:6]
records, inner = int(records), int(inner)
per, rd, wr, rs = {}, 0.0, 0.0, 0.0
have_sized = os.path.isdir(os.path.join(root, "pmc_rdreq"))
for k in sys.argv[6:]:
    f = summarize(os.path.join(root, "pmc_fetch"), k)
    w = summarize(os.path.join(root, "pmc_write"), k)
    per[k] = {"read": f["hbm_read_bytes_corrected"], "write": w["hbm_write_bytes"], "dispatches": f["_dispatches"],
              "mean_dispatch_s": f["_mean_dispatch_s"]}
    rd += f["hbm_read_bytes_corrected"]
    wr += w["hbm_write_bytes"]
    if have_sized:
        s = summarize(os.path.join(root, "pmc_rdreq"), k)
        per[k]["read_sized"] = s.get("hbm_read_bytes_sized")
        rs += s.get("hbm_read_bytes_sized") or 0.0
out = {"config": config, "direction": direction, "record_inner_bytes": inner,
       "kernel": " + ".join(sys.argv[6:]) + " (one dispatch each per step)", "records_per_dispatch": records,
       "hbm_read_bytes_per_dispatch": rd, "hbm_write_bytes_per_dispatch": wr,
       "hbm_bytes_per_record": (rd + wr) / records, "per_kernel": per,
       **({"hbm_read_bytes_per_dispatch_sized": rs, "hbm_bytes_per_record_sized": (rs + wr) / records,
           "read_counters": "TCC_EA0_RDREQ_{32B,64B,128B}_sum x size (calibrated, tools/probes/fetch_calib); "
                            "FETCH_SIZE x 2 beside it"} if have_sized else {}),
       "source": os.path.basename(root.rstrip("/")) + f" ({records} records per step)"}
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), f"traffic_{config}.json"), "w") as fh:
    json.dump(out, fh, indent=1)
    fh.write("\n")
print(json.dumps(out, indent=1))
