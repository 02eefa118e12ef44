#!/usr/bin/env python3
"""Combine a run_profile.sh output directory into one summary JSON:
per-dispatch means of every --pmc pass for the dominant kernel, plus derived
per-record figures (instructions, HBM bytes with the gfx950 FETCH_SIZE x2
correction, effective shader clock = GRBM_GUI_ACTIVE / 8 XCDs / duration).
    python profiles/combine_pmc.py gpurun_out/prof_<tag> <kernel-substring> <records-per-dispatch> > profiles/<tag>_pmc_summary.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_pmc import summarize  # noqa: E402

root, kern, records = sys.argv[1], sys.argv[2], int(sys.argv[3])
out = {}
for p in ("pmc_sq1", "pmc_sq2", "pmc_fetch", "pmc_write"):
    out[p] = summarize(os.path.join(root, p), kern)
sq1, sq2 = out["pmc_sq1"], out["pmc_sq2"]
dur = sq2.get("_mean_dispatch_s") or sq1.get("_mean_dispatch_s")
out["derived"] = {
    "records_per_dispatch": records,
    "lds_insts_per_record": sq1["SQ_INSTS_LDS"] / records,
    "valu_insts_per_record": sq1["SQ_INSTS_VALU"] / records,
    "effective_clock_ghz": sq2["GRBM_GUI_ACTIVE"] / 8 / dur / 1e9,
    "valu_active_frac_of_wave_cycles": sq2["SQ_ACTIVE_INST_VALU"] / sq1["SQ_WAVE_CYCLES"],
    "hbm_bytes_per_record": (out["pmc_fetch"]["hbm_read_bytes_corrected"] + out["pmc_write"]["hbm_write_bytes"]) / records,
}
print(json.dumps(out, indent=1))
