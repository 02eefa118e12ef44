#!/usr/bin/env python3
"""Combine a run_profile.sh output directory into one summary JSON:
per-dispatch means of every --pmc pass for the dominant kernel, plus derived
per-record figures (instructions, HBM bytes with the gfx950 FETCH_SIZE x2
correction, effective shader clock = GRBM_GUI_ACTIVE / 8 XCDs / duration) and
the busy fraction of the LDS array and the VALU:
    lds_busy  = SQ_LDS_IDX_ACTIVE (LDS-array cycles, all CUs) / (CUs x cycles)
    valu_busy = SQ_ACTIVE_INST_VALU (quad-cycles) x 4 / (4 SIMDs x CUs x cycles)
    [--valu-ticks T: the kernel's hot-loop mean issue cost per VALU instruction
     (tools/valu_mix.py over the per-class costs of tools/rate_probe.hip); the
     ceiling file then charges T instead of 4 cycles per instruction and keeps
     the 4-cycle figure as valu_x4]
(a wave64 integer VALU instruction holds its SIMD for 4 cycles: tools/chacha_probe.hip
measures the ChaCha20 block, ~990 such instructions, at the same chip-wide rate
with 1, 2, 3 or 4 waves per SIMD -- 2.0-2.3 TB/s of keystream -- i.e. the VALU,
not latency, is saturated; SQ_ACTIVE_INST_VALU = SQ_INSTS_VALU quad-cycles)
    python profiles/combine_pmc.py gpurun_out/prof_<tag> <kernel-substring> <records-per-dispatch> \
        [--ceiling profiles/ceiling_<config>.json] > profiles/<tag>_pmc_summary.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_pmc import summarize  # noqa: E402

CUS = 256
args = sys.argv[1:]
ceil_path = None
valu_ticks = None
if "--valu-ticks" in args:
    k = args.index("--valu-ticks")
    valu_ticks = float(args[k + 1])
    del args[k:k + 2]
if "--ceiling" in args:
    k = args.index("--ceiling")
    ceil_path = args[k + 1]
    del args[k:k + 2]
root, kern, records = args[0], args[1], int(args[2])
out = {}
for p in ("pmc_sq1", "pmc_sq2", "pmc_sq3", "pmc_fetch", "pmc_write", "pmc_rdreq", "pmc_tcp", "pmc_tcc"):
    if os.path.isdir(os.path.join(root, p)):
        out[p] = summarize(os.path.join(root, p), kern)
sq1, sq2 = out["pmc_sq1"], out["pmc_sq2"]
dur = sq2.get("_mean_dispatch_s") or sq1.get("_mean_dispatch_s")
cycles = sq2["GRBM_GUI_ACTIVE"] / 8                      # per XCD = shader clock cycles of the dispatch
d = {
    "records_per_dispatch": records,
    "lds_insts_per_record": sq1["SQ_INSTS_LDS"] / records,
    "valu_insts_per_record": sq1["SQ_INSTS_VALU"] / records,
    "effective_clock_ghz": cycles / dur / 1e9,
    "valu_active_frac_of_wave_cycles": sq2["SQ_ACTIVE_INST_VALU"] / sq1["SQ_WAVE_CYCLES"],
    "valu_busy_frac": sq2["SQ_ACTIVE_INST_VALU"] * 4 / (4 * CUS * cycles),
}
if "pmc_sq3" in out:
    sq3 = out["pmc_sq3"]
    c3 = sq3["GRBM_GUI_ACTIVE"] / 8
    d["lds_busy_frac"] = sq3["SQ_LDS_IDX_ACTIVE"] / (CUS * c3)
    d["lds_cycles_per_record"] = sq3["SQ_LDS_IDX_ACTIVE"] / records     # summed over CUs: per record
    d["lds_bank_conflict_frac"] = sq3["SQ_LDS_BANK_CONFLICT"] / max(1.0, sq3["SQ_LDS_IDX_ACTIVE"])
if "pmc_fetch" in out and "pmc_write" in out:
    d["hbm_bytes_per_record"] = (out["pmc_fetch"]["hbm_read_bytes_corrected"] +
                                 out["pmc_write"]["hbm_write_bytes"]) / records
    d["hbm_read_bytes_per_record_fetch_x2"] = out["pmc_fetch"]["hbm_read_bytes_corrected"] / records
    d["hbm_write_bytes_per_record"] = out["pmc_write"]["hbm_write_bytes"] / records
if "pmc_rdreq" in out and "hbm_read_bytes_sized" in out["pmc_rdreq"] and "pmc_write" in out:
    # L2->fabric reads by request size (32/64/128 B): the byte count that
    # tools/probes/fetch_calib pins for every access shape (profiles/archive/r04a)
    d["hbm_read_bytes_per_record_sized"] = out["pmc_rdreq"]["hbm_read_bytes_sized"] / records
    d["hbm_bytes_per_record_sized"] = (out["pmc_rdreq"]["hbm_read_bytes_sized"] +
                                       out["pmc_write"]["hbm_write_bytes"]) / records
if "pmc_tcp" in out:
    # vector L1 (TCP): accesses, the reads it sends to L2, and its address
    # translation (UTCL1) hits / misses
    t = out["pmc_tcp"]
    acc = t.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0.0)
    d["tcp_accesses_per_record"] = acc / records
    d["tcp_l2_reads_per_record"] = t.get("TCP_TCC_READ_REQ_sum", 0.0) / records
    tr = t.get("TCP_UTCL1_TRANSLATION_HIT_sum", 0.0) + t.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0.0)
    d["utcl1_miss_frac"] = t.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0.0) / max(1.0, tr)
    d["utcl1_misses_per_record"] = t.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0.0) / records
if "pmc_tcc" in out:
    t = out["pmc_tcc"]
    h, m = t.get("TCC_HIT_sum", 0.0), t.get("TCC_MISS_sum", 0.0)
    d["l2_hit_frac"] = h / max(1.0, h + m)
    d["l2_requests_per_record"] = (h + m) / records
    d["l2_dram_reads_per_record"] = t.get("TCC_EA0_RDREQ_DRAM_sum", 0.0) / records
out["derived"] = d
print(json.dumps(out, indent=1))
if ceil_path:
    valu = d["valu_busy_frac"] * (valu_ticks / 4 if valu_ticks else 1.0)
    units = {"lds": d.get("lds_busy_frac", 0.0), "valu": valu}
    lim = max(units, key=units.get)
    extra = {}
    if valu_ticks:
        extra = {"valu_x4": round(d["valu_busy_frac"], 4),
                 "valu_model": f"SQ_ACTIVE_INST_VALU x {valu_ticks} cycles (hot-loop mix, tools/valu_mix.py)"}
    with open(ceil_path, "w") as f:
        json.dump({"limiter": lim, "limiter_busy_frac": round(units[lim], 4),
                   "units": {k: round(v, 4) for k, v in units.items()}, **extra,
                   "effective_clock_ghz": round(d["effective_clock_ghz"], 3),
                   "lds_bank_conflict_frac": round(d.get("lds_bank_conflict_frac", 0.0), 5),
                   "source": os.path.basename(os.path.normpath(root)) + " (rocprofv3 --pmc, " + kern + ")"}, f, indent=1)
        f.write("\n")
