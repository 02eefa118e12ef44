#!/usr/bin/env python3
"""Markdown table of one round's bench rows (the JSON lines tools/gpu_r06.sh
rows writes, copied to profiles/<round>/rows/):
    python profiles/rows_table.py profiles/r06/rows"""
import glob
import json
import os
import sys

root = sys.argv[1]
print("| row | value | frac of HBM | kernel ms | CPU baseline (EVP / port) | file |")
print("|---|---|---|---|---|---|")
for f in sorted(glob.glob(os.path.join(root, "*.json"))):
    lines = [ln for ln in open(f).read().splitlines() if ln.startswith("{")]
    if not lines:
        continue
    name = os.path.basename(f)[:-5]
    for ln in lines:
        d = json.loads(ln)
        if "metric" not in d:
            print(f"| {name} | {json.dumps(d)} | | | | `{f}` |")
            continue
        r = d.get("roofline") or {}
        cpu = d.get("cpu_baseline") or {}
        legs = {lg.get("leg"): lg.get("value") for lg in cpu.get("legs", [])} or {cpu.get("leg"): cpu.get("value")}
        label = name if len(lines) == 1 else f"{name} ({d['metric'].split(' throughput')[0].split()[-1]})"
        print(f"| {label} | {d['value']} {d.get('unit', '')} | {r.get('frac', '')} | {r.get('kernel_ms_avg', '')} | "
              f"{legs.get('evp', '-')} / {legs.get('port', '-')} | `{f}` |")
