#!/usr/bin/env python3
"""DESIGN.md §4 / §5 tables from one sweep's bench lines (profiles/<round>/rows):
    python profiles/design_tables.py profiles/r06/rows roofline|rows|frows"""
import glob
import json
import os
import sys


def lines(path):
    out = []
    for ln in open(path).read().splitlines():
        if ln.startswith("{"):
            d = json.loads(ln)
            if "metric" in d:
                out.append(d)
    return out


def roofline(root):
    print("| config | achieved (algorithmic) | frac of 8 TB/s | HBM traffic / algorithmic | limiter (busy) | ceiling, frac of HBM |")
    print("|---|---|---|---|---|---|")
    for c in ["c2", "c2s", "c3", "c4", "c4s", "k4"]:
        p = os.path.join(root, c + ".json")
        if not os.path.exists(p):
            continue
        d = lines(p)[-1]
        r = d["roofline"]
        n = d["config"].get("records_per_gpu")
        algo = r.get("algorithmic_bytes_per_record")
        tr = r.get("traffic")
        ratio = f"{tr / n / algo:.3f}x" if tr and n and algo else "-"
        ce = r.get("ceiling") or {}
        lim = f"{ce.get('limiter', '?')} ({100 * ce.get('busy_frac', 0):.0f} %)" if ce else "-"
        print(f"| {c} | {r['achieved']:.0f} GB/s | {r['frac']:.4f} | {ratio} | {lim} | "
              f"{ce.get('ceiling_frac_of_hbm', '-')} |")


def rows(root):
    print("| row | GiB/s | frac | kernel ms | CPU baseline: EVP / port (16 CPUs) |")
    print("|---|---|---|---|---|")
    for f in sorted(glob.glob(os.path.join(root, "*.json"))):
        name = os.path.basename(f)[:-5]
        if name.startswith(("stream", "dtls", "keysched", "count_gpus", "dist")):
            continue
        for d in lines(f):
            r = d.get("roofline") or {}
            cpu = d.get("cpu_baseline") or {}
            legs = {lg.get("leg"): lg.get("value") for lg in cpu.get("legs", [])}
            print(f"| {name} | {d['value']:.1f} | {r.get('frac', '-')} | {r.get('kernel_ms_avg', '-')} | "
                  f"{legs.get('evp', '-')} / {legs.get('port', '-')} |")


def frows(root):
    print("| row | direction | GiB/s (records/s) | frac | call ms (GPU) | CPU baseline: EVP / port (16 CPUs) |")
    print("|---|---|---|---|---|---|")
    for f in sorted(glob.glob(os.path.join(root, "*.json"))):
        name = os.path.basename(f)[:-5]
        if not name.startswith(("stream", "dtls", "keysched", "dist")):
            continue
        for d in lines(f):
            r = d.get("roofline") or {}
            cpu = d.get("cpu_baseline") or {}
            legs = {lg.get("leg"): lg.get("value") for lg in cpu.get("legs", [])} or {cpu.get("leg"): cpu.get("value")}
            m = d["metric"]
            direction = "receive" if "decrypt" in m else ("send" if "encrypt" in m else "-")
            rps = d.get("records_per_s") or d.get("connections_per_s")
            print(f"| {name} | {direction} | {d['value']:.1f} {d.get('unit', '')}"
                  f"{f' ({rps / 1e6:.0f} M/s)' if rps else ''} | {r.get('frac', '-')} | {r.get('kernel_ms_avg', '-')} | "
                  f"{legs.get('evp', '-')} / {legs.get('port', '-')} |")


if __name__ == "__main__":
    {"roofline": roofline, "rows": rows, "frows": frows}[sys.argv[2]](sys.argv[1])
