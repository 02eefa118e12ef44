#!/usr/bin/env python3
"""Weighted VALU issue cost of a kernel's hot loop, from its gfx950 assembly.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Imbedtls_amd/csrc \
          --cuda-device-only -S mbedtls_amd/csrc/gcm_dec.hip -o /tmp/gcm_dec.s
    python tools/valu_mix.py /tmp/gcm_dec.s '<mangled kernel name>' [--need ds_read_b32=150]

Finds the kernel's loops (backward branches), takes the largest one that
holds every --need instruction count and a global load and store (the
record loop's body), and weights its VALU instructions by the issue costs
measured with tools/rate_probe.hip (8 waves x 8 chains per SIMD, shader-clock
ticks per wave64 instruction): 'fast' VOP1/VOP2-class ops and v_bitop3 2.3,
'slow' three-operand / multiply / 64-bit ops 4.2.  Prints the mix and the
mean ticks per instruction (combine_pmc.py --valu-ticks)."""
import collections
import re
import sys

SLOW = re.compile(r"^v_(alignbit|alignbyte|perm|add3|lshl_add|lshl_or|and_or|or3|xad|bfe|bfi|mad|mul|fma|"
                  r"lshrrev_b64|lshlrev_b64|ashrrev_i64|lshl_add_u64|mov_b64|cndmask_b32_e64|cmp_.*_e64)")


def loops(lines):
    lab = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            lab[m.group(1)] = i
    for i, l in enumerate(lines):
        m = re.search(r"\ts_cbranch_\w+\s+(\.LBB\w+)|\ts_branch\s+(\.LBB\w+)", l)
        if m:
            t = m.group(1) or m.group(2)
            if t in lab and lab[t] < i:
                c = collections.Counter()
                for x in lines[lab[t]:i + 1]:
                    x = x.strip()
                    if x and x[0] not in ";." and not x.endswith(":"):
                        c[x.split()[0]] += 1
                yield c


def main():
    path, name = sys.argv[1], sys.argv[2]
    need = {}
    for a in sys.argv[3:]:
        if a.startswith("--need"):
            continue
        k, v = a.split("=")
        need[k] = int(v)
    text = open(path).read().split("\n")
    start = next(i for i, l in enumerate(text) if l.startswith(name + ":"))
    end = next((i for i in range(start + 1, len(text)) if re.match(r"^_Z\w+:", text[i])), len(text))
    best = None
    for c in loops(text[start:end]):
        if c["global_load_dwordx4"] < 1 or c["global_store_dwordx4"] < 1:
            continue
        if any(c[k] < v for k, v in need.items()):
            continue
        if best is None or sum(c.values()) < sum(best.values()):
            best = c            # innermost qualifying loop
    if best is None:
        sys.exit("no qualifying loop")
    valu = {k: v for k, v in best.items() if k.startswith("v_")}
    slow = sum(v for k, v in valu.items() if SLOW.match(k))
    fast = sum(valu.values()) - slow
    ticks = (slow * 4.2 + fast * 2.3) / max(1, slow + fast)
    print(f"VALU {slow + fast}: slow {slow} fast {fast}; mean {ticks:.2f} ticks per instruction "
          f"(x4 model overstates by {4 / ticks:.2f}x)")
    for k, v in sorted(valu.items(), key=lambda kv: -kv[1])[:16]:
        print(f"  {'slow' if SLOW.match(k) else 'fast'} {k:24s} {v}")


if __name__ == "__main__":
    main()
