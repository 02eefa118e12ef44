"""Summarise a multi-library same-box A/B (tools/gpu_r06.sh multiab): per row,
each library's values over the reps and the mean ratio to the first library."""
import json
import sys
from collections import OrderedDict, defaultdict


def main(path):
    vals = defaultdict(lambda: defaultdict(list))
    libs = OrderedDict()
    for line in open(path):
        d = json.loads(line)
        vals[d["row"]][d["lib"]].append(d["value"])
        libs[d["lib"]] = True
    libs = list(libs)
    for row in vals:
        base = vals[row].get(libs[0]) or [float("nan")]
        b = sum(base) / len(base)
        parts = []
        for lib in libs:
            v = vals[row].get(lib, [])
            if v:
                m = sum(v) / len(v)
                parts.append("%s %s (%+.1f%%)" % (lib, "/".join("%.1f" % x for x in v), 100.0 * (m / b - 1.0)))
        print(row, " | ".join(parts))


if __name__ == "__main__":
    main(sys.argv[1])
