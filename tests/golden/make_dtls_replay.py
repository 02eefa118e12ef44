#!/usr/bin/env python3
"""Transcribe the reference's DTLS anti-replay test vectors into
tests/golden/dtls_replay.json (data only: inputs and expected outputs).

Run here (the reference is not on the GPU box):
    python tests/golden/make_dtls_replay.py

Source: /root/reference/tests/suites/test_suite_ssl.data:763-818, the cases
of ssl_dtls_replay (test_suite_ssl.function:1510-1541): every 6-byte record
number of `prevs` goes through mbedtls_ssl_dtls_replay_update, then
mbedtls_ssl_dtls_replay_check(new) must return `ret` (0 or -1).
"""
from __future__ import annotations

import json
import os
import re

REF = "/root/reference/tests/suites/test_suite_ssl.data"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dtls_replay.json")


def main():
    lines = open(REF).read().splitlines()
    cases = []
    for i, line in enumerate(lines):
        m = re.match(r'^ssl_dtls_replay:"([0-9a-f]*)":"([0-9a-f]*)":(-?\d+)$', line)
        if not m:
            continue
        prevs = [m.group(1)[k:k + 12] for k in range(0, len(m.group(1)), 12)]
        cases.append({"name": lines[i - 1], "line": i + 1, "prevs": prevs, "new": m.group(2),
                      "ret": int(m.group(3))})
    assert len(cases) == 19, len(cases)
    json.dump({"source": "tests/suites/test_suite_ssl.data (ssl_dtls_replay)", "cases": cases},
              open(OUT, "w"), indent=1)
    print(OUT, len(cases))


if __name__ == "__main__":
    main()
