#!/usr/bin/env python3
"""Transcribe the reference's TLS 1.3 key-schedule test vectors into
tests/golden/tls13_keys.json (data only: inputs and expected outputs).

Run here (the reference is not on the GPU box):
    python tests/golden/make_tls13_keys.py

Source: /root/reference/tests/suites/test_suite_ssl.data:2598-2850, the
cases of the test functions in test_suite_ssl.function:
  ssl_tls13_key_evolution            :2301-2323 -> mbedtls_ssl_tls13_evolve_secret
  ssl_tls13_hkdf_expand_label        :1862-1896 -> mbedtls_ssl_tls13_hkdf_expand_label
  ssl_tls13_traffic_key_generation   :1902-1950 -> mbedtls_ssl_tls13_make_traffic_keys
  ssl_tls13_derive_secret            :1960-1996 -> mbedtls_ssl_tls13_derive_secret
  ssl_tls13_exporter                 :2000-2028 -> mbedtls_ssl_tls13_exporter
  ssl_tls13_derive_{early,handshake,application,resumption}_secrets
                                     :2032-2170 -> derive_secret with the labels
                                        of ssl_tls13_keys.c:421-660
The vectors themselves come from RFC 8448 and tls13.ulfheim.net (as the
reference's comments say); two exporter vectors are OpenSSL outputs.
"""
from __future__ import annotations

import json
import os

REF = "/root/reference/tests/suites/test_suite_ssl.data"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tls13_keys.json")

# label identifiers of library/ssl_tls13_keys.h:13-33
LABELS = {
    "finished": "finished", "resumption": "resumption", "traffic_upd": "traffic upd",
    "exporter": "exporter", "key": "key", "iv": "iv", "c_hs_traffic": "c hs traffic",
    "c_ap_traffic": "c ap traffic", "c_e_traffic": "c e traffic", "s_hs_traffic": "s hs traffic",
    "s_ap_traffic": "s ap traffic", "s_e_traffic": "s e traffic", "e_exp_master": "e exp master",
    "res_master": "res master", "exp_master": "exp master", "ext_binder": "ext binder",
    "res_binder": "res binder", "derived": "derived",
}
HASH = {"PSA_ALG_SHA_256": "sha256", "PSA_ALG_SHA_384": "sha384"}


def split(line):
    """Split a .data call line on ':' outside of quotes."""
    out, cur, q = [], "", False
    for ch in line:
        if ch == '"':
            q = not q
            cur += ch
        elif ch == ":" and not q:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    out.append(cur)
    return out


def h(x):
    return x.strip('"').lower()


def lbl(x):
    return LABELS[x.replace("tls13_label_", "")]


def main():
    with open(REF) as f:
        lines = f.read().splitlines()
    out = {"source": "tests/suites/test_suite_ssl.data (Mbed TLS 4.1.0)", "evolve": [], "expand_label": [],
           "traffic_keys": [], "derive_secret": [], "exporter": []}
    title = ""
    for no, line in enumerate(lines, 1):
        if line and (no == 1 or not lines[no - 2].strip()):   # a case title follows a blank line
            title = line
            continue
        if not line.startswith("ssl_tls13_"):
            continue
        f = split(line)
        fn, args = f[0], f[1:]
        where = f"test_suite_ssl.data:{no}"
        if fn == "ssl_tls13_key_evolution":
            out["evolve"].append({"name": title, "where": where, "hash": HASH[args[0]], "secret": h(args[1]),
                                  "input": h(args[2]), "expected": h(args[3])})
        elif fn == "ssl_tls13_hkdf_expand_label":
            out["expand_label"].append({"name": title, "where": where, "hash": HASH[args[0]], "secret": h(args[1]),
                                        "label": lbl(args[2]), "ctx": h(args[3]), "len": int(args[4]),
                                        "expected": h(args[5])})
        elif fn == "ssl_tls13_traffic_key_generation":
            out["traffic_keys"].append({"name": title, "where": where, "hash": HASH[args[0]],
                                        "server_secret": h(args[1]), "client_secret": h(args[2]),
                                        "iv_len": int(args[3]), "key_len": int(args[4]),
                                        "server_key": h(args[5]), "server_iv": h(args[6]),
                                        "client_key": h(args[7]), "client_iv": h(args[8])})
        elif fn == "ssl_tls13_derive_secret":
            out["derive_secret"].append({"name": title, "where": where, "hash": HASH[args[0]], "secret": h(args[1]),
                                         "label": lbl(args[2]), "ctx": h(args[3]), "len": int(args[4]),
                                         "ctx_hashed": 1 if args[5] == "MBEDTLS_SSL_TLS1_3_CONTEXT_HASHED" else 0,
                                         "expected": h(args[6])})
        elif fn == "ssl_tls13_exporter":
            out["exporter"].append({"name": title, "where": where, "hash": HASH[args[0]], "secret": h(args[1]),
                                    "label": args[2].strip('"'), "context": args[3].strip('"'),
                                    "len": int(args[4]), "expected": h(args[5])})
        elif fn in ("ssl_tls13_derive_early_secrets", "ssl_tls13_derive_handshake_secrets",
                    "ssl_tls13_derive_application_secrets", "ssl_tls13_derive_resumption_secrets"):
            # ssl_tls13_keys.c:421-660: each helper = derive_secret(secret, label, transcript, HASHED)
            labels = {"ssl_tls13_derive_early_secrets": ["c e traffic", "e exp master"],
                      "ssl_tls13_derive_handshake_secrets": ["c hs traffic", "s hs traffic"],
                      "ssl_tls13_derive_application_secrets": ["c ap traffic", "s ap traffic", "exp master"],
                      "ssl_tls13_derive_resumption_secrets": ["res master"]}[fn]
            for lab, exp in zip(labels, args[3:]):
                out["derive_secret"].append({"name": f"{title} [{lab}]", "where": where, "hash": HASH[args[0]],
                                             "secret": h(args[1]), "label": lab, "ctx": h(args[2]),
                                             "len": len(h(exp)) // 2, "ctx_hashed": 1, "expected": h(exp)})
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print(OUT, {k: len(v) for k, v in out.items() if isinstance(v, list)})


if __name__ == "__main__":
    main()
