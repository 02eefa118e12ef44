#!/bin/bash
# Build an A/B variant of libtlsrec.so into ablib/<name>.so: the GCM units
# (or the units named in $UNITS) recompiled with extra defines, linked with
# the other objects of build/
# (run `python -m mbedtls_amd.build` first).  Measurement only -- the product
# library is mbedtls_amd/libtlsrec.so, built by mbedtls_amd/build.py.
#   tools/build_variant.sh <name> <hipcc flags...>    e.g.  abl1 -DTLSREC_ABLATE=1
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
O=$R/build/variant_$name
mkdir -p "$O" "$R/ablib"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS=(--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result -Wno-unused-value -I"$R/include" -I"$R/mbedtls_amd/csrc")
UNITS=${UNITS:-gcm_dec gcm_enc}
pids=()
for u in $UNITS; do
  "$HIPCC" "${FLAGS[@]}" "$@" -c "$R/mbedtls_amd/csrc/$u.hip" -o "$O/$u.o" & pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
objs=()
for u in gcm_dec gcm_enc gcm_alt_dec gcm_alt_enc kernels engine keysched stream ccm ticket server tlsrec_host; do
  if [ -f "$O/$u.o" ] && [[ " $UNITS " == *" $u "* ]]; then objs+=("$O/$u.o"); else objs+=("$R/build/$u.o"); fi
done
"$HIPCC" -shared -fPIC --offload-arch=gfx950 -o "$R/ablib/$name.so" "${objs[@]}"
echo "$R/ablib/$name.so"
