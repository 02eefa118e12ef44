#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 300 python3 tools/probes/pcie_duplex.py > $O/pcie.json 2> $O/pcie.err || { tail -5 $O/pcie.err; exit 1; }
cat $O/pcie.json
