#!/bin/bash
# Measurement tool (not part of the product): tools/occ_probe.py once per
# occupancy cap (one process each: the library reads ONO_EW_OCC once), one
# JSON line per cap appended to $1 (default gpurun_out/occ_sweep.jsonl).
#   ROUNDS=<r> bash tools/occ_sweep.sh [out] [caps...]
set -o pipefail
out=${1:-gpurun_out/occ_sweep.jsonl}
shift || true
caps=${*:-default 32 28 24 20 16 12 10 8}
mkdir -p "$(dirname "$out")"
for c in $caps; do
    if [ "$c" = default ]; then
        timeout -k 10 150 python -u tools/occ_probe.py 30 ${ROUNDS:-1} >> "$out" || exit $?
    else
        ONO_EW_OCC=$c timeout -k 10 150 python -u tools/occ_probe.py 30 ${ROUNDS:-1} >> "$out" || exit $?
    fi
done
