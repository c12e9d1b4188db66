#!/bin/bash
# rocprofv3 --kernel-trace --stats of a short default bench (c2x24, 10 M reads) into OUTDIR,
# then the per-kernel summary (tools/kstats.py).  Usage: tools/kstats.sh OUTDIR [bench args]
set -e -o pipefail
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- \
  python3 bench.py --no-cpu-baseline --no-pcie --steps 3 --warmup 1 "$@" > "$out/bench.json" \
  2> "$out/bench.err"
