#!/bin/bash
# A/B timing of libdmx builds on the default bench workload (c2x24, 10 M reads): one short
# bench per library (DMX_LIBDMX), results into OUTDIR/bench_<name>.json.
# Usage: tools/r6_ab.sh OUTDIR name[:lib.so] ...   ("default" = dmx/libdmx.so)
set -e -o pipefail
out=$1; shift
mkdir -p "$out"
for v in "$@"; do
  name=${v%%:*}
  lib=nanopore-barcoding-orc_amd/dmx/libdmx.so
  [ "$name" != default ] && lib=nanopore-barcoding-orc_amd/dmx/libdmx_$name.so
  DMX_LIBDMX=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pcie --steps 4 \
    --warmup 2 > "$out/bench_$name.json" 2> "$out/bench_$name.err"
done
