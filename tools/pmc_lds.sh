#!/bin/bash
# LDS behaviour per kernel: one rocprofv3 --pmc pass of LDS instructions,
# bank-conflict cycles, LDS waits and wave cycles over one bench step, for the default
# library and, optionally, A/B builds given as DMX_LIBDMX paths.
# Usage: tools/pmc_lds.sh OUTDIR [lib.so ...]    Summary: tools/pmc_lds_summary.py OUTDIR
set -e -o pipefail
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
ctr="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES"
timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$out/default" -o run -- \
  python3 bench.py --no-cpu-baseline --no-pcie --steps 1 --warmup 0 > "$out/default.log" 2>&1
for lib in "$@"; do
  name=$(basename "$lib" .so)
  DMX_LIBDMX=$lib timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$out/$name" \
    -o run -- python3 bench.py --no-cpu-baseline --no-pcie --steps 1 --warmup 0 \
    > "$out/$name.log" 2>&1
done
