#!/bin/bash
# PMC passes over one short bench run (one pass per counter group; counters never combined with
# runtime/system traces).  Pass 3 carries GRBM_GUI_ACTIVE: a kernel's effective shader clock is
# GRBM_GUI_ACTIVE / 8 (XCDs) / its duration (MI355X_MICROARCH.md, DVFS give-back).
# Usage: tools/pmc_passes.sh OUTDIR [bench args...]
# Summarise with: python tools/pmc_summary.py OUTDIR/*
set -e -o pipefail
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
passes=(
  "FETCH_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
  "WRITE_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
  "SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --pmc $p --output-format csv -d "$out/p$i" -o run -- \
    python3 bench.py --no-cpu-baseline "$@" > "$out/p$i.log" 2>&1
done
