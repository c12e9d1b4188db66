#!/bin/bash
# VALU issue evidence for the filter's ceiling: one rocprofv3 --pmc pass of
# the issue / lane-utilisation counters over one bench step, and the same pass over the VALU
# microbenchmark (tools/microbench/myers_ilp.hip: dependent / independent v_bitop3 chains and the
# 64-bit Myers step), so the filter's rates can be read against loops whose limits are known.
# Usage: tools/pmc_valu.sh OUTDIR [bench args...]   Summary: tools/pmc_valu_summary.py OUTDIR
set -e -o pipefail
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
ctr="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$out/bench" -o run -- \
  python3 bench.py --no-cpu-baseline --no-pcie --steps 1 --warmup 0 "$@" > "$out/bench.log" 2>&1
/opt/rocm/bin/hipcc -Wno-unused-value -O3 -std=c++17 --offload-arch=gfx950 -o /tmp/myers_ilp \
  "$(dirname "$0")/microbench/myers_ilp.hip"
timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$out/ilp" -o run -- \
  /tmp/myers_ilp > "$out/ilp.log" 2>&1
