#!/bin/bash
# FETCH_SIZE calibration for gathers (tools/microbench/gather_calib.hip): the plain run (HIP-event
# times), then one rocprofv3 pass per counter group, then the summary JSON.
# Usage: tools/microbench/run_gather_calib.sh OUTDIR   (run on the GPU box; binary built here)
set -e -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
bin=$(dirname "$0")/gather_calib
timeout -k 10 120 "$bin" > "$out/plain.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/p1" -o run -- "$bin" \
  > "$out/p1.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv \
  -d "$out/p2" -o run -- "$bin" > "$out/p2.log" 2>&1
python3 "$(dirname "$0")/gather_calib_summary.py" "$out" > "$out/gather_calibration.json"
