#!/bin/bash
# One profiling session on the GPU box: the default bench line, a rocprofv3 kernel-trace/stats
# run of the same command, and the two HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE; one pass
# each, never combined with runtime/system traces).  Usage: tools/profile_bench.sh OUTDIR [args]
set -e -o pipefail
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py "$@" > "$out/bench.json" 2> "$out/bench.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run \
  -- python3 bench.py --no-cpu-baseline "$@" > "$out/stats.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run \
  -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 "$@" > "$out/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run \
  -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 "$@" > "$out/write.log" 2>&1
