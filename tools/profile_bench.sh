#!/bin/bash
# One profiling session on the GPU box (default workload unless args say otherwise):
#   1. HBM-traffic PMC passes for the filter kernel (FETCH_SIZE, WRITE_SIZE; one counter per pass,
#      never combined with runtime/system traces) -> profiles/filter_pmc_traffic.json
#   2. the bench line (with cpu_baseline), which reads that traffic figure
#   3. a rocprofv3 --kernel-trace --stats run of the same bench command
# Usage: tools/profile_bench.sh OUTDIR TAG   (outputs under OUTDIR; TAG names the round)
set -e -o pipefail
out=$1; tag=$2
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run \
  -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > "$out/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run \
  -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > "$out/write.log" 2>&1
python3 tools/traffic_from_pmc.py "$out/fetch" "$out/write" c2x24 10000000 \
  profiles/filter_pmc_traffic.json > "$out/traffic.json"
cp profiles/filter_pmc_traffic.json "$out/"
timeout -k 10 400 python3 bench.py > "$out/bench.json" 2> "$out/bench.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run \
  -- python3 bench.py --no-cpu-baseline > "$out/stats.log" 2>&1
cp "$out/stats/run_kernel_stats.csv" "$out/kernel_stats_$tag.csv"
