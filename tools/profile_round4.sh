#!/bin/bash
# Round-4 measurements of the current tree (outputs under OUTDIR; the summaries are copied into
# profiles/ on the build host afterwards):
#   1. PMC tables (VALU, HBM bytes, waits, LDS, effective clock) of one step of c2x24 10M
#      -> kernel_pmc.json, and the filter's HBM traffic (FETCH_SIZE x 2: the factor holds for the
#      filter's streamed blocks and, per profiles/r4_gather_calibration.json, for 4-16 B gathers)
#   2. the VALU issue pass (tools/pmc_valu.sh) over the bench step and the VALU microbenchmark
#   3. rocprofv3 --kernel-trace --stats of the default bench command
#   4. the bench line (20 steps after 5 warm-ups) reading the tables of step 1
# Every PMC pass runs alone under its own time limit.  Usage: tools/profile_round4.sh OUTDIR
set -e -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
cp profiles/kernel_pmc.json "$out/kernel_pmc.json"
cp profiles/filter_pmc_traffic.json "$out/filter_pmc_traffic.json"
w=c2x24 n=10000000
bash tools/pmc_passes.sh "$out/pmc_$w" --workload "$w" --reads "$n" --steps 1 --warmup 0 --no-pcie
python3 tools/kernel_table_from_pmc.py "$out/pmc_$w/p1" "$out/pmc_$w/p2" "$out/pmc_$w/p3" \
  "$w" "$n" "$out/kernel_pmc.json" > "$out/kernel_pmc_$w.txt"
python3 tools/traffic_from_pmc.py "$out/pmc_$w/p1" "$out/pmc_$w/p2" "$w" "$n" \
  "$out/filter_pmc_traffic.json" filter_kernel > "$out/traffic_$w.json"
python3 tools/pmc_summary.py "$out/pmc_$w/p1" "$out/pmc_$w/p2" "$out/pmc_$w/p3" \
  > "$out/pmc_summary_$w.txt"
bash tools/pmc_valu.sh "$out/valu"
python3 tools/pmc_valu_summary.py "$out/valu" > "$out/valu_summary.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run \
  -- python3 bench.py --no-cpu-baseline --no-pcie > "$out/stats.log" 2>&1
cp "$out/stats/run_kernel_stats.csv" "$out/kernel_stats_c2x24_10M.csv"
export DMX_KERNEL_PMC="$out/kernel_pmc.json" DMX_FILTER_TRAFFIC="$out/filter_pmc_traffic.json"
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err"
