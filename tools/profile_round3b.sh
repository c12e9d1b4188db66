#!/bin/bash
# Round-3 re-measurement after the second session's kernel changes (outputs under OUTDIR; copied
# into profiles/ on the build host afterwards).  As tools/profile_round3.sh without the VALU
# ceiling run (its stamped clock, profiles/r3_valu_ceiling.json, does not depend on libdmx):
#   1. PMC tables (VALU, HBM bytes, waits, LDS, effective clock) of one step of c2x24 10M,
#      c4 6.25M and c5 10M -> kernel_pmc.json; HBM traffic of each line's dominant kernel
#   2. rocprofv3 --kernel-trace --stats of the default bench command
#   3. the bench lines (c4, c5, then c2x24 with cpu_baseline) reading the tables of step 1
# Every PMC pass runs alone (tools/pmc_passes.sh) under its own time limit.
# Usage: tools/profile_round3b.sh OUTDIR
set -e -o pipefail
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
cp profiles/kernel_pmc.json "$out/kernel_pmc.json"
cp profiles/filter_pmc_traffic.json "$out/filter_pmc_traffic.json"
run_pmc() {   # workload reads dominant-kernel
  local w=$1 n=$2 k=$3
  bash tools/pmc_passes.sh "$out/pmc_$w" --workload "$w" --reads "$n" --steps 1 --warmup 0 \
    --no-pcie
  python3 tools/kernel_table_from_pmc.py "$out/pmc_$w/p1" "$out/pmc_$w/p2" "$out/pmc_$w/p3" \
    "$w" "$n" "$out/kernel_pmc.json" > "$out/kernel_pmc_$w.txt"
  python3 tools/traffic_from_pmc.py "$out/pmc_$w/p1" "$out/pmc_$w/p2" "$w" "$n" \
    "$out/filter_pmc_traffic.json" "$k" > "$out/traffic_$w.json"
  python3 tools/pmc_summary.py "$out/pmc_$w/p1" "$out/pmc_$w/p2" "$out/pmc_$w/p3" \
    > "$out/pmc_summary_$w.txt"
}
run_pmc c2x24 10000000 filter_kernel
run_pmc c4 6250000 filter_kernel
run_pmc c5 10000000 "scan_kernel<true>@0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run \
  -- python3 bench.py --no-cpu-baseline --no-pcie > "$out/stats.log" 2>&1
cp "$out/stats/run_kernel_stats.csv" "$out/kernel_stats_c2x24_10M.csv"
export DMX_KERNEL_PMC="$out/kernel_pmc.json" DMX_FILTER_TRAFFIC="$out/filter_pmc_traffic.json"
timeout -k 10 300 python3 bench.py --workload c4 --reads 6250000 --no-cpu-baseline \
  > "$out/bench_c4.json" 2> "$out/bench_c4.err"
timeout -k 10 300 python3 bench.py --workload c5 --no-cpu-baseline > "$out/bench_c5.json" \
  2> "$out/bench_c5.err"
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err"
