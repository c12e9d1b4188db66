#!/bin/bash
# Round 6's committed measurements on the GPU box (outputs under OUTDIR, copied into profiles/
# on the build host afterwards):
#   1. PMC passes over one c2x24 10M step (tools/pmc_passes.sh; counters never combined with
#      runtime/system traces) -> per-kernel table kernel_pmc.json (VALU, HBM bytes, clock of
#      every launch; bench.py prices the dominant kernel's traffic and VALU rate from it)
#   2. rocprofv3 --kernel-trace --stats of the default bench command
#   3. the c4 bench line (6.25M reads) and its rocprofv3 --kernel-trace --stats
#   4. the default bench line with cpu_baseline (reads the table of step 1 from OUTDIR), and the
#      same workload with the piece screen off (DMX_NO_PIECES=1: the round-5 full filter pass)
# Usage: tools/profile_round6.sh OUTDIR TAG
set -e -o pipefail
out=$1; tag=$2
mkdir -p "$out"
export TMPDIR=/tmp
bash tools/pmc_passes.sh "$out/pmc" --reads 10000000 --steps 1 --warmup 0 --no-pcie
python3 tools/kernel_table_from_pmc.py "$out/pmc/p1" "$out/pmc/p2" "$out/pmc/p3" c2x24 10000000 \
  "$out/kernel_pmc.json" > "$out/kernel_pmc.txt"
python3 tools/pmc_summary.py "$out/pmc/p1" "$out/pmc/p2" "$out/pmc/p3" > "$out/pmc_summary.txt"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run \
  -- python3 bench.py --no-cpu-baseline --no-pcie > "$out/stats.log" 2>&1
cp "$out/stats/run_kernel_stats.csv" "$out/kernel_stats_c2x24_10M_$tag.csv"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats_c4" -o run \
  -- python3 bench.py --no-cpu-baseline --no-pcie --workload c4 --reads 6250000 \
  > "$out/stats_c4.log" 2>&1
cp "$out/stats_c4/run_kernel_stats.csv" "$out/kernel_stats_c4_6.25M_$tag.csv"
export DMX_KERNEL_PMC="$out/kernel_pmc.json"
timeout -k 10 400 python3 bench.py --workload c4 --reads 6250000 > "$out/bench_c4.json" \
  2> "$out/bench_c4.err"
DMX_NO_PIECES=1 timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-pcie \
  > "$out/bench_nopieces.json" 2> "$out/bench_nopieces.err"
timeout -k 10 400 python3 bench.py > "$out/bench.json" 2> "$out/bench.err"
