"""Per-kernel summary of a rocprofv3 --kernel-trace --stats run (tools/kstats.sh OUTDIR):
name, launches, average and total ms, from the kernel_stats CSV."""
import csv
import glob
import sys

out = sys.argv[1]
f = sorted(glob.glob(f"{out}/prof/**/*kernel_stats.csv", recursive=True))
if not f:
    sys.exit(f"no kernel_stats.csv under {out}/prof")
rows = list(csv.DictReader(open(f[0])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    print(f"{r['Name'][:58]:58s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e6:8.3f} "
          f"{float(r['TotalDurationNs']) / 1e6:9.2f}")
