#!/bin/bash
# Upstream parity hook: runs ONLY where a real cutadapt 4.9 is installed (not
# in this image: no network, no package).  Generates seeded synthetic reads, runs the reference
# command lines of scripts/02_cutadapt_loop.sh with the real cutadapt and with the dmx drop-in,
# and diffs every decompressed per-bin output.  Prints SKIPPED otherwise.
set -euo pipefail
REAL=${REAL_CUTADAPT:-$(command -v cutadapt || true)}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
if [ -z "$REAL" ] || [[ "$REAL" == "$ROOT"/* ]] || ! "$REAL" --version 2>/dev/null | grep -q '^4\.9'; then
    echo "SKIPPED: no cutadapt 4.9 on PATH (set REAL_CUTADAPT)"; exit 0
fi
W=$(mktemp -d)
python3 - "$W" <<'PY'
import gzip, sys
sys.path.insert(0, "nanopore-barcoding-orc_amd")
from dmx import synth
d = synth.generate("c2", n=20000, seed=123)
with gzip.open(f"{sys.argv[1]}/in.fastq.gz", "wt") as fh:
    for i, s in enumerate(synth.to_strings(d)):
        fh.write(f"@r{i}\n{s}\n+\n{'I' * len(s)}\n")
PY
SP5=$ROOT/nanopore-barcoding-orc_amd/dmx/data/M13_amplicon_indices_forward.fa
SP27=$ROOT/nanopore-barcoding-orc_amd/dmx/data/M13_amplicon_indices_reverse_rc.fa
for impl in real dmx; do
    exe=$REAL; [ $impl = dmx ] && exe=$ROOT/nanopore-barcoding-orc_amd/bin/cutadapt
    mkdir -p "$W/$impl/SP5" "$W/$impl/SP27"
    "$exe" --action=trim -e 0.1 -j 8 --rc -g file:"$SP5" -o "$W/$impl/SP5/{name}.fastq.gz" "$W/in.fastq.gz" > /dev/null
    for f in "$W/$impl"/SP5/SP5_*.fastq.gz; do
        id=$(basename "$f" .fastq.gz)
        "$exe" --action=trim -e 0.1 -j 8 --rc -a file:"$SP27" -o "$W/$impl/SP27/{name}_$id.fastq.gz" "$f" > /dev/null
    done
done
fail=0
for f in "$W"/real/SP*/*.fastq.gz; do
    g=${f/\/real\//\/dmx\/}
    if ! cmp -s <(zcat "$f") <(zcat "$g"); then echo "DIFF: ${f#$W/real/}"; fail=1; fi
done

# One case per rule the oracle marks [UNVERIFIED] (tools/unverified_cases.py: the reads make
# the two plausible readings of the rule give different outputs; tests/test_oracle.py checks
# that with oracle/pyref.py under both readings).  A DIFF names the rule to correct in the
# oracle and the kernels.
python3 "$ROOT/tools/unverified_cases.py" "$W/cases"
for impl in real dmx; do
    exe=$REAL; [ $impl = dmx ] && exe=$ROOT/nanopore-barcoding-orc_amd/bin/cutadapt
    mkdir -p "$W/$impl/rules"
    while IFS=$'\t' read -r name inp out opts; do
        # shellcheck disable=SC2086  # options and outputs are word lists by construction
        (cd "$W/cases" && "$exe" $opts ${out//@OUT@/$W/$impl/rules} "$inp" > /dev/null)
    done < "$W/cases/cases.tsv"
done
for f in "$W"/real/rules/*; do
    g=${f/\/real\//\/dmx\/}
    if ! cmp -s "$f" "$g"; then echo "DIFF (unverified rule): $(basename "$f")"; fail=1; fi
done
[ $fail = 0 ] && echo "PARITY OK: every per-bin output and every unverified-rule case identical to cutadapt $("$REAL" --version)"
exit $fail
