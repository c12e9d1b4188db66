#!/bin/bash
# Upstream parity hook for the reorientation step: runs
# ONLY where a real pychopper v2.7.0 is installed -- the version the reference pins
# (/root/reference/README.md:6); not in this image: no network, no package.  Another version is
# refused (a run on 2.7.10 would "confirm" behaviour the workflow never ran) unless
# ALLOW_OTHER_PYCHOPPER=1, which runs it with a loud warning in front of every result line.
# Writes one case per [UNVERIFIED] pychopper choice (tools/pychopper_cases.py: each case's
# outputs differ between the build's reading and the alternative one), runs every case through
# the real pychopper and through the drop-in (bin/pychopper), and diffs the four record outputs
# and the tuned cutoff.  A DIFF names the switch of oracle/chopper.py RULES to flip (and the
# kernels / drop-in to change with it).  Prints SKIPPED otherwise.
set -euo pipefail
REAL=${REAL_PYCHOPPER:-$(command -v pychopper || true)}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
if [ -z "$REAL" ] || [[ "$REAL" == "$ROOT"/* ]]; then
    echo "SKIPPED: no pychopper on PATH (set REAL_PYCHOPPER)"; exit 0
fi
VER=$("$REAL" --version 2>&1 | head -1)
WARN=""
if ! grep -Eq '(^|[^0-9.])2\.7\.0($|[^0-9])' <<<"$VER"; then
    if [ "${ALLOW_OTHER_PYCHOPPER:-0}" != 1 ]; then
        echo "REFUSED: $VER is not pychopper v2.7.0, the version the reference pins (README.md:6);"
        echo "         set ALLOW_OTHER_PYCHOPPER=1 to run it anyway (results are not a pin)"
        exit 2
    fi
    WARN="WARNING (not v2.7.0: $VER) "
    echo "${WARN}the reference pins pychopper v2.7.0; these results do not pin its behaviour"
fi
W=$(mktemp -d)
python3 "$ROOT/tools/pychopper_cases.py" "$W/cases"
fail=0
for impl in real dmx; do
    exe=$REAL; [ $impl = dmx ] && exe=$ROOT/nanopore-barcoding-orc_amd/bin/pychopper
    mkdir -p "$W/$impl"
    while IFS=$'\t' read -r name inp opts; do
        o=$W/$impl/$name
        # shellcheck disable=SC2086  # the options are a word list by construction
        (cd "$W/cases" && "$exe" $opts -w "${o}_rescued.fastq" -u "${o}_unclass.fastq" \
            -l "${o}_short.fastq" -S "${o}_stats.out" -t 4 "$inp" > "${o}_pass.fastq")
    done < "$W/cases/cases.tsv"
done
while IFS=$'\t' read -r name _ _; do
    for k in pass rescued unclass short; do
        if ! cmp -s "$W/real/${name}_$k.fastq" "$W/dmx/${name}_$k.fastq"; then
            echo "${WARN}DIFF ($name switch): ${name}_$k.fastq"; fail=1
        fi
    done
    a=$(grep -i cutoff "$W/real/${name}_stats.out" | head -1 | awk '{print $NF}')
    b=$(grep -i cutoff "$W/dmx/${name}_stats.out" | head -1 | awk '{print $NF}')
    if [ "$a" != "$b" ]; then echo "${WARN}DIFF ($name switch): cutoff $a vs $b"; fail=1; fi
done < "$W/cases/cases.tsv"
[ $fail = 0 ] && echo "${WARN}PARITY OK: every [UNVERIFIED] pychopper case identical to $VER"
exit $fail
