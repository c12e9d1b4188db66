#!/bin/bash
# A/B of in-tree libdmx builds on the GPU box: one bench line per library (no CPU baseline).
# Usage: tools/ab_bench.sh OUTDIR LIB... (paths relative to the repo root; "default" = libdmx.so)
set -e -o pipefail
out=$1; shift
mkdir -p "$out"
for l in "$@"; do
  tag=$(basename "$l" .so)
  if [ "$l" = default ]; then unset DMX_LIBDMX; else export DMX_LIBDMX=$PWD/$l; fi
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > "$out/$tag.json" 2> "$out/$tag.err"
  python3 -c "import json,sys; d=json.load(open('$out/$tag.json')); s=d['stage_ms_per_step']; print('$tag', d['value'], 'ms', d['ms_per_step'], ' '.join(f'{k} {v}' for k, v in s.items() if k not in ('scan0', 'scan1', 'total')))"
done
