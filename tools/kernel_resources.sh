#!/bin/bash
# Per-kernel register use and occupancy of libdmx's HIP kernels (compile-time, no GPU needed).
# Usage: tools/kernel_resources.sh [REPO_DIR]   (default: this repo)
set -e -o pipefail
dir=${1:-$(dirname "$0")/..}
cd "$dir/nanopore-barcoding-orc_amd"
make -s asm 2>&1 | python3 -c "
import re, sys
cur = None
for l in sys.stdin:
    m = re.search(r'Function Name: (\S+)', l)
    if m:
        if cur:
            print()
        cur = m.group(1)[:48]
        print(f'{cur:50s}', end=' ')
    for k in ('VGPRs:', 'AGPRs:', 'Occupancy \[waves/SIMD\]:', 'SGPRs Spill:', 'VGPRs Spill:'):
        m = re.search(k + r' (\d+)', l)
        if m:
            print(k.split()[0].rstrip(':'), m.group(1), end='  ')
print()
"
