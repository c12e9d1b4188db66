#!/bin/bash
# L2 behaviour of the gather kernels: one rocprofv3 --pmc pass of L2 hits /
# misses / fabric read requests and L1->L2 read requests over one bench step, for the default
# library and, optionally, A/B builds given as DMX_LIBDMX paths.
# Usage: tools/pmc_l2.sh OUTDIR [lib.so ...]    Summary: tools/pmc_l2_summary.py OUTDIR
set -e -o pipefail
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
ctr="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD SQ_WAVES"
timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$out/default" -o run -- \
  python3 bench.py --no-cpu-baseline --no-pcie --steps 1 --warmup 0 > "$out/default.log" 2>&1
for lib in "$@"; do
  name=$(basename "$lib" .so)
  DMX_LIBDMX=$lib timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$out/$name" \
    -o run -- python3 bench.py --no-cpu-baseline --no-pcie --steps 1 --warmup 0 \
    > "$out/$name.log" 2>&1
done
