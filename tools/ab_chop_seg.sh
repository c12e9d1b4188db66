# A/B of the reorientation scan's segment length (DMX_CHOP_SEG builds, dmx/libdmx_c*.so):
# the chop bench line per build.  Usage: bash tools/ab_chop_seg.sh
set -e -o pipefail
P=nanopore-barcoding-orc_amd/dmx
for v in libdmx libdmx_c256 libdmx_c384 libdmx_c768; do
  DMX_LIBDMX=$P/$v.so timeout -k 10 150 python3 bench.py --workload chop --no-cpu-baseline > gpurun_out/abc_$v.json 2> gpurun_out/abc_$v.err
done
