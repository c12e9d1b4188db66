set -e -o pipefail
export TMPDIR=/tmp
P=nanopore-barcoding-orc_amd/dmx
for v in libdmx libdmx_v512 libdmx_v256; do
  DMX_LIBDMX=$P/$v.so timeout -k 10 150 python3 bench.py --no-cpu-baseline --no-pcie --steps 10 --warmup 2 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  DMX_LIBDMX=$P/$v.so timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/ab_pmc_$v -o run -- python3 bench.py --no-cpu-baseline --no-pcie --steps 1 --warmup 0 > gpurun_out/ab_pmc_$v.log 2>&1
done
