mkdir -p gpurun_out
DMX_IO_DEBUG=1 timeout -k 10 300 python3 tools/io_pipeline_bench.py --reads 400000 --threads 16 --workdir /tmp/pd --keep --modes inflate > gpurun_out/r5_pinflate_debug.json 2> gpurun_out/r5_pinflate_debug.err
