"""dmx — MI355X-native two-round SP5 x SP27 barcode demultiplexer (cutadapt-compatible).

Drop-in for the cutadapt calls of the reference's scripts/02_cutadapt_loop.sh (and the linked
primer calls of scripts/04_cleaning_primers.sh).  Compute runs in libdmx.so (HIP, gfx950).
"""
__version__ = "0.1.0"
