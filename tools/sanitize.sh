#!/bin/bash
# Host sanitizer runs (SURVEY.md §5 "race detection / sanitizers"; CPU only, no GPU calls).
# Builds the sanitizer variants (make sanitize) and runs the host-side CPU tests against them:
#   pass 1  gcc ASan + UBSan: libdmx_io.so (reader, inflate, packer, writers, deflate, work
#           pool), libdmx_synth.so, the oracle (liborc.so)
#   pass 2  TSan: libdmx_io.so and libdmx_synth.so (threaded reader / sink / work pool)
#   pass 3  clang ASan + UBSan on libdmx.so's host code (dmx_pack, panels, exported symbols)
# Output: one log per pass under $OUT (default profiles/), ending in the pytest summary.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${OUT:-$ROOT/profiles}
TAG=${TAG:-r3}
PKG=$ROOT/nanopore-barcoding-orc_amd
make -s -C "$PKG" sanitize
make -s -C "$ROOT/oracle" sanitize
cd "$ROOT"
HOST_TESTS="tests/test_nio.py tests/test_fastx.py tests/test_oracle.py tests/test_report.py"
PY="python3 -m pytest -q -p no:cacheprovider"
export PYTEST_ADDOPTS="-m 'not gpu'"
export PYTHONMALLOC=malloc
# numpy's OpenBLAS thread pool deadlocks under the TSan runtime; the code under test is ours
export OPENBLAS_NUM_THREADS=1 OMP_NUM_THREADS=1
GCC_ASAN=$(gcc -print-file-name=libasan.so)
GCC_UBSAN=$(gcc -print-file-name=libubsan.so)
GCC_TSAN=$(gcc -print-file-name=libtsan.so)
CLANG_ASAN=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
run() {   # name, env..., -- tests
    local name=$1; shift
    local log=$OUT/${TAG}_sanitize_${name}.log
    echo "# $(date -u +%FT%TZ) $name: $*" > "$log"
    if env "$@" >> "$log" 2>&1; then echo "# exit 0" >> "$log"; else echo "# exit $?" >> "$log"; fi
    tail -3 "$log"
}
run asan_ubsan LD_PRELOAD="$GCC_ASAN:$GCC_UBSAN" \
    ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 \
    UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    DMX_LIBDIR=$PKG/build/asan DMX_LIBDMX=$PKG/dmx/libdmx.so ORC_LIBDIR=$ROOT/oracle/_san \
    $PY $HOST_TESTS
run tsan LD_PRELOAD="$GCC_TSAN" TSAN_OPTIONS=halt_on_error=1:report_signal_unsafe=0 \
    DMX_LIBDIR=$PKG/build/tsan DMX_LIBDMX=$PKG/dmx/libdmx.so \
    $PY tests/test_nio.py tests/test_fastx.py
run asan_hip LD_PRELOAD="$CLANG_ASAN" \
    ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 \
    DMX_LIBDMX=$PKG/build/asan-hip/libdmx.so \
    $PY tests/test_host.py
