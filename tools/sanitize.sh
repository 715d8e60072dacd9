#!/bin/bash
# ASan + UBSan run of the host runtime (libggml_core: allocators, graph builder, GGUF reader/writer,
# quantizers) over the host tests, malformed GGUF files included. CPU only; the release libraries
# are untouched. Writes profiles/<tag>_sanitize.txt.
set -eo pipefail
TAG=${1:-r04}
cd "$(dirname "$0")/.."
make -C ggml-imax_amd sanitize -j8 > /dev/null
export GGML_MI355X_CORE_LIB=$PWD/ggml-imax_amd/lib/san/libggml_core.so
export LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
# the interpreter itself is not instrumented: its allocations are not ASan's to report as leaks
export GGML_MI355X_ISOLATE=dlmopen
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
python -m pytest tests/test_core.py tests/test_gguf.py -q -m "not gpu" -p no:cacheprovider 2>&1 | grep -v "allocating 0 bytes" | tee profiles/${TAG}_sanitize.txt
