#!/bin/bash
# Host sanitizer runs (CPU): the native host code of the drop-in boundary --
# csrc/pyhost.c (encoder incl. its worker pool, dict assembly), csrc/graph_host.cpp (MERGE
# bookkeeping, CSR build), the C-ABI's host side -- under AddressSanitizer + UBSan, and the
# encoder's worker pool under ThreadSanitizer, through the host tests.
#   scripts/sanitize.sh [OUT_DIR]      (builds `make sanitize tsan` first)
set -euo pipefail
REPO=$(cd "$(dirname "$0")/.." && pwd)
PKG=$REPO/kubernetes-aiops-evidence-graph_amd
OUT=${1:-$REPO/profiles}
make -C "$PKG" -j8 sanitize tsan > /dev/null
CLANG=/opt/rocm/llvm/bin/clang
TESTS="tests/test_pyhost.py tests/test_native_host.py tests/test_seeds_native.py tests/test_encoder.py"
cd "$REPO"
echo "== ASan + UBSan: libegraph.so (host code) + _egr_pyhost ==" | tee "$OUT/r03_sanitize_asan.txt"
LD_PRELOAD=$($CLANG -print-file-name=libclang_rt.asan-x86_64.so) \
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:alloc_dealloc_mismatch=0:detect_odr_violation=0 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
EGRAPH_LIB=$PKG/lib/asan/libegraph.so EGRAPH_PYHOST_DIR=$PKG/lib/asan \
  python -m pytest $TESTS -q -p no:xdist -p no:cacheprovider 2>&1 | tee -a "$OUT/r03_sanitize_asan.txt"
# the instrumented builds are the ones loaded (and the runtime is in the process)
LD_PRELOAD=$($CLANG -print-file-name=libclang_rt.asan-x86_64.so) ASAN_OPTIONS=detect_leaks=0:alloc_dealloc_mismatch=0 \
EGRAPH_LIB=$PKG/lib/asan/libegraph.so EGRAPH_PYHOST_DIR=$PKG/lib/asan PYTHONPATH=$PKG \
  python -c "import egraph._lib as L; m = open('/proc/self/maps').read(); \
assert 'lib/asan/libegraph.so' in m and 'lib/asan/_egr_pyhost' in m and 'clang_rt.asan' in m; \
print('loaded:', L.LIB_PATH, L.pyhost.__file__)" | tee -a "$OUT/r03_sanitize_asan.txt"
echo "== TSan: _egr_pyhost (the worker pool: encoder, seed attachment, seed keys) ==" | tee "$OUT/r03_sanitize_tsan.txt"
LD_PRELOAD=$($CLANG -print-file-name=libclang_rt.tsan-x86_64.so) \
TSAN_OPTIONS=halt_on_error=1:report_signal_unsafe=0 \
EGRAPH_PYHOST_DIR=$PKG/lib/tsan EGRAPH_ENCODE_THREADS=8 \
  python -m pytest tests/test_pyhost.py tests/test_encoder.py tests/test_seeds_native.py tests/test_native_host.py \
    -q -p no:xdist -p no:cacheprovider 2>&1 | tee -a "$OUT/r03_sanitize_tsan.txt"
LD_PRELOAD=$($CLANG -print-file-name=libclang_rt.tsan-x86_64.so) \
EGRAPH_PYHOST_DIR=$PKG/lib/tsan PYTHONPATH=$PKG \
  python -c "import egraph._lib as L; m = open('/proc/self/maps').read(); \
assert 'lib/tsan/_egr_pyhost' in m and 'clang_rt.tsan' in m; print('loaded:', L.pyhost.__file__)" \
  | tee -a "$OUT/r03_sanitize_tsan.txt"
