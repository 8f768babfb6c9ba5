#!/bin/bash
# Build the host-native C++ into an ASan+UBSan executable and run the repo's
# native-facing CPU tests inside it.  CPU only; no GPU involved.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${OUT:-/tmp/omnia_sanitize}
mkdir -p "$OUT"
PYINC=$(python3 -c "import sysconfig; print(sysconfig.get_paths()['include'])")
PBINC=$(python3 -c "import pybind11; print(pybind11.get_include())")
g++ -O1 -g -std=c++17 -fsanitize=address,undefined -fno-omit-frame-pointer \
    -fno-sanitize-recover=undefined -maes -mpclmul -mssse3 -msse4.1 \
    -I"$PYINC" -I"$PBINC" \
    "$ROOT"/omnia_amd/native/csrc/*.cpp "$ROOT"/scripts/native/sanitize_driver.cpp \
    $(python3-config --ldflags --embed) -o "$OUT/omnia_native_asan"
cd "$ROOT"
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
  "$OUT/omnia_native_asan" "$ROOT" -q -p no:cacheprovider -m "not gpu" \
  tests/test_ee.py::test_aes_gcm_nist_vectors tests/test_ee.py::test_envelope_message_roundtrip_and_rotation \
  tests/test_guided.py "$@"
