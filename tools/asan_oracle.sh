#!/bin/bash
# Host sanitizer run (CPU only, this container): the oracle built with
# AddressSanitizer + UBSan (oracle/Makefile `asan`), loaded through
# MGS_ORACLE_LIB into the CPU test suites that drive it.  Never on the GPU box.
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -C oracle asan
ASAN_LIB=$(gcc -print-file-name=libasan.so)
UBSAN_LIB=$(gcc -print-file-name=libubsan.so)
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:allocator_may_return_null=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export OMP_NUM_THREADS=4
if [ $# -eq 0 ]; then
  set -- tests/test_oracle.py tests/test_golden_harness.py tests/test_golden_more.py tests/test_contact_sampler.py \
    tests/test_clutter.py
fi
MGS_ORACLE_LIB=$PWD/oracle/_asan/libmgs_oracle.so LD_PRELOAD="$ASAN_LIB:$UBSAN_LIB" \
  python -m pytest -q -x -p no:cacheprovider -m "not gpu" "$@"
