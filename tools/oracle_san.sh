#!/bin/bash
# Sanitizer pass over the CPU oracle: the ASan + UBSan stand-alone driver, then the
# whole CPU pytest suite against the UBSan build of librefcpu (TSDB_ORACLE_LIB).
set -e -o pipefail
cd "$(dirname "$0")/.."
make -s -C oracle san
./oracle/build/san_driver
TSDB_ORACLE_LIB=$PWD/oracle/build/librefcpu_ubsan.so UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  python -m pytest tests -m "not gpu" -x -q -p no:cacheprovider "$@"
