#!/bin/bash
# The CPU suite (oracle golden vectors, KATs, physics laws, edited scenes, height-field prisms) against
# the AddressSanitizer + UndefinedBehaviorSanitizer build of the checker (oracle/Makefile ASAN=1),
# with the ASan runtime preloaded into this process so heap accesses are checked as well.
set -o pipefail
cd "$(dirname "$0")/.."
make -s -C oracle ASAN=1
LD_PRELOAD=$(gcc -print-file-name=libasan.so)${LD_PRELOAD:+:$LD_PRELOAD} ORACLE_LIB=$PWD/oracle/liboracle_asan.so ASAN_OPTIONS=detect_leaks=0 \
  python -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@"
