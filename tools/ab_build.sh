#!/bin/bash
# Build libduck_A.so from a git revision (default HEAD) next to the working tree's libduck.so,
# for same-box A/B timing (tools/gpu_ab.sh).
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" open_duck_playground_amd include tools | tar -x -C "$TMP"
(cd "$TMP" && python -c "
from open_duck_playground_amd import native
native.build(out='$ROOT/open_duck_playground_amd/libduck_A.so')
")
rm -rf "$TMP"
echo built libduck_A.so from $REV
