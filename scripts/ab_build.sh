#!/bin/bash
# Build libmi_engine_<name>.so from git revision <rev> (default HEAD) for same-box A/B runs:
#   scripts/ab_build.sh base HEAD   then on the GPU:  MI_ENGINE_LIB=base python bench.py ...
set -e
NAME=${1:?name}; REV=${2:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/mi_ab_$NAME
rm -rf "$WT"; mkdir -p "$WT"
git -C "$ROOT" archive "$REV" blama_amd/csrc include | tar -x -C "$WT"
make -C "$WT/blama_amd/csrc" -j4 >/dev/null
cp "$WT/blama_amd/libmi_engine.so" "$ROOT/blama_amd/libmi_engine_$NAME.so"
echo "built blama_amd/libmi_engine_$NAME.so from $REV"
