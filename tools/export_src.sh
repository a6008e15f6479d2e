#!/bin/bash
# Export the engine sources of a commit into build/src_NAME (for an A/B
# variant of an older kernel set: SRC=build/src_NAME tools/build_variant.sh NAME).
# Usage: bash tools/export_src.sh COMMIT NAME
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/build/src_$2
mkdir -p $D/csrc $D/include
for f in $(git -C $ROOT ls-tree --name-only $1 map-oxidize_amd/csrc/); do git -C $ROOT show $1:$f > $D/csrc/$(basename $f); done
git -C $ROOT show $1:include/mox.h > $D/include/mox.h
# the sources include ../../include/mox.h
mkdir -p $D/x && mv $D/csrc $D/x/csrc && ln -sfn x/csrc $D/csrc 2>/dev/null || true
echo $D/x/csrc
