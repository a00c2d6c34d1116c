#!/bin/bash
# Build libmagpie_hip.so of git revision REV into ab_libs/NAME.so (an A/B baseline that
# travels with the tree; MAGPIE_LIB selects it). usage: tools_dev/build_rev.sh REV NAME
set -e -o pipefail
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=/tmp/mp_rev_$NAME
rm -rf "$SRC"
git -C "$ROOT" worktree add -f --detach "$SRC" "$REV" > /dev/null
make -C "$SRC/magpie-tts.cpp_amd" -j8 lib/libmagpie_hip.so > /dev/null
mkdir -p "$ROOT/ab_libs"
cp "$SRC/magpie-tts.cpp_amd/lib/libmagpie_hip.so" "$ROOT/ab_libs/$NAME.so"
git -C "$ROOT" worktree remove --force "$SRC"
echo "built ab_libs/$NAME.so from $(git -C "$ROOT" rev-parse --short "$REV")"
