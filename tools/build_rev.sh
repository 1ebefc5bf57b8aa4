#!/bin/bash
# Builds libqgcm.so of git revision <rev> as ab/libqgcm_<tag>.so, for in-process A/B against the
# working tree (tools/ab_libs.py).  Usage: bash tools/build_rev.sh <rev> <tag>
set -eu
REV=$1; TAG=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d /tmp/qgcm_rev_XXXX)
git -C "$ROOT" archive "$REV" quantum_amd/csrc include | tar -x -C "$TMP"
mkdir -p "$ROOT/ab"
make -s -C "$TMP/quantum_amd/csrc" -j8 OUT="$TMP" >/dev/null
cp "$TMP/libqgcm.so" "$ROOT/ab/libqgcm_$TAG.so"
rm -rf "$TMP"
echo "ab/libqgcm_$TAG.so"
