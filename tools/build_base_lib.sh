#!/bin/bash
# Build the library from a git revision's sources (csrc/ + include/) into
# chroma-lite_amd/chroma/_lib/ab/libchroma_amd_<NAME>.so -- the "before" side of a
# library A/B (tools/gpu_ab_libs.sh).  usage: tools/build_base_lib.sh REV NAME [EXTRA flags]
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2; EXTRA=${3:-}
T=$(mktemp -d /tmp/abbuild.XXXX)
mkdir -p "$T/chroma-lite_amd" "$T/include" "$R/chroma-lite_amd/chroma/_lib/ab"
git -C "$R" archive "$REV" chroma-lite_amd/csrc include tools/source_sha.py | tar -x -C "$T"
make -s -C "$T/chroma-lite_amd/csrc" -j8 OUT="$R/chroma-lite_amd/chroma/_lib/ab/libchroma_amd_$NAME.so" \
    PROF_OUT="$T/prof.so" EXTRA="$EXTRA" "$R/chroma-lite_amd/chroma/_lib/ab/libchroma_amd_$NAME.so"
rm -rf "$T"
echo "$R/chroma-lite_amd/chroma/_lib/ab/libchroma_amd_$NAME.so"
