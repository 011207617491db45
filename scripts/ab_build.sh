#!/bin/bash
# Builds libepp.so as of git revision $1 into scripts/dbg/libepp_$2.so (diagnostics A/B: the
# probes load it through EPP_LIB, so two versions are timed on the same GPU box in one call).
set -eu
cd "$(dirname "$0")/.."
rev=$1; name=$2
dir=scripts/dbg/src_$name
rm -rf "$dir" && mkdir -p "$dir"
git archive "$rev" efficient-path-planner_amd/csrc efficient-path-planner_amd/Makefile include | tar -x -C "$dir"
make -s -j8 -C "$dir/efficient-path-planner_amd" ROOT="$PWD/$dir" BUILD=build LIB="$PWD/scripts/dbg/libepp_$name.so" \
  "$PWD/scripts/dbg/libepp_$name.so"
rm -rf "$dir"
echo "scripts/dbg/libepp_$name.so"
