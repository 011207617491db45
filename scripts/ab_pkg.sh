#!/bin/bash
# Builds the whole package (libepp.so + the pybind modules + eppamd) as of git revision $1
# into scripts/dbg/pkg_$2/ (diagnostics A/B: scripts/plan_probe.py loads it with
# EPP_PKG=scripts/dbg/pkg_$2, so two versions of the full planner run on the same GPU box).
set -eu
cd "$(dirname "$0")/.."
rev=$1; name=$2
dir=scripts/dbg/src_$name
rm -rf "$dir" "scripts/dbg/pkg_$name" && mkdir -p "$dir"
git archive "$rev" efficient-path-planner_amd include | tar -x -C "$dir"
make -s -j8 -C "$dir/efficient-path-planner_amd" ROOT="$PWD/$dir" PYTHON=python3 > /dev/null
mkdir -p "scripts/dbg/pkg_$name"
cp -r "$dir/efficient-path-planner_amd/eppamd" "$dir"/efficient-path-planner_amd/*.so "scripts/dbg/pkg_$name/"
rm -rf "$dir"
echo "scripts/dbg/pkg_$name"
