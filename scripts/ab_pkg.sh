#!/bin/bash
# Builds the whole package (libepp.so + the pybind modules + eppamd) as of git revision $1
# ("WORKTREE": the working tree) with the extra compiler flags $EXTRA into ab/pkg_$2/
# (diagnostics A/B: scripts/plan_probe.py loads it with EPP_PKG=ab/pkg_$2, so two versions
# of the full planner run on the same GPU box).  ab/ is git-ignored (not gpurun-ignored).
set -eu
cd "$(dirname "$0")/.."
rev=$1; name=$2
dir=ab/src_$name
rm -rf "$dir" "ab/pkg_$name" && mkdir -p "$dir"
if [ "$rev" = WORKTREE ]; then
  tar -c --exclude='*.so' --exclude='build*' --exclude=testhooks efficient-path-planner_amd include | tar -x -C "$dir"
else
  git archive "$rev" efficient-path-planner_amd include | tar -x -C "$dir"
fi
make -s -j8 -C "$dir/efficient-path-planner_amd" ROOT="$PWD/$dir" PYTHON=python3 EXTRA="${EXTRA:-}" \
  libepp.so online_traj_planner$(python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))") > /dev/null
mkdir -p "ab/pkg_$name"
cp -r "$dir/efficient-path-planner_amd/eppamd" "$dir"/efficient-path-planner_amd/*.so "ab/pkg_$name/"
rm -rf "$dir"
echo "ab/pkg_$name"
