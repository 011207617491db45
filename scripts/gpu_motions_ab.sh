# A/B of motion-kernel builds on C3 (each run its own process, time-limited): a reference
# build (e.g. HEAD's library built into scripts/dbg/libepp_head.so) against the tree's.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for cfg in "scripts/dbg/libepp_head.so" "" "scripts/dbg/libepp_head.so" ""; do
  timeout -k 10 120 python scripts/motions_ab.py $cfg || exit $?
done
