#!/bin/bash
# c5_native against libepp as of git revision $1 (scripts/dbg/c5_native_$2), for
# scripts/c5_ab.py (diagnostics A/B on one box).
set -eu
cd "$(dirname "$0")/.."
bash scripts/ab_build.sh "$1" "$2" > /dev/null
/opt/rocm/bin/hipcc -O2 -std=c++17 -ffp-contract=off -Iinclude -o "scripts/dbg/c5_native_$2" tools/c5_native.cpp \
  -Lscripts/dbg -l:"libepp_$2.so" -Wl,-rpath,'$ORIGIN'
echo "scripts/dbg/c5_native_$2"
