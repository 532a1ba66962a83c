#!/usr/bin/env bash
# Compile the reference solvers from their own single source files, exactly as
# their file headers say (cavity-01.cpp:18, channel-01.cpp:19,
# backwards_step-01.cpp:20): g++ -std=c++17 -O2 -Wall <file> -o <name>.
# Outputs go ONLY to oracle/_ref/ (git-ignored). Nothing is copied from the
# reference tree; the sources are compiled where they lie.
# Usage: oracle/build_ref.sh [REF_DIR]   (default /root/reference)
set -euo pipefail
REF="${1:-/root/reference}"
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="$HERE/_ref"
mkdir -p "$OUT"
if [ ! -d "$REF" ]; then
  echo "reference tree $REF not present; skipping reference build" >&2
  exit 0
fi
for pair in cavity:cavity-01.cpp channel:channel-01.cpp backwards_step:backwards_step-01.cpp; do
  name="${pair%%:*}"; src="${pair#*:}"
  if [ ! -x "$OUT/$name" ] || [ "$REF/$src" -nt "$OUT/$name" ]; then
    g++ -std=c++17 -O2 -Wall "$REF/$src" -o "$OUT/$name"
  fi
done
echo "built reference binaries into $OUT"
