#!/bin/bash
# Build libmicrorts_amd.so of a git revision (default HEAD; WORKTREE = the working
# tree) into scripts/ab/libs/<name>.so, for same-box interleaved A/B runs
# (scripts/ab/ab_bench.sh).  Extra make variables after the revision, e.g. STAMPS=1.
#   bash scripts/ab/build_variant.sh <name> [rev] [VAR=value ...]
set -euo pipefail
NAME=$1; REV=${2:-HEAD}; shift $(( $# >= 2 ? 2 : 1 ))
REPO=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d /tmp/mrts_variant.XXXX)
if [ "$REV" = WORKTREE ]; then
  (cd "$REPO" && tar -cf - microrts-py_amd/csrc/*.hip microrts-py_amd/csrc/*.h microrts-py_amd/csrc/*.cpp microrts-py_amd/csrc/Makefile include) | tar -x -C "$T"
else
  git -C "$REPO" archive "$REV" microrts-py_amd/csrc include | tar -x -C "$T"
fi
mkdir -p "$REPO/scripts/ab/libs"
make -s -j3 -C "$T/microrts-py_amd/csrc" OUT="$REPO/scripts/ab/libs/$NAME.so" OBJDIR="$T/build" "$@"
rm -rf "$T"
echo "scripts/ab/libs/$NAME.so from $REV $*"
