#!/bin/bash
# Builds the library of a git revision (default HEAD) as A/B variant "prev":
#   tools/ab_prev.sh [rev]  ->  tools/bin/ab/prev/libneurokmer.so
set -eu
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/nk_wt.XXXXXX)
git -C "$ROOT" worktree add -f "$WT" "$REV" -q
make -s -j8 -C "$WT/neurokmer_amd/csrc" OBJDIR="$WT/obj" LIBDIR="$ROOT/tools/bin/ab/prev" \
  "$ROOT/tools/bin/ab/prev/libneurokmer.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "$ROOT/tools/bin/ab/prev/libneurokmer.so ($REV)"
