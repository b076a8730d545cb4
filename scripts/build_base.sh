#!/bin/bash
# Build the committed tree's librtbvh.so (git HEAD, or $1) into ablib/librtbvh_base.so for A/B runs.
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/rtbvh_wt.XXXX)
git -C "$REPO" worktree add -f "$WT" "${1:-HEAD}" >/dev/null 2>&1
mkdir -p "$REPO/ablib"
make -C "$WT/raytracebvh_amd/csrc" -j8 OUT="$REPO/ablib/librtbvh_base.so" OBJDIR="$WT/obj" >/dev/null
git -C "$REPO" worktree remove --force "$WT"
git -C "$REPO" worktree prune
ls -la "$REPO/ablib/librtbvh_base.so"
