#!/bin/bash
# Build libkrylov_amd.so as of git revision $1 into $2 (for same-box A/B runs:
# KRYLOV_AMD_LIB=$2 python bench.py ...). Uses a temporary worktree.
set -e
rev=$1; out=$(realpath -m $2)
wt=$(mktemp -d /tmp/krwt.XXXX)
git worktree add -q --detach $wt $rev
make -s -C $wt/parallel-krylov_amd/csrc -j8 OUT=$out BUILD=$wt/build >/dev/null
git worktree remove --force $wt
echo "built $rev -> $out"
