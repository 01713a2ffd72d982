#!/bin/bash
# Populate ab_old/ (git-ignored, shipped to the GPU box) with the tree of a previous revision for A/B runs.
set -e
rev=${1:-HEAD~1}
root=$(git rev-parse --show-toplevel)
rm -rf /tmp/ncc_ab_wt "$root/ab_old"
git -C "$root" worktree add -f /tmp/ncc_ab_wt "$rev" -q
mkdir "$root/ab_old"
(cd /tmp/ncc_ab_wt && tar cf - --exclude=.git --exclude=gpurun_out --exclude=profiles .) | (cd "$root/ab_old" && tar xf -)
rm -f "$root"/ab_old/ncc/_native*.so
git -C "$root" worktree remove --force /tmp/ncc_ab_wt
echo "ab_old = $(git -C "$root" rev-parse --short "$rev")"
