#!/bin/bash
# Build a previous commit's package + extension into ./ab_old (git-excluded; its build/ objects
# gpurun-ignored) for a same-box A/B against the working tree: `tools/gpu.sh abtree` then
# alternates bench.py runs of both trees on one GPU box (box-to-box spread is ~3 %, larger than
# the effects being measured).   usage: tools/ab_tree.sh <commit>
set -e
c=${1:?commit}
cd "$(dirname "$0")/.."
rm -rf ab_old /tmp/ab_old_wt
git worktree add -q /tmp/ab_old_wt "$c"
mkdir -p ab_old
cp -r /tmp/ab_old_wt/deep_vision_amd /tmp/ab_old_wt/csrc /tmp/ab_old_wt/bench.py ab_old/
git worktree remove --force /tmp/ab_old_wt
grep -qx "ab_old/" .git/info/exclude || echo "ab_old/" >> .git/info/exclude
rm -f ab_old/deep_vision_amd/*.so
(cd ab_old && python -c "from deep_vision_amd import _build; _build.build(verbose=False); _build.build_host(verbose=False)")
echo "ab_old/ = $c ($(git log -1 --format=%s "$c" | cut -c1-80))"
