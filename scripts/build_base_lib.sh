#!/bin/bash
# Build libmiclip.so of a git revision (default HEAD) into build/ab/libmiclip_<rev>.so,
# for same-process / same-box A/B runs against the working tree's library:
#   MICLIP_LIB=build/ab/libmiclip_HEAD.so python scripts/bench_ops.py ...
set -eu
cd "$(dirname "$0")/.."
rev=${1:-HEAD}
tag=$(echo "$rev" | tr '/~^' '___')
wt=$(mktemp -d /tmp/miclip_ab.XXXXXX)
git worktree add -f --detach "$wt" "$rev" > /dev/null
make -C "$wt" -j8 > /dev/null
mkdir -p build/ab
cp "$wt/aihab-clip_amd/miclip/libmiclip.so" "build/ab/libmiclip_$tag.so"
git worktree remove --force "$wt"
echo "build/ab/libmiclip_$tag.so"
