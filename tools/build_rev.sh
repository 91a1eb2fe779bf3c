#!/bin/bash
# Build libqhuff.so of git revision REV (default HEAD) into
# ls-qpack_amd/<OUT> (default libqhuff_base.so), for A/Bs against the
# working tree.  Usage: tools/build_rev.sh [REV] [OUT]
set -e
rev=${1:-HEAD}
out=${2:-libqhuff_base.so}
root=$(cd "$(dirname "$0")/.." && pwd)
wt=$(mktemp -d /tmp/qhuff_rev.XXXXXX)
git -C "$root" worktree add -q --detach "$wt" "$rev"
make -s -C "$wt/ls-qpack_amd" -j8 > /dev/null
cp "$wt/ls-qpack_amd/libqhuff.so" "$root/ls-qpack_amd/$out"
git -C "$root" worktree remove --force "$wt"
echo "built $rev -> ls-qpack_amd/$out"
