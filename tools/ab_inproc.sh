#!/bin/bash
# in-process A/B (tools/ab_inproc.py) of current libqhuff.so vs libqhuff_old.so
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-abin}
mkdir -p $o
timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/libqhuff.so ls-qpack_amd/libqhuff_old.so ${2:-20} ${3:-10} > $o/ab_inproc.json
cat $o/ab_inproc.json
