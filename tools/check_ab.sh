#!/bin/bash
# GPU suite on the current tree, then an interleaved A/B of the bench line:
# current libqhuff.so vs libqhuff_old.so.  Usage: TAG
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-ab}
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $o/pytest_gpu.log 2>&1
bash tools/ab_libs.sh ls-qpack_amd/libqhuff.so ls-qpack_amd/libqhuff_old.so
python tools/ab_show.py > $o/ab.txt
cat $o/ab.txt
