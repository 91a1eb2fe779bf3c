#!/bin/bash
# GPU suite on the current tree and on libqhuff_d3.so, then an interleaved
# A/B/C of the bench line (tools/ab3.sh).  Usage: TAG
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-ab3}
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $o/pytest_gpu.log 2>&1
QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_d3.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_concurrency.py tests/test_exhaustive.py > $o/pytest_gpu_d3.log 2>&1
bash tools/ab3.sh
python tools/ab_show.py > $o/ab.txt
cat $o/ab.txt
