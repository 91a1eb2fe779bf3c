#!/bin/bash
# Candidate library CAND (ls-qpack_amd/<CAND>) against the default build:
# GPU suite on the candidate (QHUFF_LIB), then an in-process A/B
# (tools/ab_inproc.py).  Optional: the step lab's refill A/B.  Usage: TAG CAND [lab]
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1
mkdir -p $o
if [ -n "$3" ]; then
  timeout -k 10 200 tools/micro/step_lab 32 ab > $o/step_lab.txt 2>&1
fi
QHUFF_LIB=$PWD/ls-qpack_amd/$2 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $o/pytest_gpu.log 2>&1
tail -1 $o/pytest_gpu.log
timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/$2 ls-qpack_amd/libqhuff.so 20 10 > $o/ab_inproc.json
cat $o/ab_inproc.json
