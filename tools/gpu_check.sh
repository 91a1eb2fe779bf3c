#!/bin/bash
# one GPU test file (or node id) on the box, under a time limit:
# tools/gpu_check.sh TESTS...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest "$@" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_check.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_check.log
exit $rc
