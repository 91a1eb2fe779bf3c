#!/bin/bash
# Phase timelines (prof builds) of two libraries: TAG LIB_A LIB_B
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1
mkdir -p $o
TIMELINE=1 SLOW=1 QHUFF_LIB=$PWD/ls-qpack_amd/$2 timeout -k 10 200 python -u tools/profile_phases.py > $o/phases_a.txt 2>&1
TIMELINE=1 SLOW=1 QHUFF_LIB=$PWD/ls-qpack_amd/$3 timeout -k 10 200 python -u tools/profile_phases.py > $o/phases_b.txt 2>&1
echo phases-done
