#!/bin/bash
# Batch-size scan (tools/scaling.py) of two libraries on one box, A B A B
# in fresh processes.  Usage: tools/scal_ab.sh TAG LIB_A LIB_B [n ...]
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; a=$2; b=$3; shift 3
ns=${*:-64 4096 65536 196608 393216 1048576}
mkdir -p $o
for r in 1 2; do
  for l in $a $b; do
    QHUFF_LIB=$PWD/ls-qpack_amd/$l timeout -k 10 120 python -u tools/scaling.py $ns > $o/scal_${l%.so}_$r.txt 2>&1
  done
done
