#!/bin/bash
# Corpus-decode A/Bs of several compile-time variants against BASE
# (libqhuff_base.so): VARS="s64 c96" names ls-qpack_amd/libqhuff_<v>.so
# (built with make OUT=libqhuff_<v>.so OBJDIR=build_<v> DEFS=...), two
# rounds of in-process pairs in both orders (tools/ab_inproc.py, R rounds
# of 5 launches each, WORKLOAD=corpus) into gpurun_out/$OUTD.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${OUTD}; mkdir -p $o
for rep in 1 2; do for n in ${VARS}; do
  WORKLOAD=corpus timeout -k 10 200 python -u tools/ab_inproc.py ls-qpack_amd/libqhuff_$n.so ls-qpack_amd/libqhuff_base.so ${R:-6} 5 > $o/${n}_${rep}_cb.json
  WORKLOAD=corpus timeout -k 10 200 python -u tools/ab_inproc.py ls-qpack_amd/libqhuff_base.so ls-qpack_amd/libqhuff_$n.so ${R:-6} 5 > $o/${n}_${rep}_bc.json
  echo done $n
done; done
