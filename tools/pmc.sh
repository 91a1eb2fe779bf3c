#!/bin/bash
# PMC passes over tools/ablate.py (one counter group per pass, kernel-trace
# only, as the profiling guide prescribes).  Usage: tools/pmc.sh OUTDIR variants...
set -e
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o pmc -- python tools/ablate.py "$@" > "$out/p$i.log" 2>&1
done
echo pmc-done
