#!/bin/bash
# PMC passes over tools/scaling.py (1M strings, enc + dec, 23 launches each):
# one counter group per rocprofv3 run (kernel trace only), summarised per
# kernel by tools/pmc_median.py.  Usage: tools/pmc_pass.sh OUTDIR
set -e
out=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_SMEM" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o pmc -- python tools/scaling.py 1048576 > "$out/p$i.log" 2>&1
done
python tools/pmc_median.py "$out"
