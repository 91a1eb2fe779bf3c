#!/bin/bash
# SQ counter passes over tools/scaling.py (1M strings, enc + dec, 23
# launches each): one counter group per rocprofv3 run (kernel trace only,
# no other tracing), summarised per kernel by tools/pmc_median.py.  A pass
# that fails is reported and skipped.  Usage: tools/sq_pass.sh OUTDIR
out=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" ; do
  i=$((i+1))
  if timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o pmc -- python tools/scaling.py 1048576 > "$out/p$i.log" 2>&1; then
    echo "pass $i ok: $grp"
  else
    echo "pass $i FAILED ($?): $grp"
  fi
done
python tools/pmc_median.py "$out"
