# kernel times (tools/scaling.py at 1M strings) + the two SQ counter passes
# for each library variant: tools/exp_pmc.sh OUTDIR LIB...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=$1; shift
mkdir -p "$out"
for lib in "$@"; do
  name=$(basename "$lib" .so)
  d="$out/$name"
  mkdir -p "$d"
  QHUFF_LIB=$PWD/$lib timeout -k 10 120 python -u tools/scaling.py 1048576 > "$d/times.txt" 2>&1
  QHUFF_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d "$d/p1" -o pmc -- python tools/scaling.py 1048576 > "$d/p1.log" 2>&1
  QHUFF_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE --output-format csv -d "$d/p2" -o pmc -- python tools/scaling.py 1048576 > "$d/p2.log" 2>&1
  python tools/pmc_median.py "$d" > "$d/summary.txt"
  rm -rf "$d/p1" "$d/p2"
  echo "== $name"; cat "$d/times.txt" "$d/summary.txt"
done
