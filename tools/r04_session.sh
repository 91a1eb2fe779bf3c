#!/bin/bash
# One GPU session of round 4: GPU suite, bench line, rocprofv3 kernel stats of
# the same bench command, phase timelines (profile build) and optional A/B
# candidates.  Every GPU step has its own time limit; the steps are chained
# so that a failure stops the session.  Usage: tools/r04_session.sh TAG
# [CAND.so ...]  (candidates: ls-qpack_amd/<CAND>, A/B against libqhuff.so)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
o=gpurun_out/$tag
mkdir -p $o
echo "== gpu suite"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
    --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -30 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
echo "== bench"
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > $o/bench.json 2> $o/bench.err
head -c 600 $o/bench.json; echo
echo "== rocprof kernel stats (bench, no side legs)"
B="bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path --no-workloads --no-overlap"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- python $B > $o/trace_bench.json 2> $o/trace.log
find $o/trace -name "*kernel_stats.csv" -exec cp {} $o/kernel_stats.csv \;
grep qhuff $o/kernel_stats.csv | cut -c1-140
echo "== phases"
TIMELINE=1 SLOW=1 RAW=$o/raw.npz QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_prof.so \
    timeout -k 10 240 python -u tools/profile_phases.py > $o/phases.txt 2>&1
python tools/tail_report.py $o/raw.npz > $o/tail.txt 2>&1 || true
cat $o/tail.txt
for cand in "$@"; do
  echo "== A/B $cand"
  for r in 1 2; do
    timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/$cand ls-qpack_amd/libqhuff.so 20 10 > $o/ab_${cand}_${r}_cb.json
    timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/libqhuff.so ls-qpack_amd/$cand 20 10 > $o/ab_${cand}_${r}_bc.json
    cat $o/ab_${cand}_${r}_cb.json $o/ab_${cand}_${r}_bc.json
  done
done
echo session-done
