#!/bin/bash
# One GPU session of round 4.  Every GPU step has its own time limit; a step
# that crashes or times out ends the session (a failing test does not).
#   1. parity suite on the candidate CAND0 (QHUFF_LIB) when given
#   2. GPU suite on libqhuff.so
#   3. bench line (all legs) and rocprofv3 kernel stats of the same command
#   4. in-process A/B of each candidate against libqhuff.so: synthetic both
#      orders, corpus both orders
#   5. phase timelines (profile build) + tail report
# Usage: tools/r04_session.sh TAG [CAND.so ...]   (ls-qpack_amd/<CAND>)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
o=gpurun_out/$tag
mkdir -p $o
fatal() { [ "$1" -ge 124 ] && { echo "step rc=$1: stopping"; exit "$1"; }; return 0; }
if [ -n "$1" ]; then
  echo "== parity on $1"
  QHUFF_LIB=$PWD/ls-qpack_amd/$1 timeout -k 10 400 python -u -m pytest \
      tests/test_gpu_parity.py tests/test_lsqpack_shim.py -m gpu -x -q \
      --timeout 120 --timeout-method thread > $o/pytest_cand.log 2>&1
  rc=$?; tail -3 $o/pytest_cand.log; fatal $rc
fi
echo "== gpu suite"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
    --timeout-method thread > $o/pytest_gpu.log 2>&1
rc=$?; tail -3 $o/pytest_gpu.log; fatal $rc
echo "== bench"
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > $o/bench.json 2> $o/bench.err
rc=$?; head -c 1500 $o/bench.json; echo; fatal $rc
echo "== rocprof kernel stats (bench, no side legs)"
B="bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path --no-workloads --no-overlap"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- python $B > $o/trace_bench.json 2> $o/trace.log
rc=$?; fatal $rc
find $o/trace -name "*kernel_stats.csv" -exec cp {} $o/kernel_stats.csv \;
grep qhuff $o/kernel_stats.csv | cut -c1-140
for cand in "$@"; do
  for wl in synthetic corpus; do
    echo "== A/B $cand $wl"
    WORKLOAD=$wl timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/$cand ls-qpack_amd/libqhuff.so 12 10 > $o/ab_${cand}_${wl}_cb.json
    rc=$?; fatal $rc
    WORKLOAD=$wl timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/libqhuff.so ls-qpack_amd/$cand 12 10 > $o/ab_${cand}_${wl}_bc.json
    rc=$?; fatal $rc
    cat $o/ab_${cand}_${wl}_cb.json $o/ab_${cand}_${wl}_bc.json
  done
done
echo "== phases"
TIMELINE=1 SLOW=1 RAW=$o/raw.npz QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_prof.so \
    timeout -k 10 240 python -u tools/profile_phases.py > $o/phases.txt 2>&1
rc=$?; fatal $rc
python tools/tail_report.py $o/raw.npz > $o/tail.txt 2>&1
cat $o/tail.txt
echo session-done
