#!/bin/bash
# Round-end evidence on one GPU box.  Every GPU step has its own time limit;
# a step that crashes or times out ends the session (a failing test does
# not stop the measurements).  Usage: tools/round_evidence.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=${1:-round_final}
o=gpurun_out/$tag
mkdir -p $o
fatal() { [ "$1" -ge 124 ] && { echo "step rc=$1: stopping"; exit "$1"; }; return 0; }
echo "== gpu suite"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 \
    --timeout-method thread > $o/pytest_gpu.log 2>&1
rc=$?; tail -2 $o/pytest_gpu.log; fatal $rc
echo "== smoke"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1
rc=$?; tail -1 $o/smoke.log; fatal $rc
echo "== bench"
timeout -k 10 300 python -u bench.py > $o/bench.json 2> $o/bench.err
rc=$?; head -c 600 $o/bench.json; echo; fatal $rc
echo "== bench config 4"
timeout -k 10 300 python -u bench.py --config4 --steps 20 --warmup 5 > $o/bench_config4.json 2> $o/bench_config4.err
rc=$?; head -c 400 $o/bench_config4.json; echo; fatal $rc
B="bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path --no-workloads --no-overlap"
echo "== rocprof kernel stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- python $B > $o/trace_bench.json 2> $o/trace.log
rc=$?; fatal $rc
find $o/trace -name "*kernel_stats.csv" -exec cp {} $o/kernel_stats.csv \;
grep qhuff $o/kernel_stats.csv | cut -c1-160
echo "== PMC"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/fetch -o run -- python $B > $o/fetch.log 2>&1
rc=$?; fatal $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/write -o run -- python $B > $o/write.log 2>&1
rc=$?; fatal $rc
python tools/pmc_summary.py $o/fetch $o/write 1048576 $o/pmc.json > /dev/null && cat $o/pmc.json | head -c 600; echo
echo "== SQ"
bash tools/sq_pass.sh $o/sq > $o/sq.txt 2>&1; tail -30 $o/sq.txt
echo "== phases"
# (the lean kernels by default: the profile build's stamps perturb the full
# decode kernel's register allocation; PHASE_KERNELS=full for those)
QHUFF_KERNELS=${PHASE_KERNELS:-lean} TIMELINE=1 SLOW=1 RAW=$o/raw.npz QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_prof.so \
    timeout -k 10 240 python -u tools/profile_phases.py > $o/phases.txt 2>&1
rc=$?; fatal $rc
python tools/wave_report.py $o/raw.npz > $o/wave_report.txt 2>&1
python tools/tail_report.py $o/raw.npz > $o/tail.txt 2>&1
cat $o/tail.txt
echo final-done
