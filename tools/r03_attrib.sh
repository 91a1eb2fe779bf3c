#!/bin/bash
# Attribution pass of a tree: per-phase stamps (prof build), SQ counter
# groups, kernel time vs batch size, one bench line.  Usage: TAG
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-r03_b}
mkdir -p $o
TIMELINE=1 QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_prof.so timeout -k 10 200 python -u tools/profile_phases.py > $o/phases_timeline.txt 2>&1
timeout -k 10 200 python -u tools/scaling.py > $o/scaling.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --cpu-seconds 0 --no-host-path > $o/bench.json 2> $o/bench.err
timeout -k 10 500 bash tools/sq_pass.sh $o/sq > $o/sq_counters.txt 2>&1
timeout -k 10 120 tools/micro/step_lab 32 > $o/step_lab.txt 2>&1
echo attrib-done
