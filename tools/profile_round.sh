#!/bin/bash
# One GPU profiling pass for the round: bench line, rocprofv3 kernel-trace
# stats of the same bench command, and separate FETCH_SIZE / WRITE_SIZE PMC
# passes.  Writes under gpurun_out/<tag>/.  Usage: tools/profile_round.sh TAG
set -e
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$tag
mkdir -p $o
B="bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path --no-workloads --no-overlap"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- python $B > $o/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/fetch -o run -- python $B > $o/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/write -o run -- python $B > $o/write.log 2>&1
python tools/pmc_summary.py $o/fetch $o/write 1048576 $o/pmc.json > /dev/null
cp $o/pmc.json $o/pmc_latest.json
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $o/bench.json 2> $o/bench.err
cat $o/bench.json
echo profile-done
