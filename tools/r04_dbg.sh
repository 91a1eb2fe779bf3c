# bench with the CPU leg last (hash-leg timing vs rocprof), and a corpus phase profile of the final tree
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_h2; mkdir -p $o
timeout -k 10 300 python -u bench.py > $o/bench.json 2> $o/bench.err || exit $?
B="bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path --no-workloads --no-overlap"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/trace -o run -- python $B > $o/trace_bench.json 2> $o/trace.log || exit $?
find $o/trace -name "*kernel_stats.csv" -exec cp {} $o/kernel_stats.csv \;
python - <<'P'
import json
b=json.loads(open("gpurun_out/r04_h2/bench.json").read().strip().splitlines()[-1])
print("value", b["value"], "enc", b["enc_kernel_us"], "dec", b["dec_kernel_us"], "hash", b["xxh32_headers"]["kernel_us"])
for l in open("gpurun_out/r04_h2/kernel_stats.csv"):
    if "qhuff" in l: print(l.strip()[:150])
P
WORKLOAD=corpus TIMELINE=1 RAW=$o/raw_corpus.npz QHUFF_KERNELS=full QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_prof.so timeout -k 10 240 python -u tools/profile_phases.py > $o/phases_corpus.txt 2>&1 || exit $?
python tools/tile_costs.py $o/raw_corpus.npz > $o/tile_costs_corpus.txt 2>&1
head -12 $o/tile_costs_corpus.txt
