set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_m; mkdir -p $o
QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_rf.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $o/pytest_gpu.log 2>&1 || { tail -30 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
NOTEST=1 REPS=3 BASE="libqhuff_base.so" WORKLOADS="corpus" timeout -k 10 600 tools/ab_cand.sh r06_m/ab libqhuff_rf.so > $o/ab.txt 2>&1
grep -v amdgpu.ids $o/ab.txt
B="bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path --no-workloads --no-overlap"
export QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_rf.so
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o/fetch -o run -- python $B > $o/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o/write -o run -- python $B > $o/write.log 2>&1
python tools/pmc_summary.py $o/fetch $o/write 1048576 $o/pmc.json | head -c 900
