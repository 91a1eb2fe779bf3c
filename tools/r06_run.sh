set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_d; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $o/pytest_gpu.log 2>&1 || { tail -30 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
for r in 1 2; do
  for L in norec lazy; do
    QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_$L.so timeout -k 10 200 python bench.py --no-workloads --no-host-path --no-overlap --cpu-seconds 0 --steps 300 > $o/bench_${L}_$r.json 2>/dev/null
    python -c "import json,sys;d=json.loads(open('$o/bench_${L}_$r.json').read().strip().splitlines()[-1]);print('$L',d['value'],d['enc_kernel_us'],d['dec_kernel_us'])"
  done
done
