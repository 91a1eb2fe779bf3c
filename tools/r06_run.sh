set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_p; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_memory.py tests/test_concurrency.py tests/test_multi.py -x -v --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
timeout -k 10 300 python bench.py --no-host-path --no-workloads --cpu-seconds 0 > $o/bench.json 2> $o/bench.err
python -c "import json;d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['enc_kernel_us'], d['dec_kernel_us'], json.dumps(d.get('two_streams')))"
