set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_o; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_host_register.py tests/test_multi.py -x -v --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
timeout -k 10 300 python bench.py --host-path > $o/bench.json 2> $o/bench.err
python -c "import json;d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1]);print(d['value'], json.dumps(d.get('host_path')))"
