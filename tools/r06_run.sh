set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_k; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $o/pytest_gpu.log 2>&1 || { tail -30 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
timeout -k 10 200 python bench.py > $o/bench.json 2> $o/bench.err
python - $o/bench.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d['value'], d['enc_kernel_us'], d['dec_kernel_us'], d['roofline']['frac'], d['roofline']['frac_survey'])
q=d['workloads']['qif_corpus']; print('corpus', q['enc_kernel_us'], q['dec_kernel_us'], q['first_launch_us'])
PY
