# experiment record (profiles/r04_et): encode table loads issued behind the ticket atomics
# and stored after them (libqhuff_et.so); neutral, not kept
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_et; mkdir -p $o
A=ls-qpack_amd
QHUFF_LIB=$PWD/$A/libqhuff_et.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_service.py -m gpu -q -x --timeout 120 --timeout-method thread > $o/pytest_et.log 2>&1
rc=$?; tail -1 $o/pytest_et.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for pair in "libqhuff_et.so libqhuff.so" "libqhuff.so libqhuff_et.so"; do
  set -- $pair
  timeout -k 10 300 python -u tools/ab_inproc.py $A/$1 $A/$2 8 10 > $o/ab_${r}_${1}_${2}.json || exit $?
done
done
for f in $o/ab_*.json; do python -c "
import json; d=json.load(open('$f')); print(d['libs'][0].split('/')[-1], d['libs'][1].split('/')[-1], 'enc b/a', d['enc_b_over_a'], 'dec b/a', d['dec_b_over_a'], d['a_enc_med'], d['b_enc_med'])"; done
