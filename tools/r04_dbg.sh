# two-ahead claims + youngest waves stop claiming near the end (QH_TAIL_STOP 2/4/6): A/B vs libqhuff.so
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_z2; mkdir -p $o
A=ls-qpack_amd
QHUFF_LIB=$PWD/$A/libqhuff_ts8.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_concurrency.py -m gpu -q -x --timeout 120 --timeout-method thread > $o/pytest_ts8.log 2>&1
rc=$?; tail -1 $o/pytest_ts8.log; [ $rc -ne 0 ] && exit $rc
for v in ts6 ts8 ts12; do
for pair in "libqhuff_$v.so libqhuff.so" "libqhuff.so libqhuff_$v.so"; do
  set -- $pair
  timeout -k 10 300 python -u tools/ab_inproc.py $A/$1 $A/$2 8 10 > $o/ab_${1}_${2}.json || exit $?
done
done
for f in $o/ab_*.json; do python -c "
import json; d=json.load(open('$f')); print(d['libs'][0].split('/')[-1], d['libs'][1].split('/')[-1], 'enc b/a', d['enc_b_over_a'], 'dec b/a', d['dec_b_over_a'], d['a_enc_med'], d['b_enc_med'], d['a_dec_med'], d['b_dec_med'])"; done
