# experiment record (profiles/r04_t1): the second-youngest waves stop claiming QH_TAIL_STOP1
# quarter-rounds before the end, with one more claim in their last iteration (liveness);
# libqhuff_t1{off,s2,s4}.so built with make -C ls-qpack_amd OUT=... DEFS=-DQH_TAIL_STOP1=0|2|4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_t1; mkdir -p $o
A=ls-qpack_amd
QHUFF_LIB=$PWD/$A/libqhuff_t1s4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_concurrency.py -m gpu -q -x --timeout 120 --timeout-method thread > $o/pytest_t1s4.log 2>&1
rc=$?; tail -1 $o/pytest_t1s4.log; [ $rc -ne 0 ] && exit $rc
for v in t1off t1s2 t1s4; do
for pair in "libqhuff_$v.so libqhuff.so" "libqhuff.so libqhuff_$v.so"; do
  set -- $pair
  timeout -k 10 300 python -u tools/ab_inproc.py $A/$1 $A/$2 8 10 > $o/ab_${1}_${2}.json || exit $?
done
done
for f in $o/ab_*.json; do python -c "
import json; d=json.load(open('$f')); print(d['libs'][0].split('/')[-1], d['libs'][1].split('/')[-1], 'enc b/a', d['enc_b_over_a'], 'dec b/a', d['dec_b_over_a'], d['a_enc_med'], d['b_enc_med'], d['a_dec_med'], d['b_dec_med'])"; done
