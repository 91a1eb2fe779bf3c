# full kernels with a slot-held oldest pending tile (one more iteration of look-back slack): parity, corpus A/B, phases
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_far; mkdir -p $o
A=ls-qpack_amd
QHUFF_KERNELS=full QHUFF_LIB=$PWD/$A/libqhuff_far.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_concurrency.py tests/test_lsqpack_shim.py -m gpu -q -x --timeout 120 --timeout-method thread > $o/pytest_far_full.log 2>&1
rc=$?; tail -1 $o/pytest_far_full.log; [ $rc -ne 0 ] && exit $rc
QHUFF_LIB=$PWD/$A/libqhuff_far.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > $o/pytest_far.log 2>&1
rc=$?; tail -1 $o/pytest_far.log; [ $rc -ne 0 ] && exit $rc
for wl in corpus alphabet_c; do
for pair in "libqhuff_far.so libqhuff.so" "libqhuff.so libqhuff_far.so"; do
  set -- $pair
  WORKLOAD=$wl timeout -k 10 300 python -u tools/ab_inproc.py $A/$1 $A/$2 6 5 > $o/ab_${wl}_${1}_${2}.json || exit $?
done
done
for f in $o/ab_*.json; do python -c "
import json; d=json.load(open('$f')); print(d['workload'], d['libs'][0].split('/')[-1], d['libs'][1].split('/')[-1], 'enc b/a', d['enc_b_over_a'], 'dec b/a', d['dec_b_over_a'], d['a_enc_med'], d['b_enc_med'], d['a_dec_med'], d['b_dec_med'])"; done
WORKLOAD=corpus TIMELINE=1 RAW=$o/raw_corpus.npz QHUFF_KERNELS=full QHUFF_LIB=$PWD/$A/libqhuff_proffar.so timeout -k 10 240 python -u tools/profile_phases.py > $o/phases_corpus.txt 2>&1 || exit $?
grep -A1 "iter  3" $o/phases_corpus.txt | head -6
