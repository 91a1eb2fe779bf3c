# cooperative bitmaps in the strings' own arena slots: parity (full kernels), corpus + synthetic A/B, corpus tile costs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_bm; mkdir -p $o
A=ls-qpack_amd
QHUFF_KERNELS=full QHUFF_LIB=$PWD/$A/libqhuff_bm.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_service.py tests/test_lsqpack_shim.py -m gpu -q -x --timeout 120 --timeout-method thread > $o/pytest_bm_full.log 2>&1
rc=$?; tail -1 $o/pytest_bm_full.log; [ $rc -ne 0 ] && exit $rc
QHUFF_LIB=$PWD/$A/libqhuff_bm.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_concurrency.py -m gpu -q -x --timeout 120 --timeout-method thread > $o/pytest_bm.log 2>&1
rc=$?; tail -1 $o/pytest_bm.log; [ $rc -ne 0 ] && exit $rc
for wl in corpus synthetic; do
for pair in "libqhuff_bm.so libqhuff.so" "libqhuff.so libqhuff_bm.so"; do
  set -- $pair
  WORKLOAD=$wl timeout -k 10 300 python -u tools/ab_inproc.py $A/$1 $A/$2 6 5 > $o/ab_${wl}_${1}_${2}.json || exit $?
done
done
for f in $o/ab_*.json; do python -c "
import json; d=json.load(open('$f')); print(d['workload'], d['libs'][0].split('/')[-1], d['libs'][1].split('/')[-1], 'enc b/a', d['enc_b_over_a'], 'dec b/a', d['dec_b_over_a'], d['a_enc_med'], d['b_enc_med'], d['a_dec_med'], d['b_dec_med'])"; done
WORKLOAD=corpus TIMELINE=1 RAW=$o/raw_corpus.npz QHUFF_KERNELS=full QHUFF_LIB=$PWD/$A/libqhuff_profbm.so timeout -k 10 240 python -u tools/profile_phases.py > $o/phases_corpus.txt 2>&1 || exit $?
python tools/tile_costs.py $o/raw_corpus.npz > $o/tile_costs_corpus.txt 2>&1
head -12 $o/tile_costs_corpus.txt
