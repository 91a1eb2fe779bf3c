# s3 (lean kernel by default, full kernel chosen per kind by the rare flag): parity auto + full, synthetic A/B vs HEAD and s2nb, corpus vs s2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_q; mkdir -p $o
A=ls-qpack_amd
T="tests/test_gpu_parity.py tests/test_lsqpack_shim.py tests/test_service.py tests/test_concurrency.py"
QHUFF_LIB=$PWD/$A/libqhuff_s3.so timeout -k 10 400 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread > $o/pytest_s3.log 2>&1
rc=$?; tail -3 $o/pytest_s3.log; [ $rc -ge 124 ] && exit $rc
QHUFF_KERNELS=full QHUFF_LIB=$PWD/$A/libqhuff_s3.so timeout -k 10 400 python -u -m pytest $T -m gpu -q --timeout 120 --timeout-method thread > $o/pytest_s3full.log 2>&1
rc=$?; tail -3 $o/pytest_s3full.log; [ $rc -ge 124 ] && exit $rc
for pair in "libqhuff_s3.so libqhuff.so" "libqhuff.so libqhuff_s3.so" "libqhuff_s3.so libqhuff_s2nb.so" "libqhuff_s2nb.so libqhuff_s3.so"; do
  set -- $pair
  timeout -k 10 300 python -u tools/ab_inproc.py $A/$1 $A/$2 8 10 > $o/ab_${1}_${2}.json || exit $?
  cat $o/ab_${1}_${2}.json
done
WORKLOAD=corpus timeout -k 10 300 python -u tools/ab_inproc.py $A/libqhuff_s3.so $A/libqhuff_s2.so 6 5 > $o/ab_s3_s2_corpus.json || exit $?
cat $o/ab_s3_s2_corpus.json
WORKLOAD=corpus timeout -k 10 300 python -u tools/ab_inproc.py $A/libqhuff_s3.so $A/libqhuff.so 6 5 > $o/ab_s3_head_corpus.json || exit $?
cat $o/ab_s3_head_corpus.json
