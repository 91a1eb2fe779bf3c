# tickets claimed two iterations ahead (read after the codec) vs three: parity, A/B both orders, phases
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_x; mkdir -p $o
A=ls-qpack_amd
QHUFF_LIB=$PWD/$A/libqhuff_nc.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_concurrency.py tests/test_lsqpack_shim.py -m gpu -q -x --timeout 120 --timeout-method thread > $o/pytest_nc.log 2>&1
rc=$?; tail -1 $o/pytest_nc.log; [ $rc -ne 0 ] && exit $rc
for pair in "libqhuff_nc.so libqhuff.so" "libqhuff.so libqhuff_nc.so"; do
  set -- $pair
  timeout -k 10 300 python -u tools/ab_inproc.py $A/$1 $A/$2 8 10 > $o/ab_${1}_${2}.json || exit $?
  cat $o/ab_${1}_${2}.json
done
WORKLOAD=corpus timeout -k 10 300 python -u tools/ab_inproc.py $A/libqhuff_nc.so $A/libqhuff.so 6 5 > $o/ab_nc_corpus.json || exit $?
cat $o/ab_nc_corpus.json
TIMELINE=1 SLOW=1 RAW=$o/raw_profnc.npz QHUFF_LIB=$PWD/$A/libqhuff_profnc.so timeout -k 10 240 python -u tools/profile_phases.py > $o/phases_profnc.txt 2>&1 || exit $?
python tools/wave_report.py $o/raw_profnc.npz > $o/wave_report_profnc.txt 2>&1
grep -E "drain|wave end|age rank" $o/wave_report_profnc.txt
