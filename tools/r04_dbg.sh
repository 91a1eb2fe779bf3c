# look-back re-polls of invalid flags only (rp), + spin backoff (rpb): parity, A/B vs libqhuff.so, phases
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_y; mkdir -p $o
A=ls-qpack_amd
QHUFF_LIB=$PWD/$A/libqhuff_rp.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_concurrency.py -m gpu -q -x --timeout 120 --timeout-method thread > $o/pytest_rp.log 2>&1
rc=$?; tail -1 $o/pytest_rp.log; [ $rc -ne 0 ] && exit $rc
for v in rp rpb; do
for pair in "libqhuff_$v.so libqhuff.so" "libqhuff.so libqhuff_$v.so"; do
  set -- $pair
  timeout -k 10 300 python -u tools/ab_inproc.py $A/$1 $A/$2 8 10 > $o/ab_${1}_${2}.json || exit $?
  cat $o/ab_${1}_${2}.json
done
done
TIMELINE=1 SLOW=1 RAW=$o/raw_profrp.npz QHUFF_LIB=$PWD/$A/libqhuff_profrp.so timeout -k 10 240 python -u tools/profile_phases.py > $o/phases_profrp.txt 2>&1 || exit $?
python tools/wave_report.py $o/raw_profrp.npz > $o/wave_report_profrp.txt 2>&1
grep -E "drain|wave end|age rank" $o/wave_report_profrp.txt
