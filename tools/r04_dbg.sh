# on top of the late double claim: depth 2, 10 and 8 waves per workgroup
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_v; mkdir -p $o
A=ls-qpack_amd
for v in lcd2 lcw10 lcw8; do
  QHUFF_LIB=$PWD/$A/libqhuff_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "launch_shapes or kats or big_tile" --timeout 120 --timeout-method thread > $o/pytest_$v.log 2>&1
  rc=$?; tail -1 $o/pytest_$v.log; [ $rc -ne 0 ] && exit $rc
  for pair in "libqhuff_$v.so libqhuff_lc.so" "libqhuff_lc.so libqhuff_$v.so"; do
    set -- $pair
    timeout -k 10 300 python -u tools/ab_inproc.py $A/$1 $A/$2 8 10 > $o/ab_${1}_${2}.json || exit $?
    cat $o/ab_${1}_${2}.json
  done
done
