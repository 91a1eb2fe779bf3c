# slot-based big tiles: parity, synthetic A/B both orders vs HEAD and r3slow, corpus A/B, corpus profile
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_n; mkdir -p $o
A=ls-qpack_amd
QHUFF_LIB=$PWD/$A/libqhuff_slot.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_lsqpack_shim.py tests/test_service.py tests/test_concurrency.py -m gpu -q --timeout 120 --timeout-method thread > $o/pytest_slot.log 2>&1
rc=$?; tail -3 $o/pytest_slot.log; [ $rc -ge 124 ] && exit $rc
for pair in "libqhuff_slot.so libqhuff.so" "libqhuff.so libqhuff_slot.so" "libqhuff_r3slow.so libqhuff.so" "libqhuff.so libqhuff_r3slow.so"; do
  set -- $pair
  timeout -k 10 300 python -u tools/ab_inproc.py $A/$1 $A/$2 10 10 > $o/ab_${1}_${2}.json || exit $?
  cat $o/ab_${1}_${2}.json
done
WORKLOAD=corpus timeout -k 10 300 python -u tools/ab_inproc.py $A/libqhuff_slot.so $A/libqhuff.so 6 5 > $o/ab_slot_corpus.json || exit $?
cat $o/ab_slot_corpus.json
WORKLOAD=corpus RAW=$o/raw_slot.npz QHUFF_LIB=$PWD/$A/libqhuff_profslot.so timeout -k 10 240 python -u tools/profile_phases.py > $o/phases_slot.txt 2>&1 || exit $?
python tools/tile_costs.py $o/raw_slot.npz > $o/tile_costs_slot.txt 2>&1; head -24 $o/tile_costs_slot.txt
