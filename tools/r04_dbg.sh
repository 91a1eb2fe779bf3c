# synthetic A/B: big-tile path vs round-3 slow path vs mtrep-only vs HEAD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_m; mkdir -p $o
A=ls-qpack_amd
for pair in "libqhuff_big3.so libqhuff_r3slow.so" "libqhuff_r3slow.so libqhuff_mtrep.so" "libqhuff_big3.so libqhuff_mtrep.so" "libqhuff_mtrep.so libqhuff.so"; do
  set -- $pair
  timeout -k 10 300 python -u tools/ab_inproc.py $A/$1 $A/$2 12 10 > $o/ab_${1}_${2}.json || exit $?
  cat $o/ab_${1}_${2}.json
done
