# experiment record (profiles/r04_tune): the variant libraries were built with
# make -C ls-qpack_amd OUT=libqhuff_<v>.so OBJDIR=build_<v> DEFS=-DQH_SPIN_BACKOFF=4|16 / -DQH_TAIL_STOP=5|7
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_tune; mkdir -p $o
A=ls-qpack_amd
for v in bo4 bo16 ts5 ts7; do
for pair in "libqhuff_$v.so libqhuff.so" "libqhuff.so libqhuff_$v.so"; do
  set -- $pair
  timeout -k 10 300 python -u tools/ab_inproc.py $A/$1 $A/$2 8 10 > $o/ab_${1}_${2}.json || exit $?
done
done
for f in $o/ab_*.json; do python -c "
import json; d=json.load(open('$f')); print(d['libs'][0].split('/')[-1], d['libs'][1].split('/')[-1], 'enc b/a', d['enc_b_over_a'], 'dec b/a', d['dec_b_over_a'])"; done
