#!/bin/bash
# A/B on one box: ls-qpack_amd/libqhuff.so (candidate) against
# ls-qpack_amd/libqhuff_base.so (tools/build_rev.sh), the synthetic token
# batch (REPS pairs, both orders) and the QIF corpus (one pair), each run a
# fresh process (tools/ab_inproc.py); optional GPU suite first.
# Usage: tools/ab_pair.sh TAG [test]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=gpurun_out/$1; mkdir -p $o
if [ "$2" = test ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1
  rc=$?
  tail -15 $o/pytest.log
  echo "pytest rc=$rc"
  [ $rc -le 1 ] || exit 1
fi
for r in $(seq 1 ${REPS:-1}); do
  timeout -k 10 200 python -u tools/ab_inproc.py ls-qpack_amd/libqhuff.so ls-qpack_amd/libqhuff_base.so 12 8 > $o/ab_${r}_cb.json || exit 1
  timeout -k 10 200 python -u tools/ab_inproc.py ls-qpack_amd/libqhuff_base.so ls-qpack_amd/libqhuff.so 12 8 > $o/ab_${r}_bc.json || exit 1
done
if [ -z "$NOCORPUS" ]; then
  WORKLOAD=corpus timeout -k 10 200 python -u tools/ab_inproc.py ls-qpack_amd/libqhuff.so ls-qpack_amd/libqhuff_base.so 6 5 > $o/ab_corpus_cb.json || exit 1
  WORKLOAD=corpus timeout -k 10 200 python -u tools/ab_inproc.py ls-qpack_amd/libqhuff_base.so ls-qpack_amd/libqhuff.so 6 5 > $o/ab_corpus_bc.json || exit 1
fi
python - $o <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/ab_*.json")):
    d = json.load(open(f))
    cand = "a" if d["libs"][0].endswith("libqhuff.so") else "b"
    base = "b" if cand == "a" else "a"
    print("%-28s enc cand %8.2f base %8.2f | dec cand %8.2f base %8.2f"
          % (f.split("/")[-1], d[cand + "_enc_med"], d[base + "_enc_med"],
             d[cand + "_dec_med"], d[base + "_dec_med"]))
PY
