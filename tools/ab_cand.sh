#!/bin/bash
# Candidate library CAND (ls-qpack_amd/<CAND>) against BASE (default
# libqhuff_base.so, e.g. from tools/build_rev.sh): GPU suite on the
# candidate (QHUFF_LIB; skipped with NOTEST=1), then REPS (default 3) pairs
# of in-process A/Bs (tools/ab_inproc.py), each pair in both orders, each in
# a fresh process (the first library's context of a process has shown a
# 2-4 % bias, which the pairs cancel).  Optional third argument: also the
# step lab's refill A/B.  WORKLOADS="corpus alphabet_c": one more pair per
# real-workload batch (qhuff/workload.py), printed after the summary.
# Usage: TAG CAND [lab]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1
b=${BASE:-libqhuff_base.so}
mkdir -p $o
if [ -n "$3" ]; then
  timeout -k 10 200 tools/micro/step_lab 32 ab > $o/step_lab.txt 2>&1
fi
if [ -z "$NOTEST" ]; then
  QHUFF_LIB=$PWD/ls-qpack_amd/$2 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $o/pytest_gpu.log 2>&1
  tail -1 $o/pytest_gpu.log
fi
for r in $(seq 1 ${REPS:-3}); do
  timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/$2 ls-qpack_amd/$b 20 10 > $o/ab_${r}_cb.json
  timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/$b ls-qpack_amd/$2 20 10 > $o/ab_${r}_bc.json
done
for w in $WORKLOADS; do
  WORKLOAD=$w timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/$2 ls-qpack_amd/$b 6 5 > $o/wl_${w}_cb.json
  WORKLOAD=$w timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/$b ls-qpack_amd/$2 6 5 > $o/wl_${w}_bc.json
done
python - $o <<'PY'
import glob, json, statistics, sys
o = sys.argv[1]
rat = {"enc": [], "dec": []}
cand = {"enc": [], "dec": []}
base = {"enc": [], "dec": []}
for f in sorted(glob.glob(o + "/ab_*_cb.json")):
    a = json.load(open(f))
    b = json.load(open(f.replace("_cb.json", "_bc.json")))
    for k in ("enc", "dec"):
        c = (a["a_%s_med" % k] + b["b_%s_med" % k]) / 2
        s = (a["b_%s_med" % k] + b["a_%s_med" % k]) / 2
        cand[k].append(c); base[k].append(s); rat[k].append(c / s)
for k in ("enc", "dec"):
    print("%s: candidate %.2f us, base %.2f us, cand/base %.4f (pairs: %s)"
          % (k, statistics.mean(cand[k]), statistics.mean(base[k]),
             statistics.mean(rat[k]), " ".join("%.3f" % r for r in rat[k])))
json.dump({"cand": cand, "base": base, "ratio": rat}, open(o + "/ab_summary.json", "w"))
PY
for w in $WORKLOADS; do
  python - $o/wl_${w}_cb.json $o/wl_${w}_bc.json <<'PY'
import json, sys
a, b = (json.load(open(f)) for f in sys.argv[1:3])
for k in ("enc", "dec"):
    c = (a["a_%s_med" % k] + b["b_%s_med" % k]) / 2
    s = (a["b_%s_med" % k] + b["a_%s_med" % k]) / 2
    print("%s %s: candidate %.2f us, base %.2f us, cand/base %.4f"
          % (a["workload"], k, c, s, c / s))
PY
done
