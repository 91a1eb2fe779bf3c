#!/bin/bash
# Candidate library CAND (ls-qpack_amd/<CAND>) against BASE (default
# libqhuff_base.so, e.g. from tools/build_rev.sh): GPU suite on the
# candidate (QHUFF_LIB), then in-process A/Bs (tools/ab_inproc.py) in both
# orders (the first library of a pair has shown a ~2 % encode bias).
# Optional third argument: also the step lab's refill A/B.
# Usage: TAG CAND [lab]
set -e
cd "$GRAFT_REPO_ROOT"
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
timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/$2 ls-qpack_amd/$b 20 10 > $o/ab_inproc.json
timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/$b ls-qpack_amd/$2 20 10 > $o/ab_inproc_swapped.json
python - $o <<'PY'
import json, sys
o = sys.argv[1]
a = json.load(open(o + "/ab_inproc.json"))
b = json.load(open(o + "/ab_inproc_swapped.json"))
for k in ("enc", "dec"):
    cand = (a["a_%s_med" % k] + b["b_%s_med" % k]) / 2
    base = (a["b_%s_med" % k] + b["a_%s_med" % k]) / 2
    print("%s: candidate %.2f us, base %.2f us (medians, both orders), cand/base %.4f"
          % (k, cand, base, cand / base))
PY
