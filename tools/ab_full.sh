#!/bin/bash
# Candidate CAND (ls-qpack_amd/<CAND>) against libqhuff_base.so with both
# libraries pinned to their full kernels (QHUFF_KERNELS=full), in-process
# pairs in both orders (tools/ab_inproc.py), into gpurun_out/TAG.
# Usage: TAG CAND
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1
mkdir -p $o
for r in $(seq 1 ${REPS:-2}); do
  timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/$2@QHUFF_KERNELS=full ls-qpack_amd/libqhuff_base.so@QHUFF_KERNELS=full 20 10 > $o/full_${r}_cb.json
  timeout -k 10 300 python -u tools/ab_inproc.py ls-qpack_amd/libqhuff_base.so@QHUFF_KERNELS=full ls-qpack_amd/$2@QHUFF_KERNELS=full 20 10 > $o/full_${r}_bc.json
done
python - $o <<'PY'
import glob, json, sys
o = sys.argv[1]
for f in sorted(glob.glob(o + "/full_*_cb.json")):
    a = json.load(open(f)); b = json.load(open(f.replace("_cb", "_bc")))
    print("full: enc %.4f %.4f  dec %.4f %.4f (cand/base)" % (
        a["a_enc_med"] / a["b_enc_med"], b["b_enc_med"] / b["a_enc_med"],
        a["a_dec_med"] / a["b_dec_med"], b["b_dec_med"] / b["a_dec_med"]))
PY
