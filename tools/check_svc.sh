#!/bin/bash
# service suite + latency table on the GPU box.  Usage: TAG [calls]
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-svc}
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_service.py > $o/pytest_svc.log 2>&1
tail -3 $o/pytest_svc.log
timeout -k 10 400 python -u tools/svc_latency.py ${2:-1000} > $o/svc_latency.json 2> $o/svc_latency.err
cat $o/svc_latency.json
timeout -k 10 300 tools/svc_lat 3000 > $o/svc_lat_c.json
cat $o/svc_lat_c.json
