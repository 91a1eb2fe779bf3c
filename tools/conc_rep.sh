set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/conc
for i in 1 2 3 4; do
  timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu tests/test_concurrency.py > gpurun_out/conc/run$i.log 2>&1
done
