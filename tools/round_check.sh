# full GPU suite + smoke + profile pass for a checkpoint: TAG
set -e
cd $GRAFT_REPO_ROOT
tag=${1:-r02_b}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/$tag/pytest_gpu.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$tag/smoke.log 2>&1
timeout -k 10 700 bash tools/profile_round.sh $tag > gpurun_out/$tag/profile.log 2>&1
TIMELINE=1 timeout -k 10 200 python -u tools/profile_phases.py > gpurun_out/$tag/phases_timeline.txt 2>&1
