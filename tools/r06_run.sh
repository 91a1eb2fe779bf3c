set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BASE=libqhuff.so REPS=3 WORKLOADS="corpus" timeout -k 10 800 bash tools/ab_cand.sh r06_ei libqhuff_ei.so > gpurun_out/r06_ei.txt 2>&1 || { cat gpurun_out/r06_ei.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ei.txt
