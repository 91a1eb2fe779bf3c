set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in 3 2 4; do
  if [ $L = 3 ]; then unset NOTEST; else export NOTEST=1; fi
  BASE=libqhuff.so REPS=2 WORKLOADS="corpus" timeout -k 10 600 bash tools/ab_cand.sh r06_late/l$L libqhuff_l$L.so > gpurun_out/r06_late_l$L.txt 2>&1 || { cat gpurun_out/r06_late_l$L.txt; exit 1; }
  echo "== L=$L"; cat gpurun_out/r06_late_l$L.txt
done
