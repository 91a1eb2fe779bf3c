# three library builds interleaved: a (libqhuff), b (_old), c (_d3)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ablib
rm -f gpurun_out/ablib/*.json
for i in 1 2 3; do
  for v in a:libqhuff.so b:libqhuff_old.so c:libqhuff_d3.so; do
    t=${v%%:*}; l=${v#*:}
    [ -f ls-qpack_amd/$l ] || continue
    QHUFF_LIB=$PWD/ls-qpack_amd/$l timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --cpu-seconds 0 --no-host-path > gpurun_out/ablib/$t$i.json 2>/dev/null || true
  done
done
