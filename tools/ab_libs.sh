# bench lines for two library builds, interleaved A B A B A B
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ablib
rm -f gpurun_out/ablib/*.json
A=${1:-ls-qpack_amd/libqhuff.so}; B=${2:-ls-qpack_amd/libqhuff_old.so}
for i in 1 2 3; do
  QHUFF_LIB=$PWD/$A timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --cpu-seconds 0 --no-host-path > gpurun_out/ablib/a$i.json 2>/dev/null
  QHUFF_LIB=$PWD/$B timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --cpu-seconds 0 --no-host-path > gpurun_out/ablib/b$i.json 2>/dev/null
done
