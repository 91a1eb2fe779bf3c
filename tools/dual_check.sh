# QH_DUAL experiment: GPU parity suite on the dual library, then on the
# default library, then interleaved bench A/B (dual vs default)
set -e
cd $GRAFT_REPO_ROOT
o=gpurun_out/dual
mkdir -p $o
QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_dual.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $o/pytest_dual.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $o/pytest_default.log 2>&1
timeout -k 10 900 bash tools/ab_libs.sh ls-qpack_amd/libqhuff_dual.so ls-qpack_amd/libqhuff.so > $o/ab.log 2>&1
python tools/ab_show.py gpurun_out/ablib > $o/ab_summary.txt 2>&1 || true
cat $o/ab_summary.txt
