# interleaved bench A/B of two library builds + the GPU parity suite on A:
# tools/ab_quick.sh LIB_A LIB_B TAG
set -e
cd $GRAFT_REPO_ROOT
o=gpurun_out/$3
mkdir -p $o
QHUFF_LIB=$PWD/$1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $o/pytest_a.log 2>&1
tail -n 1 $o/pytest_a.log
timeout -k 10 900 bash tools/ab_libs.sh $1 $2 > $o/ab.log 2>&1
python tools/ab_show.py > $o/ab.txt 2>&1 || true
cat $o/ab.txt
