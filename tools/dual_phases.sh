# QH_DUAL experiment: per-phase stamps of the default and dual decode, and a
# bench A/B of the depth-3 dual build
set -e
cd $GRAFT_REPO_ROOT
o=gpurun_out/dual2
mkdir -p $o
QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_prof.so timeout -k 10 200 python -u tools/profile_phases.py > $o/phases_default.txt 2>&1
QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_dual_prof.so timeout -k 10 200 python -u tools/profile_phases.py > $o/phases_dual.txt 2>&1
timeout -k 10 900 bash tools/ab_libs.sh ls-qpack_amd/libqhuff_dual3.so ls-qpack_amd/libqhuff.so > $o/ab.log 2>&1
python tools/ab_show.py > $o/ab_dual3.txt 2>&1 || true
cat $o/ab_dual3.txt
