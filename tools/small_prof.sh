set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r03_smallp
mkdir -p $o
for n in 4096 65536 196608; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o/n$n -o run -- python3 -u tools/scaling.py $n > $o/n$n.txt 2>&1
done
N=4096 QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_prof.so timeout -k 10 120 python -u tools/profile_phases.py > $o/phases_4096.txt 2>&1
N=196608 SLOW=1 QHUFF_LIB=$PWD/ls-qpack_amd/libqhuff_prof.so timeout -k 10 120 python -u tools/profile_phases.py > $o/phases_196608.txt 2>&1
