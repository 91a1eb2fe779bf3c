#!/bin/bash
# GPU diagnostics: GPU parity tests on the default library, then one short
# bench line per library variant (QHUFF_LIB).  Build everything here first
# (make -C ls-qpack_amd; variants with OUT=... OBJDIR=... ENC_WAVES=...).
# Usage (on the GPU box): tools/diag.sh [lib.so ...]; writes gpurun_out/diag/.
# Stops at the first step that times out, aborts or faults; a failing test
# (exit 1) does not stop the benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
o=gpurun_out/diag
mkdir -p $o
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
if [ -z "$SKIP_TESTS" ]; then
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 \
        --timeout-method thread > $o/pytest.log 2>&1
    rc=$?
    tail -5 $o/pytest.log
    fatal $rc && { echo "pytest fatal rc=$rc"; exit $rc; }
fi
libs=("$@")
[ ${#libs[@]} -eq 0 ] && libs=(ls-qpack_amd/libqhuff.so)
for lib in "${libs[@]}"; do
    tag=$(basename "$lib" .so)
    QHUFF_LIB=$PWD/$lib timeout -k 10 180 python -u bench.py --steps 30 \
        --warmup 5 --cpu-seconds 0 --no-host-path > $o/bench_$tag.json 2> $o/bench_$tag.err
    rc=$?
    echo "$tag rc=$rc: $(cat $o/bench_$tag.json)"
    fatal $rc && exit $rc
done
echo diag-done
