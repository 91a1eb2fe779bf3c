#!/bin/bash
# the bench line's xxh32_headers leg on library variants, interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/${TAG:-hash_ab}; mkdir -p $o
for rep in 1 2 3; do
for L in "$@"; do
  QHUFF_LIB=$PWD/ls-qpack_amd/$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-host-path --no-workloads --no-overlap > $o/b_${L}_$rep.json 2> $o/b_$L.err || exit 1
  python -c "import json;d=json.loads(open('$o/b_${L}_$rep.json').read().strip().splitlines()[-1]);h=d['xxh32_headers'];print('$L', h['kernel_us'], h['roofline_frac'], d['value'])"
done
done
