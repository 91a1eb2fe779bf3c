set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_l; mkdir -p $o
for G in 1 2 3; do
  timeout -k 10 300 python bench.py --config4 --gpus $G --steps 10 --warmup 3 > $o/config4_g$G.json 2> $o/config4_g$G.err || { tail -20 $o/config4_g$G.err; exit 1; }
  python -c "import json;d=json.loads(open('$o/config4_g$G.json').read().strip().splitlines()[-1]);print($G, d['value'], d['ms_per_step'], d['stitched_equals_single_pass'], d['roundtrip_ok'], d['config']['shard_strings'])"
done
