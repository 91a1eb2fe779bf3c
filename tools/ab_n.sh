# bench lines for N library builds, interleaved (3 rounds of L1 L2 ... LN):
# tools/ab_n.sh OUTDIR LIB...
set -e
cd $GRAFT_REPO_ROOT
out=$1; shift
mkdir -p $out
for i in 1 2 3; do
  for lib in "$@"; do
    name=$(basename $lib .so)
    QHUFF_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --cpu-seconds 0 --no-host-path > $out/$name.$i.json 2>/dev/null
  done
done
python - "$out" <<'PY'
import glob, json, os, sys, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f))
    r[os.path.basename(f).rsplit(".", 2)[0]].append((d["value"], d["enc_kernel_us"], d["dec_kernel_us"]))
for k, v in r.items():
    n = len(v)
    print("%-22s GB/s %7.1f  enc %6.2f  dec %6.2f   (%s)" % (k, sum(x[0] for x in v) / n, sum(x[1] for x in v) / n, sum(x[2] for x in v) / n,
          " ".join("%.1f/%.1f" % (x[1], x[2]) for x in v)))
PY
