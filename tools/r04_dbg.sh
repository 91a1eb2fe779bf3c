# bench line with the workload batches warmed (kernel variant chosen and loaded before timing)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_wl; mkdir -p $o
timeout -k 10 300 python -u bench.py > $o/bench.json 2> $o/bench.err || exit $?
python - <<'P'
import json
b=json.loads(open("gpurun_out/r04_wl/bench.json").read().strip().splitlines()[-1])
print("value", b["value"], "enc", b["enc_kernel_us"], "dec", b["dec_kernel_us"], "hash", b["xxh32_headers"]["kernel_us"])
w=b["workloads"]
for n in ("qif_corpus","base64","alphabet_c"):
    print(n, w[n]["enc_kernel_us"], w[n]["dec_kernel_us"], w[n]["enc_dec_gbps"], w[n]["vs_synthetic_token"], w[n]["roundtrip_ok"])
P
