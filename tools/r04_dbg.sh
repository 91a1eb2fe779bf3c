# adaptive kernel choice counted on launches seen to run: parity + bench workloads leg
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r04_w; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_lsqpack_shim.py tests/test_concurrency.py tests/test_service.py -m gpu -q -x --timeout 120 --timeout-method thread > $o/pytest.log 2>&1
rc=$?; tail -1 $o/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --cpu-seconds 0 --no-host-path --no-overlap > $o/bench.json 2> $o/bench.err || exit $?
python - <<'P'
import json
b=json.loads(open("gpurun_out/r04_w/bench.json").read().strip().splitlines()[-1])
print(b["value"], b["roofline"]["kernel_us"], b.get("enc_kernel_us"), b.get("dec_kernel_us"))
w=b["workloads"]
for n in ("qif_corpus","base64","alphabet_c"):
    print(n, w[n]["enc_kernel_us"], w[n]["dec_kernel_us"], w[n]["vs_synthetic_token"], w[n]["roundtrip_ok"])
P
