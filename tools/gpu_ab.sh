set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_concurrency.py tests/test_interop_rebuild.py > gpurun_out/ab/tests.log 2>&1
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --cpu-seconds 0 --no-host-path > gpurun_out/ab/bench.json 2>gpurun_out/ab/bench.err
timeout -k 10 200 python -u tools/profile_phases.py > gpurun_out/ab/phases.txt 2>&1
