set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_seeds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_seeds.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_seeds.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/seeds_probe.py --repeat 1 > gpurun_out/seeds_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -1 gpurun_out/seeds_probe.log; exit $rc
