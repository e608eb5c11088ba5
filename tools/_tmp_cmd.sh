set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_seeds.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_seeds.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_seeds.log
exit $rc
