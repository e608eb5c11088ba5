set -u
mkdir -p gpurun_out/prof_seeds2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_seeds.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_seeds.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_seeds.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_seeds2/trace -o run -- python3 tools/seeds_probe.py --repeat 2 > gpurun_out/prof_seeds2/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 gpurun_out/prof_seeds2/trace.log; exit $rc
