set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_loopback.py -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_verify.json 2> gpurun_out/bench_verify.err; rc=$?; cat gpurun_out/bench_verify.json; tail -3 gpurun_out/bench_verify.err; exit $rc
