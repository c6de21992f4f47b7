set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_frames.py tests/test_gpu_dist.py > gpurun_out/r05w_pytest.log 2>&1 || { tail -30 gpurun_out/r05w_pytest.log; exit 1; }
tail -1 gpurun_out/r05w_pytest.log
timeout -k 10 600 python -u bench.py --config c2 > gpurun_out/r05w_bench_c2.log 2>&1 || { tail -20 gpurun_out/r05w_bench_c2.log; exit 1; }
tail -1 gpurun_out/r05w_bench_c2.log | cut -c1-300
