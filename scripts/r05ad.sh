set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ad_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05ad_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05ad_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05ad_smoke.log 2>&1 || { tail -20 gpurun_out/r05ad_smoke.log; exit 1; }
tail -1 gpurun_out/r05ad_smoke.log
timeout -k 10 600 python -u bench.py --config c2 > gpurun_out/r05ad_bench_c2.log 2>&1 || { tail -20 gpurun_out/r05ad_bench_c2.log; exit 1; }
tail -1 gpurun_out/r05ad_bench_c2.log | cut -c1-300
