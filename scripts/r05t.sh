set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dwt.py tests/test_gpu_00_configs.py -k "rows or adj or wavedec or c4 or ig" > gpurun_out/r05t_pytest.log 2>&1 || { tail -30 gpurun_out/r05t_pytest.log; exit 1; }
tail -1 gpurun_out/r05t_pytest.log
timeout -k 10 600 python -u bench.py --config c4 > gpurun_out/r05t_bench_c4.log 2>&1 || { tail -20 gpurun_out/r05t_bench_c4.log; exit 1; }
tail -1 gpurun_out/r05t_bench_c4.log | cut -c1-300
timeout -k 10 600 python -u bench.py --config c2 > gpurun_out/r05t_bench_c2.log 2>&1 || { tail -20 gpurun_out/r05t_bench_c2.log; exit 1; }
tail -1 gpurun_out/r05t_bench_c2.log | cut -c1-300
timeout -k 10 600 bash scripts/trace_config.sh c2 3 400 > gpurun_out/r05t_trace_c2.log 2>&1 || { tail -20 gpurun_out/r05t_trace_c2.log; exit 1; }
cat gpurun_out/trace_c2/window.txt | head -30
