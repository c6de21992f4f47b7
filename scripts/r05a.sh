set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dwt.py -k "line_stream or noisy_wavedec_equals or plane_coop or plane_resident or item_sigma" > gpurun_out/r05a_pytest.log 2>&1 || { tail -40 gpurun_out/r05a_pytest.log; exit 1; }
tail -3 gpurun_out/r05a_pytest.log
for f in 0 32 0 32; do timeout -k 10 120 python -u scripts/kbench_levels.py --iters 20 --levels 3 --flags $f 2>&1 | grep -v copy | sed "s/^/f$f /" | tee -a gpurun_out/r05a_kbench.log || exit 1; done
