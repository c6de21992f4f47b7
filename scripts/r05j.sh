set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dwt.py -k "item_sigma" > gpurun_out/r05j_pytest.log 2>&1 || { tail -30 gpurun_out/r05j_pytest.log; exit 1; }
tail -1 gpurun_out/r05j_pytest.log
timeout -k 10 200 python -u scripts/kbench_sigma.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05j_sigma_cold.log
timeout -k 10 200 python -u scripts/kbench_sigma.py --single-block 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05j_sigma_cold.log
