set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_frames.py > gpurun_out/r05p_pytest.log 2>&1 || { tail -30 gpurun_out/r05p_pytest.log; exit 1; }
tail -1 gpurun_out/r05p_pytest.log
OUT=r05p_sq PROBE=pmc_probe_c4.py KREGEX="k_dwt2_syn|k_adj_maps" bash scripts/pmc_probe.sh > gpurun_out/r05p_sq.log 2>&1 || { tail gpurun_out/r05p_sq.log; exit 1; }
python3 scripts/pmc_sq.py gpurun_out/r05p_sq > gpurun_out/r05p_sq_summary.log && cat gpurun_out/r05p_sq_summary.log
