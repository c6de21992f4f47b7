set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
WAM_LIB_PATH=$R/build/exp/c16b.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dwt.py -k "sigma" > gpurun_out/r05z_pytest.log 2>&1 || { tail -30 gpurun_out/r05z_pytest.log; exit 1; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dwt.py -k "sigma" >> gpurun_out/r05z_pytest.log 2>&1 || { tail -30 gpurun_out/r05z_pytest.log; exit 1; }
tail -1 gpurun_out/r05z_pytest.log
for r in 1 2; do
for v in base c16 c16b; do
  echo "== $v" | tee -a gpurun_out/r05z_sigma.log
  WAM_LIB_PATH=$R/build/exp/$v.so timeout -k 10 120 python -u scripts/kbench_sigma.py --iters 20 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05z_sigma.log || exit 1
done
done
