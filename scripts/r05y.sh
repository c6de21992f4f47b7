set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dwt.py -k "noisy_wavedec_equals or philox" > gpurun_out/r05y_pytest.log 2>&1 || { tail -30 gpurun_out/r05y_pytest.log; exit 1; }
WAM_LIB_PATH=$R/build/exp/hl.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dwt.py -k "noisy_wavedec_equals or philox" >> gpurun_out/r05y_pytest.log 2>&1 || { tail -30 gpurun_out/r05y_pytest.log; exit 1; }
tail -1 gpurun_out/r05y_pytest.log
for r in 1 2; do
for v in cur hl; do
  if [ $v = cur ]; then L=""; else L=$R/build/exp/$v.so; fi
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/ab_line.py --iters 20 --samples 25 --flags 0 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05y_ab_philox_mulhl.log || exit 1
done
for v in cur pf3 pf6 pf8; do
  if [ $v = cur ]; then L=""; else L=$R/build/exp/$v.so; fi
  echo "== $v" | tee -a gpurun_out/r05y_kbench_syn_pf.log
  KBENCH_PLANE_ONLY=1 WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/kbench.py --iters 10 2>&1 | grep -v amdgpu.ids | grep -A1 "waverec" | tee -a gpurun_out/r05y_kbench_syn_pf.log || exit 1
done
done
