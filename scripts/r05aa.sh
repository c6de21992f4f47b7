set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dwt.py tests/test_gpu_00_configs.py -k "noisy or plane or philox or fused_2d or wavedec or c2 or c1" > gpurun_out/r05aa_pytest.log 2>&1 || { tail -30 gpurun_out/r05aa_pytest.log; exit 1; }
tail -1 gpurun_out/r05aa_pytest.log
for r in 1 2 3; do
for v in cur nopair; do
  if [ $v = cur ]; then L=""; else L=$R/build/exp/$v.so; fi
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/ab_line.py --iters 20 --samples 25 --flags 0 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05aa_ab_paircol.log || exit 1
done
done
OUT=r05aa_pmc KREGEX="k_plane_ana" bash scripts/pmc_traffic.sh > gpurun_out/r05aa_pmc.log 2>&1 || { tail gpurun_out/r05aa_pmc.log; exit 1; }
tail -12 gpurun_out/r05aa_pmc.log
