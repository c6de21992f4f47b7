set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./build/ubench_rng > gpurun_out/r05m_ubench_rng.log 2>&1 || { tail gpurun_out/r05m_ubench_rng.log; exit 1; }
cat gpurun_out/r05m_ubench_rng.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_frames.py tests/test_gpu_dwt.py tests/test_gpu_00_configs.py -k "frames or trapz or coef_order or waverec or synthesis or alpha or rows or adj or wavedec" > gpurun_out/r05m_pytest.log 2>&1 || { tail -30 gpurun_out/r05m_pytest.log; exit 1; }
tail -1 gpurun_out/r05m_pytest.log
for r in 1 2; do
for v in cur base; do
  if [ $v = cur ]; then L=""; else L=build/exp/$v.so; fi
  echo "== $v" | tee -a gpurun_out/r05m_kbench.log
  KBENCH_PLANE_ONLY=1 WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/kbench.py --iters 10 2>&1 | grep -v amdgpu.ids | grep -A3 "waverec" | tee -a gpurun_out/r05m_kbench.log || exit 1
  WAM_LIB_PATH=$L timeout -k 10 150 python -u scripts/kbench_c4.py --iters 3 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05m_kbench_c4.log || exit 1
done
done
OUT=r05m_pmc_cur KREGEX=k_plane_syn bash scripts/pmc_traffic.sh > gpurun_out/r05m_pmc_cur.log 2>&1 || { tail gpurun_out/r05m_pmc_cur.log; exit 1; }
WAM_LIB_PATH=build/exp/base.so OUT=r05m_pmc_base KREGEX=k_plane_syn bash scripts/pmc_traffic.sh > gpurun_out/r05m_pmc_base.log 2>&1 || { tail gpurun_out/r05m_pmc_base.log; exit 1; }
for v in cur base; do
  if [ $v = cur ]; then L=""; else L=build/exp/$v.so; fi
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/pmc_probe_frames.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05m_frames_time.log || exit 1
  WAM_LIB_PATH=$L OUT=r05m_pmcf_$v KREGEX=k_frame PROBE=pmc_probe_frames.py bash scripts/pmc_traffic.sh > gpurun_out/r05m_pmcf_$v.log 2>&1 || { tail gpurun_out/r05m_pmcf_$v.log; exit 1; }
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/pmc_probe_c4.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05m_c4probe_time.log || exit 1
  WAM_LIB_PATH=$L OUT=r05m_pmc4_$v KREGEX="k_ana_rows|k_adj_maps|k_dwt2_syn" PROBE=pmc_probe_c4.py bash scripts/pmc_traffic.sh > gpurun_out/r05m_pmc4_$v.log 2>&1 || { tail gpurun_out/r05m_pmc4_$v.log; exit 1; }
done
tail -3 gpurun_out/r05m_pmc_cur.log gpurun_out/r05m_pmc_base.log gpurun_out/r05m_pmcf_cur.log gpurun_out/r05m_pmcf_base.log gpurun_out/r05m_pmc4_cur.log gpurun_out/r05m_pmc4_base.log
