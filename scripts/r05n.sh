set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for v in cur base; do
  if [ $v = cur ]; then L=""; else L=$R/build/exp/$v.so; fi
  echo "== $v" | tee -a gpurun_out/r05n_frames_time.log
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/pmc_probe_frames.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05n_frames_time.log || exit 1
  WAM_LIB_PATH=$L OUT=r05n_pmcf_$v KREGEX=k_frame PROBE=pmc_probe_frames.py bash scripts/pmc_traffic.sh > gpurun_out/r05n_pmcf_$v.log 2>&1 || { tail gpurun_out/r05n_pmcf_$v.log; exit 1; }
  echo "== $v" | tee -a gpurun_out/r05n_c4probe_time.log
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/pmc_probe_c4.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05n_c4probe_time.log || exit 1
  WAM_LIB_PATH=$L OUT=r05n_pmc4_$v KREGEX="k_ana_rows|k_adj_maps|k_dwt2_syn" PROBE=pmc_probe_c4.py bash scripts/pmc_traffic.sh > gpurun_out/r05n_pmc4_$v.log 2>&1 || { tail gpurun_out/r05n_pmc4_$v.log; exit 1; }
done
WAM_LIB_PATH=$R/build/exp/base.so OUT=r05n_pmc_syn_base KREGEX=k_plane_syn bash scripts/pmc_traffic.sh > gpurun_out/r05n_pmc_syn_base.log 2>&1 || { tail gpurun_out/r05n_pmc_syn_base.log; exit 1; }
echo done
