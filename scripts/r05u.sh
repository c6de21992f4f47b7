set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for v in cur a2 a4 a8; do
  if [ $v = cur ]; then L=""; else L=$R/build/exp/$v.so; fi
  echo "== $v" | tee -a gpurun_out/r05u_frames_time.log
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/pmc_probe_frames.py 2>&1 | grep -v amdgpu.ids | grep accumulate | tee -a gpurun_out/r05u_frames_time.log || exit 1
  WAM_LIB_PATH=$L OUT=r05u_pmcf_$v KREGEX=k_frame_accumulate PROBE=pmc_probe_frames.py bash scripts/pmc_traffic.sh > gpurun_out/r05u_pmcf_$v.log 2>&1 || { tail gpurun_out/r05u_pmcf_$v.log; exit 1; }
done
for v in cur a2 a4 a8; do
  if [ $v = cur ]; then L=""; else L=$R/build/exp/$v.so; fi
  echo "== $v" | tee -a gpurun_out/r05u_frames_time.log
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/pmc_probe_frames.py 2>&1 | grep -v amdgpu.ids | grep accumulate | tee -a gpurun_out/r05u_frames_time.log || exit 1
done
echo done
