set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for v in cur t4k t2k; do
  if [ $v = cur ]; then L=""; else L=$R/build/exp/$v.so; fi
  echo "== $v" | tee -a gpurun_out/r05s_kbench_c4.log
  WAM_LIB_PATH=$L timeout -k 10 150 python -u scripts/kbench_c4.py --iters 3 2>&1 | grep -v amdgpu.ids | grep -B1 -A5 "adjoint\|wavedec" | tee -a gpurun_out/r05s_kbench_c4.log || exit 1
done
done
for v in cur t4k t2k; do
  if [ $v = cur ]; then L=""; else L=$R/build/exp/$v.so; fi
  WAM_LIB_PATH=$L OUT=r05s_pmc4_$v KREGEX="k_ana_rows|k_adj_maps" PROBE=pmc_probe_c4.py bash scripts/pmc_traffic.sh > gpurun_out/r05s_pmc4_$v.log 2>&1 || { tail gpurun_out/r05s_pmc4_$v.log; exit 1; }
done
echo done
