set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for v in cur c1big c1all; do
  if [ $v = cur ]; then L=""; else L=$R/build/exp/$v.so; fi
  echo "== $v" | tee -a gpurun_out/r05q_kbench_c4.log
  WAM_LIB_PATH=$L timeout -k 10 150 python -u scripts/kbench_c4.py --iters 3 2>&1 | grep -v amdgpu.ids | grep -A6 "adjoint" | tee -a gpurun_out/r05q_kbench_c4.log || exit 1
done
done
