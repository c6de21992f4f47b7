set -o pipefail
mkdir -p gpurun_out
for v in cur nx2 w5 nx2w5; do
  if [ $v = cur ]; then L=""; F="0,32"; else L=build/exp/$v.so; F="0"; fi
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/ab_line.py --iters 20 --samples 25,21,17 --flags $F 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05b_ab_line.log || exit 1
done
