set -o pipefail
mkdir -p gpurun_out
for v in cur nonoise nopush row0 nosched; do
  if [ $v = cur ]; then L=""; F="32,0"; else L=build/exp/$v.so; F="32"; fi
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/ab_line.py --iters 20 --samples 25,21 --flags $F 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05c_ab_line.log || exit 1
done
