set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for v in cur at32; do
  if [ $v = cur ]; then L=""; else L=build/exp/$v.so; fi
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/kbench_levels.py --iters 20 --levels 3 2>&1 | grep -v "amdgpu.ids\|copy" | sed "s/^/$v /" | tee -a gpurun_out/r05h_ab_at32.log || exit 1
done
done
