# A/B timing of 1D tile-kernel variants (build/exp/<name>.so) at the c3 shape
set -o pipefail
for r in 1 2; do
for v in ${VARIANTS:-cur}; do
  if [ $v = cur ]; then L=""; else L=build/exp/$v.so; fi
  WAM_LIB_PATH=$L timeout -k 10 180 python -u scripts/kbench_nd.py --iters 5 --only c3 2>/dev/null | sed "s/^/$v /" || exit 1
done
done
