# A/B timing of plane-analysis variants on one box: libwam_hip.so builds under build/exp/<name>.so
# (scripts/build_variants.py) and plan flags, J=3 c2 group shape (scripts/kbench_levels.py)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for v in ${VARIANTS:-cur}; do
  if [ $v = cur ]; then L=""; else L=build/exp/$v.so; fi
  for f in ${FLAGS:-0}; do
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/kbench_levels.py --iters 20 --levels ${LEVELS:-3} --flags $f 2>/dev/null | grep -v copy | sed "s/^/$v f$f /" || exit 1
  done
done
done
