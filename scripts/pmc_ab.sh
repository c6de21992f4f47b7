# FETCH_SIZE / WRITE_SIZE passes of a probe script for the in-tree library and build/exp variants
# usage: VARIANTS="cur old" KREGEX=k_dwt2_syn PROBE=pmc_probe_c4.py bash scripts/pmc_ab.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
for v in ${VARIANTS:-cur}; do
  if [ $v = cur ]; then L=""; else L=$R/build/exp/$v.so; fi
  (cd /tmp && WAM_LIB_PATH=$L timeout -k 10 120 python3 $R/scripts/$PROBE 2>/dev/null | sed "s/^/$v /") || exit 1
  WAM_LIB_PATH=$L OUT=pmc_$v KREGEX=$KREGEX PROBE=$PROBE bash $R/scripts/pmc_traffic.sh > /tmp/pmc_$v.txt 2>&1 || { tail /tmp/pmc_$v.txt; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$R/gpurun_out/pmc_$v/traffic.json')); [print('$v', k, v) for k, v in d['per_call'].items()]"
done
