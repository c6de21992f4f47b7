set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
for mode in default fast; do
  D=/tmp/mdb_${mode}_$r; rm -rf $D; mkdir -p $D
  if [ $mode = fast ]; then FM=FAST; else FM=""; fi
  MIOPEN_USER_DB_PATH=$D MIOPEN_CUSTOM_CACHE_DIR=$D MIOPEN_FIND_MODE=$FM timeout -k 10 400 python -u bench.py --config c2 --extras off --cpu-baseline off --pmc off > gpurun_out/r05ah_${mode}_$r.log 2>&1 || { tail -5 gpurun_out/r05ah_${mode}_$r.log; exit 1; }
  grep '^{"metric"' gpurun_out/r05ah_${mode}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode', $r, d['value'], d['ms_per_step'])" | tee -a gpurun_out/r05ah_find_mode.log
done
done
