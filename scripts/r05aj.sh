set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --config c2 --extras off --cpu-baseline off --pmc off > gpurun_out/r05aj_$r.log 2>&1 || { tail -5 gpurun_out/r05aj_$r.log; exit 1; }
  grep '^{"metric"' gpurun_out/r05aj_$r.log | cut -c100-200 | tee -a gpurun_out/r05aj_shipped_db.log
done
timeout -k 10 900 python -u bench.py --config c2 > gpurun_out/r05aj_full.log 2>&1 || { tail -5 gpurun_out/r05aj_full.log; exit 1; }
grep '^{"metric"' gpurun_out/r05aj_full.log | cut -c100-200 | tee -a gpurun_out/r05aj_shipped_db.log
