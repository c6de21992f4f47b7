set -o pipefail
mkdir -p gpurun_out/miopen_db
D=$GRAFT_REPO_ROOT/gpurun_out/miopen_db
MIOPEN_USER_DB_PATH=$D timeout -k 10 500 python -u bench.py --config c2 --extras off --cpu-baseline off --pmc off > gpurun_out/r05ai_gen.log 2>&1 || { tail -5 gpurun_out/r05ai_gen.log; exit 1; }
grep '^{"metric"' gpurun_out/r05ai_gen.log | cut -c100-200
ls -la $D
for r in 1 2; do
  MIOPEN_USER_DB_PATH=$D timeout -k 10 400 python -u bench.py --config c2 --extras off --cpu-baseline off --pmc off > gpurun_out/r05ai_reuse_$r.log 2>&1 || { tail -5 gpurun_out/r05ai_reuse_$r.log; exit 1; }
  grep '^{"metric"' gpurun_out/r05ai_reuse_$r.log | cut -c100-200
done
