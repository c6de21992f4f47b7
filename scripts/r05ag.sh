set -o pipefail
mkdir -p gpurun_out/r05ag
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2 3 4; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05ag_$r -o run -- python3 $R/bench.py --config c2 --extras off --cpu-baseline off --pmc off > $R/gpurun_out/r05ag/bench_$r.log 2>&1 || { tail -5 $R/gpurun_out/r05ag/bench_$r.log; exit 1; }
  KS=$(find /tmp/r05ag_$r -name "*kernel_stats.csv" | head -1)
  cp "$KS" $R/gpurun_out/r05ag/kernel_stats_$r.csv
  rm -rf /tmp/r05ag_$r
  grep -v amdgpu.ids $R/gpurun_out/r05ag/bench_$r.log | tail -1 | cut -c150-260
done
