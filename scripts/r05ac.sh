set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --config c2 --extras off --cpu-baseline off --pmc off > gpurun_out/r05ac_bench_c2_quick.log 2>&1 || { tail -20 gpurun_out/r05ac_bench_c2_quick.log; exit 1; }
tail -1 gpurun_out/r05ac_bench_c2_quick.log | cut -c1-260
hostname
