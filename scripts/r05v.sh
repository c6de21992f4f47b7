set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --config c3 > gpurun_out/r05v_bench_c3.log 2>&1 || { tail -20 gpurun_out/r05v_bench_c3.log; exit 1; }
tail -1 gpurun_out/r05v_bench_c3.log | cut -c1-200
timeout -k 10 600 python -u bench.py --config c5 > gpurun_out/r05v_bench_c5.log 2>&1 || { tail -20 gpurun_out/r05v_bench_c5.log; exit 1; }
tail -1 gpurun_out/r05v_bench_c5.log | cut -c1-200
timeout -k 10 300 python -u bench.py --config c1 > gpurun_out/r05v_bench_c1.log 2>&1 || { tail -20 gpurun_out/r05v_bench_c1.log; exit 1; }
tail -1 gpurun_out/r05v_bench_c1.log | cut -c1-200
timeout -k 10 600 python -u bench.py --config c2 --gpus 2 --dist-backend gloo --single-device --steps 3 --warmup 1 --cpu-baseline off --extras off > gpurun_out/r05v_bench_c2_n2_gloo.log 2>&1 || { tail -20 gpurun_out/r05v_bench_c2_n2_gloo.log; exit 1; }
tail -1 gpurun_out/r05v_bench_c2_n2_gloo.log | cut -c1-200
