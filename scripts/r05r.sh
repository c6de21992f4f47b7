set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05r_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05r_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05r_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05r_smoke.log 2>&1 || { tail -20 gpurun_out/r05r_smoke.log; exit 1; }
tail -1 gpurun_out/r05r_smoke.log
timeout -k 10 600 python -u bench.py --config c4 > gpurun_out/r05r_bench_c4.log 2>&1 || { tail -20 gpurun_out/r05r_bench_c4.log; exit 1; }
tail -1 gpurun_out/r05r_bench_c4.log | cut -c1-400
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for v in cur pf3; do
  if [ $v = cur ]; then L=""; else L=$R/build/exp/$v.so; fi
  echo "== $v" | tee -a gpurun_out/r05r_kbench_c4_pf3.log
  WAM_LIB_PATH=$L timeout -k 10 150 python -u scripts/kbench_c4.py --iters 3 2>&1 | grep -v amdgpu.ids | grep -A6 "waverec" | tee -a gpurun_out/r05r_kbench_c4_pf3.log || exit 1
done
done
