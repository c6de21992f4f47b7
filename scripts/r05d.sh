set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dwt.py -k "line_stream or noisy_wavedec_equals or plane_coop or plane_resident" > gpurun_out/r05d_pytest.log 2>&1 || { tail -30 gpurun_out/r05d_pytest.log; exit 1; }
tail -2 gpurun_out/r05d_pytest.log
for r in 1 2; do
for v in cur pair0; do
  if [ $v = cur ]; then L=""; else L=build/exp/$v.so; fi
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/ab_line.py --iters 20 --samples 25 --flags 0 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05d_ab_pair.log || exit 1
done
done
