set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dwt.py -k "noisy_wavedec_equals or plane_coop or plane_resident or line_stream or philox" > gpurun_out/r05l_pytest.log 2>&1 || { tail -30 gpurun_out/r05l_pytest.log; exit 1; }
tail -1 gpurun_out/r05l_pytest.log
for r in 1 2; do
for v in cur base; do
  if [ $v = cur ]; then L=""; else L=build/exp/$v.so; fi
  echo "== $v" | tee -a gpurun_out/r05l_ab.log
  WAM_LIB_PATH=$L timeout -k 10 120 python -u scripts/ab_line.py --iters 20 --samples 25 --flags 0 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r05l_ab.log || exit 1
done
done
