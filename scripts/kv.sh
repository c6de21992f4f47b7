set -o pipefail
mkdir -p gpurun_out/kv
timeout -k 10 200 python -u -m pytest tests/test_gpu_dwt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/kv/pytest.log 2>&1 || { tail -20 gpurun_out/kv/pytest.log; exit 1; }
tail -2 gpurun_out/kv/pytest.log
for v in v0 v1 v2 v3; do
  echo "== $v"; WAM_LIB_PATH=build/exp/$v.so KBENCH_PLANE_ONLY=1 timeout -k 10 120 python scripts/kbench.py --iters 20 > gpurun_out/kv/$v.log 2>&1 || exit 1
  grep -A1 "noisy S=25\|plane wavedec:" gpurun_out/kv/$v.log
done
