# plane-kernel parity subset (bit-exact and pywt-pinned tests of the plane / per-level / noisy paths)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dwt.py > gpurun_out/tplane.log 2>&1 || { tail -40 gpurun_out/tplane.log; exit 1; }
tail -2 gpurun_out/tplane.log
