set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/check_pow2_seed.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05ae_pow2_seed.log
