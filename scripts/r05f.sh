set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dwt.py -k "item_sigma" > gpurun_out/r05f_pytest.log 2>&1 || { tail -30 gpurun_out/r05f_pytest.log; exit 1; }
tail -1 gpurun_out/r05f_pytest.log
true
timeout -k 10 200 python -u - <<'PY' 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r05f_sigma.log
import torch, wam_amd
from wam_amd import plan as P
from scripts.kbench_levels import timed
for items, n in ((64, 3*224*224), (256, 80000), (16, 128**3), (1, 3*224*224)):
    x = torch.randn(items * n, device="cuda")
    r = timed(lambda: P.item_sigma(x, n, n, 0.25), 20)
    for name, (us, nb) in r.items():
        print(f"sigma items={items} len={n} {name} {us:.1f} us {nb/us/1e3:.0f} GB/s", flush=True)
PY
