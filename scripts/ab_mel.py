"""A/B of the mel kernels, one library per process (WAM_LIB_PATH=build/exp/<variant>.so for the
other arm). usage: python scripts/ab_mel.py <out.npz>  -> saves forwards and adjoints of several
shapes (compare with scripts/ab_mel_cmp.py) and prints the c3-group times."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from wam_amd import melspec as M  # noqa: E402

CASES = [(1024, 80000, 128, 16000, 3), (1024, 8000, 128, 44100, 2), (256, 1001, 40, 8000, 2), (64, 33, 8, 16000, 2),
         (2048, 4096, 128, 44100, 2), (2048, 10000, 256, 44100, 2), (512, 300, 64, 22050, 2), (128, 1000, 16, 8000, 3),
         (1024, 1023, 128, 16000, 1), (1024, 1025, 128, 16000, 1)]
out = {}
for i, (n, t, m, sr, b) in enumerate(CASES):
    g = torch.Generator().manual_seed(i)
    x = torch.randn(b, t, generator=g).cuda()
    go = torch.randn(b, t // (n // 2) + 1, m, generator=g).cuda()
    out["c%d" % i] = M.mel_adjoint(x, go, n, sr, m).cpu().numpy()
    out["f%d" % i] = M.mel_forward(x, n, sr, m).cpu().numpy()
x = torch.randn(1280, 80000, device="cuda")
go = torch.randn(1280, 157, 128, device="cuda")
tag = os.environ.get("WAM_LIB_PATH", "in-tree libwam_hip.so")
for name, fn in (("mel_forward", lambda: M.mel_forward(x, 1024, 16000, 128)),
                 ("mel_adjoint", lambda: M.mel_adjoint(x, go, 1024, 16000, 128))):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        fn()
    e.record()
    torch.cuda.synchronize()
    print("%s: %s c3 group (1280 x 80000): %.1f us" % (tag, name, 1e3 * s.elapsed_time(e) / 10))
np.savez(sys.argv[1], **out)
