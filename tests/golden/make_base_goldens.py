"""BaseWAM2D goldens (round 2): the REFERENCE's own ``lib/wam_2D.py`` BaseWAM2D single pass and
its ``.scales`` side attribute (``disentangle_scales``, lib/wam_2D.py:133-198, including the stale
``img_batch`` quirk of the approximation row), run here with the stand-ins of
make_glue_goldens.py (ptwt := oracle.ptwt_torch, cv2.resize := F.interpolate bilinear).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_base_goldens.py

Writes tests/golden/base_goldens.npz (outputs only; inputs regenerated from RandomState).
"""
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.golden.make_glue_goldens import import_reference, install_standins  # noqa: E402
from tests.golden.glue_cases import BASE_CASES, make_inputs, make_model  # noqa: E402


def main():
    install_standins()
    _, w2, _ = import_reference()
    torch.set_num_threads(min(8, os.cpu_count()))
    out = {}
    for name, case in BASE_CASES.items():
        x, y = make_inputs(case)
        ex = w2.BaseWAM2D(make_model(case), **case["kw"])
        out[name] = ex(x, y)
        out[name + "_scales"] = ex.scales
        print(name, out[name].shape, out[name + "_scales"].shape)
    np.savez_compressed(os.path.join(HERE, "base_goldens.npz"), **out)


if __name__ == "__main__":
    main()
