"""Glue goldens: run the REFERENCE's own ``lib/wam_{1,2,3}D.py`` here and store its outputs.

Run in this container only (``/root/reference`` does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_glue_goldens.py

The reference imports packages that are absent offline; stand-ins are installed in
``sys.modules`` before importing it:

* ``ptwt``      := ``oracle.ptwt_torch`` (the ptwt algorithm restated on torch-CPU, itself pinned
                   to PyWavelets 1.1.1 by ``tests/golden/pywt_dwt.npz``);
* ``cv2``       := ``resize`` via ``F.interpolate(bilinear, align_corners=False)`` (half-pixel
                   centres, edge clamp = cv2 INTER_LINEAR for upsampling; only ``.scales`` uses it);
* ``torchaudio.transforms`` := ``oracle.melspec`` (torchaudio's documented defaults; unpinned);
* ``pywt``, ``librosa`` := empty modules (imported at module level by ``lib/wam_1D.py`` but only
                   used by its visualisation helpers, which are not on the path).

So these goldens pin the reference GLUE (noise stream, per-sample loop, channel mean, batch-global
normalisation, mosaic layout, trapezoid, loss scaling, 3D cube/averaging) -- not ptwt or cv2.
Only outputs and the tiny seeds/configs are stored; inputs are regenerated from RandomState.
"""
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import melspec, ptwt_torch  # noqa: E402
import testmodels  # noqa: E402
from tests.golden.glue_cases import CASES, make_inputs, make_model  # noqa: E402


def install_standins():
    sys.modules["ptwt"] = ptwt_torch.as_module()
    cv2 = types.ModuleType("cv2")
    cv2.INTER_LINEAR = 1

    def resize(a, dsize, interpolation=1):
        t = torch.as_tensor(np.ascontiguousarray(a))[None, None]
        out = F.interpolate(t, size=(dsize[1], dsize[0]), mode="bilinear", align_corners=False)
        return out[0, 0].numpy()

    cv2.resize = resize
    sys.modules["cv2"] = cv2
    ta = types.ModuleType("torchaudio")
    tat = types.ModuleType("torchaudio.transforms")
    tat.MelSpectrogram = melspec.MelSpectrogram
    tat.AmplitudeToDB = melspec.AmplitudeToDB
    ta.transforms = tat
    sys.modules["torchaudio"] = ta
    sys.modules["torchaudio.transforms"] = tat
    sys.modules["pywt"] = types.ModuleType("pywt")
    sys.modules["librosa"] = types.ModuleType("librosa")


def import_reference():
    sys.path.insert(0, "/root/reference")
    import lib.wam_1D as w1  # noqa
    import lib.wam_2D as w2  # noqa
    import lib.wam_3D as w3  # noqa
    return w1, w2, w3


def main():
    install_standins()
    w1, w2, w3 = import_reference()
    torch.set_num_threads(min(8, os.cpu_count()))
    out = {}
    for name, case in CASES.items():
        x, y = make_inputs(case)
        model = make_model(case)
        kw = dict(case["kw"])
        if case["dim"] == 2:
            ex = w2.WaveletAttribution2D(model, **kw)
            res = ex(x, y)
            out[name] = res
            if case.get("scales"):
                out[name + "_scales"] = ex.scales.astype(np.float32)
        elif case["dim"] == 1:
            ex = w1.WaveletAttribution1D(model, **kw)
            mel, coeffs = ex(x, y)
            out[name + "_mel"] = mel
            for j, c in enumerate(coeffs):
                out[name + "_c%d" % j] = c
        else:
            ex = w3.WaveletAttribution3D(model, **kw)
            out[name] = ex(x, y)
        print(name, "ok")
    np.savez_compressed(os.path.join(HERE, "glue_goldens.npz"), **out)
    with open(os.path.join(HERE, "glue_goldens.json"), "w") as f:
        json.dump({"torch": torch.__version__, "numpy": np.__version__,
                   "cases": {k: {kk: vv for kk, vv in v.items()} for k, v in CASES.items()}}, f, indent=1,
                  default=str)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
