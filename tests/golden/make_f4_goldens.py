"""f4 goldens: the REFERENCE's own ``WaveletAttribution3D.visualize`` (lib/wam_3D.py:662-719) on
given |grad| cubes, run here with the stand-ins of make_glue_goldens.py (ptwt := oracle.ptwt_torch;
visualize itself only uses numpy and the real scipy.ndimage.zoom).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_f4_goldens.py

Writes tests/golden/f4_goldens.npz (outputs only; cubes regenerated from RandomState).
"""
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.golden.make_glue_goldens import import_reference, install_standins  # noqa: E402

VIS_CASES = {"vis_s32_j2": (2, 32, 2, 401), "vis_s16_j1": (3, 16, 1, 402), "vis_s64_j3": (1, 64, 3, 403)}


def cube(n, S, seed):
    return np.abs(np.random.RandomState(seed).standard_normal((n, S, S, S))).astype(np.float32)


def main():
    install_standins()
    _, _, w3 = import_reference()
    import testmodels
    out = {}
    for name, (n, S, J, seed) in VIS_CASES.items():
        ex = w3.WaveletAttribution3D(testmodels.TinyVoxel(), wavelet="haar", J=J)
        ex.grads = cube(n, S, seed)
        ex.input_size = S
        out[name] = ex.visualize()
        print(name, out[name].shape, out[name].dtype)
    np.savez_compressed(os.path.join(HERE, "f4_goldens.npz"), **out)


if __name__ == "__main__":
    main()
