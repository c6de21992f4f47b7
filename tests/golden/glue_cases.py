"""Shared definitions of the glue golden cases (inputs regenerated from numpy RandomState)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import testmodels  # noqa: E402

CASES = {
    # 2D SmoothGrad, haar (the only wavelet whose legacy canvas is 224 at 224), list y
    "s2_haar_list": dict(dim=2, shape=(2, 3, 224, 224), seed=101, y=[3, 7], model="tiny2d", scales=False,
                         kw=dict(wavelet="haar", method="smooth", J=3, mode="reflect", n_samples=3)),
    # int y (loss scale 1/N^2), zero mode, J=2, approx coefficients in .scales
    "s2_haar_int": dict(dim=2, shape=(1, 3, 224, 224), seed=102, y=4, model="tiny2d", scales=True,
                        kw=dict(wavelet="haar", method="smooth", J=2, mode="zero", n_samples=2,
                                approx_coeffs=True)),
    # Integrated gradients, db4, list y
    "ig2_db4_list": dict(dim=2, shape=(2, 3, 224, 224), seed=103, y=[1, 2], model="tiny2d", scales=False,
                         kw=dict(wavelet="db4", method="integratedgrad", J=3, mode="reflect", n_samples=4)),
    # Integrated gradients, sym8, int y, symmetric mode
    "ig2_sym8_int": dict(dim=2, shape=(1, 3, 224, 224), seed=104, y=5, model="tiny2d", scales=False,
                         kw=dict(wavelet="sym8", method="integratedgrad", J=2, mode="symmetric", n_samples=3)),
    # 1D SmoothGrad db6 J=5 (config c3 wavelet), list y
    "s1_db6_list": dict(dim=1, shape=(3, 8000), seed=105, y=[0, 1, 2], model="tinyaudio",
                        kw=dict(wavelet="db6", J=5, method="smooth", mode="reflect", n_samples=3,
                                sample_rate=16000, stdev_spread=0.01)),
    # 1D IG haar J=3, int y
    "ig1_haar_int": dict(dim=1, shape=(2, 4000), seed=106, y=3, model="tinyaudio",
                         kw=dict(wavelet="haar", J=3, method="integratedgrad", mode="reflect", n_samples=3,
                                 sample_rate=16000)),
    # 3D SmoothGrad haar J=2 (config c5 wavelet/mode), list y -- legacy in-loop averaging
    "s3_haar_list": dict(dim=3, shape=(2, 1, 16, 16, 16), seed=107, y=[1, 4], model="tinyvoxel",
                         kw=dict(wavelet="haar", J=2, method="smooth", mode="symmetric", n_samples=4,
                                 stdev_spread=0.05)),
    # 3D IG haar J=2 at 16^3 (the only size legacy 3D IG runs at)
    "ig3_haar_int": dict(dim=3, shape=(1, 1, 16, 16, 16), seed=108, y=2, model="tinyvoxel",
                         kw=dict(wavelet="haar", J=2, method="integratedgrad", mode="symmetric", n_samples=3)),
}


def make_inputs(case):
    rs = np.random.RandomState(case["seed"])
    x = rs.standard_normal(case["shape"]).astype(np.float32)
    if case["dim"] == 3:
        x = (x > 0.3).astype(np.float32)
    return torch.tensor(x), case["y"]


def make_model(case):
    if case["model"] == "tiny2d":
        return testmodels.TinySmooth2D()
    if case["model"] == "tinyaudio":
        return testmodels.TinyAudio()
    if case["model"] == "tinyvoxel":
        return testmodels.TinyVoxel()
    raise KeyError(case["model"])


# BaseWAM2D single passes with their .scales (disentangle_scales) -- make_base_goldens.py
BASE_CASES = {
    # approx row written for the last image only (stale img_batch); list y
    "b2_haar_approx": dict(dim=2, shape=(3, 3, 224, 224), seed=201, y=[1, 4, 2], model="tiny2d",
                           kw=dict(wavelet="haar", J=3, mode="reflect", approx_coeffs=True)),
    # db4 at 224: .scales canvas 230 (2 * finest width), int y, symmetric mode
    "b2_db4_int": dict(dim=2, shape=(2, 3, 224, 224), seed=202, y=6, model="tiny2d",
                       kw=dict(wavelet="db4", J=2, mode="symmetric", approx_coeffs=False)),
}
