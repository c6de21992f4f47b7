"""f2 goldens: the REFERENCE's own wavelet-domain filters of ``lib/wam_1D.py`` with the REAL
PyWavelets 1.1.1 -- ``BaseWAM1D.filter`` (:221-246) and ``VisualizerWAM1D.
filter_from_wavelet_coefficients`` ('ht', 'st', 'modulation'; :532-587).

    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 tests/golden/make_f2_goldens.py

Python 3.9 has PyWavelets but no torch: torch / torchaudio / ptwt / librosa are empty stand-in
modules (these methods use numpy and pywt only); instances are made without __init__ and given
the attributes the methods read. Writes tests/golden/f2_goldens.npz (outputs only).
"""
import os
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))

CASES = {"db6_J3": ("db6", 3, (3, 4001), 501), "haar_J2": ("haar", 2, (2, 1000), 502),
         "sym4_J4": ("sym4", 4, (2, 3000), 503)}


def inputs(wav, J, shape, seed, pywt_mod=None):
    """coefficients (pywt wavedec, mode reflect, of a random signal) and random gradients"""
    rs = np.random.RandomState(seed)
    x = rs.standard_normal(shape).astype(np.float32)
    if pywt_mod is None:
        from oracle import dwt
        coeffs = [c.astype(np.float32) for c in dwt.wavedec(x.astype(np.float64), wav, J, mode="reflect")]
    else:
        coeffs = [c.astype(np.float32) for c in pywt_mod.wavedec(x, wav, level=J, mode="reflect")]
    grads = [rs.standard_normal(c.shape).astype(np.float32) for c in coeffs]
    return x, coeffs, grads


def main():
    for name in ("torch", "torchaudio", "torchaudio.transforms", "ptwt", "librosa"):
        sys.modules[name] = types.ModuleType(name)
    sys.modules["torchaudio.transforms"].MelSpectrogram = sys.modules["torchaudio.transforms"].AmplitudeToDB = object
    sys.modules["torchaudio"].transforms = sys.modules["torchaudio.transforms"]
    sys.path.insert(0, "/root/reference")
    import pywt
    import lib.wam_1D as w1
    out = {}
    for name, (wav, J, shape, seed) in CASES.items():
        x, coeffs, grads = inputs(wav, J, shape, seed, pywt)
        v = object.__new__(w1.VisualizerWAM1D)
        v.wavelet = wav
        for m in ("ht", "st", "modulation"):
            out["%s_%s" % (name, m)] = v.filter_from_wavelet_coefficients(coeffs, grads, filtering_method=m, EPS=0.2)
        b = object.__new__(w1.BaseWAM1D)
        b.wavelet, b.gradient_coeffs, b.wavelet_coeffs = wav, grads, coeffs
        out["%s_filter" % name] = b.filter(0.3)
        print(name, {k: v.shape for k, v in out.items() if k.startswith(name)})
    np.savez_compressed(os.path.join(HERE, "f2_goldens.npz"), **out)


if __name__ == "__main__":
    main()
