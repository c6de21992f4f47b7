"""Test helpers shared by the CPU and GPU suites."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_NPZ = {}


def npz(name):
    if name not in _NPZ:
        _NPZ[name] = np.load(os.path.join(GOLDEN, name))
    return _NPZ[name]


def pywt_cases(dim):
    d = npz("pywt_dwt.npz")
    keys = sorted({k[:6] for k in d.files if k.startswith("d%d_" % dim)})
    out = []
    for k in keys:
        wav, mode, J = d[k + "_meta"]
        out.append((k, str(wav), str(mode), int(J)))
    return out


def pywt_coeffs(case, dim, J, prefix="c"):
    """Load [A, details...] of a fixture case in the oracle's container format."""
    d = npz("pywt_dwt.npz")
    if dim == 1:
        return [d["%s_%s%d" % (case, prefix, j)] for j in range(J + 1)]
    if dim == 2:
        return [d["%s_%s0" % (case, prefix)]] + [tuple(d["%s_%s%d%s" % (case, prefix, j, n)] for n in "hvd")
                                                for j in range(1, J + 1)]
    keys = ["aad", "ada", "add", "daa", "dad", "dda", "ddd"]
    return [d["%s_%s0" % (case, prefix)]] + [{k: d["%s_%s%d%s" % (case, prefix, j, k)] for k in keys}
                                            for j in range(1, J + 1)]


def flat_bands(coeffs, dim):
    """oracle container -> list of band arrays in ptwt order."""
    if dim == 1:
        return list(coeffs)
    if dim == 2:
        return [coeffs[0]] + [t for lv in coeffs[1:] for t in lv]
    keys = ["aad", "ada", "add", "daa", "dad", "dda", "ddd"]
    return [coeffs[0]] + [lv[k] for lv in coeffs[1:] for k in keys]


def max_rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(1e-30, np.abs(b).max()))
