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


# ------------------------------------------------------------------ Philox noise stream (host)
# Host restatement of wam_amd/csrc/rng.hpp (the library's own 'philox' noise stream; the reference
# has no counterpart -- its noise is numpy's legacy stream, see oracle.wam_ref.legacy_noise_stream).
_M0, _M1, _W0, _W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
_U32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 (Salmon et al., SC'11) on uint32 arrays -> 4 uint32 arrays."""
    c = [np.asarray(v, dtype=np.uint64) & _U32 for v in (c0, c1, c2, c3)]
    k0, k1 = np.uint64(k0) & _U32, np.uint64(k1) & _U32
    for _ in range(10):
        p0 = np.uint64(_M0) * c[0]
        p1 = np.uint64(_M1) * c[2]
        c = [(p1 >> np.uint64(32)) ^ c[1] ^ k0, p1 & _U32, (p0 >> np.uint64(32)) ^ c[3] ^ k1, p0 & _U32]
        k0 = (k0 + np.uint64(_W0)) & _U32
        k1 = (k1 + np.uint64(_W1)) & _U32
    return [v.astype(np.uint32) for v in c]


def philox_normals(n_elems, item, sample, seed):
    """The N(0,1) values wam_noise_add draws for elements 0..n_elems-1 of (item, sample)."""
    g = np.arange((n_elems + 3) // 4, dtype=np.uint64)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    c1 = (g >> np.uint64(32)) ^ np.uint64((item << 8) & 0xFFFFFFFF)
    r = philox4x32_10(g, c1, np.full_like(g, sample), np.full_like(g, item), k0, k1)
    out = np.empty((g.size, 4))
    for pair, (a, b) in enumerate(((r[0], r[1]), (r[2], r[3]))):
        u1 = (a.astype(np.float32) + np.float32(1.0)) * np.float32(2.0 ** -32)
        u2 = b.astype(np.float32) * np.float32(2.0 ** -32)
        rad = np.sqrt(-2.0 * np.log(u1.astype(np.float64)))
        out[:, 2 * pair] = rad * np.cos(2 * np.pi * u2.astype(np.float64))
        out[:, 2 * pair + 1] = rad * np.sin(2 * np.pi * u2.astype(np.float64))
    return out.reshape(-1)[:n_elems]
