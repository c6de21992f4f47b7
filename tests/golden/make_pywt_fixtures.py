"""Generate the DWT known-answer fixtures that pin the oracle (and through it the HIP kernels).

Run with the interpreter that has PyWavelets 1.1.1 (this container: ``/opt/conda/bin/python3.9``):

    /opt/conda/bin/python3.9 tests/golden/make_pywt_fixtures.py

Why pywt: the reference delegates all wavelet arithmetic to ``ptwt`` (an unvendored, unpinned PyPI
dependency, ``requirements.txt:7`` ``ptwt>=0.1.0``; de-facto 1.0.1 per ``Fourier(1).ipynb``), whose
documented design target is equality with PyWavelets for the modes WAM uses. ptwt is not available
offline; PyWavelets 1.1.1 is. So the fixtures are pywt outputs, plus a subset of the MATLAB R2012a
single-level known answers that ship inside pywt's own test data.

Outputs (all small, committed):
  wam_amd/data/filters.json       -- filter banks (dec_lo, dec_hi, rec_lo, rec_hi), float64, every
                                     discrete pywt wavelet. Data table only.
  tests/golden/pywt_dwt.npz       -- multilevel wavedec / waverec known answers, 1D / 2D / 3D
  tests/golden/matlab_dwt.npz     -- MATLAB R2012a single-level dwt subset (inputs + ma + md)
"""
import json
import os

import numpy as np
import pywt

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def export_filters():
    out = {}
    for name in pywt.wavelist(kind="discrete"):
        w = pywt.Wavelet(name)
        out[name] = {
            "dec_lo": list(map(float, w.dec_lo)),
            "dec_hi": list(map(float, w.dec_hi)),
            "rec_lo": list(map(float, w.rec_lo)),
            "rec_hi": list(map(float, w.rec_hi)),
            "orthogonal": bool(w.orthogonal),
        }
    path = os.path.join(REPO, "wam_amd", "data", "filters.json")
    with open(path, "w") as f:
        json.dump({"source": "PyWavelets %s" % pywt.__version__, "wavelets": out}, f)
    print("wrote", path, len(out), "wavelets")


def _put(store, key, arr):
    assert key not in store, key
    store[key] = np.asarray(arr)


def dwt_cases():
    store = {}
    rs = np.random.RandomState(20240601)
    modes = ["reflect", "zero", "symmetric", "constant", "periodic"]

    # ---- 1D: wavedec / waverec --------------------------------------------------------------
    idx = 0
    for wav in ["haar", "db2", "db4", "db6", "sym4", "sym8", "coif2"]:
        for mode in modes:
            for n, J in [(64, 3), (101, 3), (37, 2)]:
                x = rs.randn(2, n)
                cs = pywt.wavedec(x, wav, mode=mode, level=J, axis=-1)
                rec = pywt.waverec(cs, wav, mode=mode, axis=-1)
                # independent synthesis check: random coefficients of the same shapes
                rcs = [rs.randn(*c.shape) for c in cs]
                rrec = pywt.waverec(rcs, wav, mode=mode, axis=-1)
                k = "d1_%03d" % idx
                _put(store, k + "_meta", np.array([wav, mode, str(J)]))
                _put(store, k + "_x", x)
                for j, c in enumerate(cs):
                    _put(store, k + "_c%d" % j, c)
                    _put(store, k + "_r%d" % j, rcs[j])
                _put(store, k + "_rec", rec)
                _put(store, k + "_rrec", rrec)
                idx += 1

    # ---- 2D: wavedec2 / waverec2 --------------------------------------------------------------
    idx = 0
    for wav in ["haar", "db4", "db6", "sym8", "coif1"]:
        for mode in modes:
            cases = [((24, 24), 2), ((29, 35), 2)]
            if wav in ("haar", "db4") and mode in ("reflect", "zero", "symmetric"):
                cases.append(((48, 48), 3))
            for shape, J in cases:
                x = rs.randn(1, *shape)
                cs = pywt.wavedec2(x, wav, mode=mode, level=J, axes=(-2, -1))
                rec = pywt.waverec2(cs, wav, mode=mode, axes=(-2, -1))
                rcs = [rs.randn(*cs[0].shape)] + [tuple(rs.randn(*d.shape) for d in t) for t in cs[1:]]
                rrec = pywt.waverec2(rcs, wav, mode=mode, axes=(-2, -1))
                k = "d2_%03d" % idx
                _put(store, k + "_meta", np.array([wav, mode, str(J)]))
                _put(store, k + "_x", x)
                _put(store, k + "_c0", cs[0])
                _put(store, k + "_r0", rcs[0])
                for j, (t, rt) in enumerate(zip(cs[1:], rcs[1:])):
                    for o, name in enumerate("hvd"):
                        _put(store, k + "_c%d%s" % (j + 1, name), t[o])
                        _put(store, k + "_r%d%s" % (j + 1, name), rt[o])
                _put(store, k + "_rec", rec)
                _put(store, k + "_rrec", rrec)
                idx += 1

    # ---- 3D: wavedecn / waverecn ------------------------------------------------------------
    idx = 0
    keys = ["aad", "ada", "add", "daa", "dad", "dda", "ddd"]
    for wav in ["haar", "db4"]:
        for mode in ["reflect", "zero", "symmetric"]:
            for shape, J in [((12, 12, 12), 2), ((13, 11, 10), 2)]:
                x = rs.randn(1, *shape)
                cs = pywt.wavedecn(x, wav, mode=mode, level=J, axes=(-3, -2, -1))
                rec = pywt.waverecn(cs, wav, mode=mode, axes=(-3, -2, -1))
                rcs = [rs.randn(*cs[0].shape)] + [{kk: rs.randn(*d[kk].shape) for kk in keys} for d in cs[1:]]
                rrec = pywt.waverecn(rcs, wav, mode=mode, axes=(-3, -2, -1))
                k = "d3_%03d" % idx
                _put(store, k + "_meta", np.array([wav, mode, str(J)]))
                _put(store, k + "_x", x)
                _put(store, k + "_c0", cs[0])
                _put(store, k + "_r0", rcs[0])
                for j, (d, rd) in enumerate(zip(cs[1:], rcs[1:])):
                    for kk in keys:
                        _put(store, k + "_c%d%s" % (j + 1, kk), d[kk])
                        _put(store, k + "_r%d%s" % (j + 1, kk), rd[kk])
                _put(store, k + "_rec", rec)
                _put(store, k + "_rrec", rrec)
                idx += 1
    path = os.path.join(HERE, "pywt_dwt.npz")
    np.savez_compressed(path, **store)
    print("wrote", path, len(store), "arrays")


def matlab_subset():
    """Replays pywt's own test_matlab_compatibility input stream (RandomState(1234), sizes
    (dec_len, dec_len+1) per wavelet in family order) and keeps the orthogonal-family cases for
    the modes ptwt exposes."""
    ref = np.load(os.path.join(os.path.dirname(pywt.__file__), "tests", "data",
                               "dwt_matlabR2012a_result.npz"))
    modes = [("zero", "zpd"), ("constant", "sp0"), ("symmetric", "sym"), ("reflect", "symw"),
             ("periodic", "ppd")]
    keep = {"db1", "db2", "db4", "db6", "db8", "sym4", "sym8", "coif1", "coif3"}
    families = ("db", "sym", "coif", "bior", "rbio")
    wavelets = sum([pywt.wavelist(name) for name in families], [])
    rstate = np.random.RandomState(1234)
    store = {}
    n_kept = 0
    for wav in wavelets:
        w = pywt.Wavelet(wav)
        for N in (w.dec_len, w.dec_len + 1):
            data = rstate.randn(N)
            if wav not in keep:
                continue
            for pmode, mmode in modes:
                ma = np.asarray(ref["_".join([mmode, wav, str(N), "ma"])]).ravel()
                md = np.asarray(ref["_".join([mmode, wav, str(N), "md"])]).ravel()
                pa, pd = pywt.dwt(data, w, pmode)
                # the replayed input stream must reproduce pywt's own agreement with MATLAB
                assert np.sqrt(np.mean((pa - ma) ** 2)) < 5e-5, (wav, N, pmode)
                assert np.sqrt(np.mean((pd - md) ** 2)) < 5e-5, (wav, N, pmode)
                k = "%s_%s_%d" % (pmode, wav, N)
                store[k + "_x"] = data
                store[k + "_ma"] = ma
                store[k + "_md"] = md
                n_kept += 1
    path = os.path.join(HERE, "matlab_dwt.npz")
    np.savez_compressed(path, **store)
    print("wrote", path, n_kept, "cases")


if __name__ == "__main__":
    export_filters()
    dwt_cases()
    matlab_subset()
