"""Filter banks (PyWavelets 1.1.1 tables exported to data/filters.json by
tests/golden/make_pywt_fixtures.py). Accepts a wavelet name, a pywt.Wavelet-like object
(``.name`` / ``.filter_bank``) or a ``Wavelet`` from this module, as ptwt does."""
import json
import os
from collections import namedtuple

Wavelet = namedtuple("Wavelet", ["name", "dec_lo", "dec_hi", "rec_lo", "rec_hi"])

_TABLE = None


def _table():
    global _TABLE
    if _TABLE is None:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "filters.json")) as f:
            _TABLE = json.load(f)["wavelets"]
    return _TABLE


def wavelist():
    return sorted(_table())


def get_wavelet(w):
    if isinstance(w, Wavelet):
        return w
    if isinstance(w, str):
        t = _table()
        if w not in t:
            raise ValueError("Unknown wavelet name '%s', check wavelist() for the list of available builtin "
                             "wavelets." % w)
        e = t[w]
        return Wavelet(w, tuple(e["dec_lo"]), tuple(e["dec_hi"]), tuple(e["rec_lo"]), tuple(e["rec_hi"]))
    fb = getattr(w, "filter_bank", None)
    if fb is not None:
        return Wavelet(getattr(w, "name", "custom"), *[tuple(map(float, f)) for f in fb])
    raise TypeError("wavelet must be a name, a pywt.Wavelet-like object or wam_amd.filters.Wavelet")


MODES = {"zero": 0, "reflect": 1, "symmetric": 2, "constant": 3, "periodic": 4}


def mode_id(mode):
    if mode not in MODES:
        raise ValueError("Padding mode not supported: %r (wam_amd supports %s)" % (mode, sorted(MODES)))
    return MODES[mode]
