"""wam_amd -- MI355X-native Wavelet Attribution Method (WAM) hot path.

Drop-in for the reference's ``lib/wam_1D.py``, ``lib/wam_2D.py`` and ``lib/wam_3D.py``
(same classes, signatures, return types) with every WAM-owned operation on hand-written gfx950
HIP kernels (``libwam_hip.so``, C-ABI in ``include/wam_hip.h``). The explained model's
forward/backward stays in PyTorch-ROCm.

    from wam_amd.wam_2D import WaveletAttribution2D      # was: from lib.wam_2D import ...

Importing this package loads libwam_hip.so and fails loudly when it is missing.
"""
from . import _lib  # noqa: F401  (loads libwam_hip.so; raises ImportError if absent)
from .constants import WaveletDetailTuple2d
from .transforms import wavedec, wavedec2, wavedec3, waverec, waverec2, waverec3
from .wam_1D import BaseWAM1D, VisualizerWAM1D, WaveletAttribution1D
from .wam_2D import BaseWAM2D, WaveletAttribution2D
from .wam_3D import BaseWAM3D, WaveletAttribution3D
from .evaluation import Eval2DWAM

__all__ = ["WaveletDetailTuple2d", "wavedec", "waverec", "wavedec2", "waverec2", "wavedec3", "waverec3",
           "BaseWAM1D", "WaveletAttribution1D", "VisualizerWAM1D", "BaseWAM2D", "WaveletAttribution2D", "BaseWAM3D",
           "WaveletAttribution3D", "Eval2DWAM"]
