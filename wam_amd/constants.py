"""ptwt-compatible containers (ptwt.constants.WaveletDetailTuple2d, used at lib/wam_2D.py:29,41,105,469)."""
from collections import namedtuple

WaveletDetailTuple2d = namedtuple("WaveletDetailTuple2d", ["horizontal", "vertical", "diagonal"])

# 3D detail keys in ptwt / pywt order (first letter = axis -3; 'a' = lowpass, 'd' = highpass)
KEYS3 = ("aad", "ada", "add", "daa", "dad", "dda", "ddd")
