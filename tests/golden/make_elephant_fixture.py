"""Config-c1 input fixture: assets/elephant.jpg preprocessed like wam_example.ipynb
(torchvision Resize(256) = PIL bilinear resize of the short side to 256, CenterCrop(224)),
stored as the uint8 RGB crop (ToTensor/Normalize are applied in the tests).
Run here only (the reference tree is absent on the GPU box):
    python tests/golden/make_elephant_fixture.py
"""
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
img = Image.open("/root/reference/assets/elephant.jpg").convert("RGB")
w, h = img.size
if w < h:
    nw, nh = 256, int(256 * h / w)
else:
    nw, nh = int(256 * w / h), 256
img = img.resize((nw, nh), Image.BILINEAR)
left = int(round((nw - 224) / 2.0))
top = int(round((nh - 224) / 2.0))
crop = np.asarray(img.crop((left, top, left + 224, top + 224)), dtype=np.uint8)
np.savez_compressed(os.path.join(HERE, "elephant_224.npz"), crop=crop)
print(crop.shape, crop.dtype, crop.mean())
