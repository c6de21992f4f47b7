"""f3 goldens: the REFERENCE's own ``src/evaluation_helpers.py`` with the REAL PyWavelets 1.1.1.

Run in this container only, with the survey's Python 3.9 (PyWavelets 1.1.1, scipy 1.7.1, PIL 8.4;
no torch there, so ``torch`` / ``torchaudio`` are empty stand-in modules -- the helpers used below
never touch them):

    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 tests/golden/make_eval_goldens.py

Captured (outputs only; inputs regenerated from RandomState / random.seed in the tests):
  masks      generate_masks(8, wam) insertion / deletion masks (:455-505)
  rec_haar   reconstruct_images(img, 3, masks, 'haar') -> uint8 images (pywt.coeffs_to_array layout,
             float32 analysis, float64 synthesis, min-max normalise, uint8) (:507-541)
  rec_db2    the same for db2 (non-dyadic 231x231 coefficient array, 226x226 reconstructions)
  auc        compute_auc (:437-453); importances: sum_importance with generate_subsets (:361-393,
             :580-594); zoom_map: scipy zoom order 0 of a cell-index grid; gauss: gaussian_filter
"""
import os
import random
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))


def install_standins():
    torch = types.ModuleType("torch")
    nn = types.ModuleType("torch.nn")
    fn = types.ModuleType("torch.nn.functional")
    torch.nn, nn.functional = nn, fn
    ta = types.ModuleType("torchaudio")
    tat = types.ModuleType("torchaudio.transforms")
    tat.MelSpectrogram = tat.AmplitudeToDB = object
    ta.transforms = tat
    sys.modules.update({"torch": torch, "torch.nn": nn, "torch.nn.functional": fn, "torchaudio": ta,
                        "torchaudio.transforms": tat})


def inputs():
    img = np.random.RandomState(301).uniform(size=(224, 224, 3)).astype(np.float32)
    wam = np.random.RandomState(302).uniform(size=(224, 224))
    masks_db2 = np.random.RandomState(303).uniform(size=(2, 231, 231))
    probs = np.random.RandomState(304).uniform(size=17).astype(np.float32)
    return img, wam, masks_db2, probs


def main():
    install_standins()
    sys.path.insert(0, "/root/reference/src")
    import evaluation_helpers as eh  # noqa: E402
    from scipy.ndimage import gaussian_filter, zoom  # noqa: E402
    img, wam, masks_db2, probs = inputs()
    ins, dele = eh.generate_masks(8, wam)
    out = {"ins": ins.astype(np.uint8), "del": dele.astype(np.uint8)}
    sel = ins[[0, 2, 5, 8]]
    out["rec_haar"] = np.stack([np.array(im) for im in eh.reconstruct_images(img, 3, sel, wavelet="haar")])
    out["rec_db2"] = np.stack([np.array(im) for im in eh.reconstruct_images(img, 3, masks_db2, wavelet="db2")])
    out["auc"] = np.float32(eh.compute_auc(probs))
    random.seed(7)
    idx = eh.generate_subsets(28, 157, 16)
    out["subsets"] = np.array(idx, dtype=np.int16)
    out["importances"] = eh.sum_importance(wam, idx, 28, 16, batch_size=5)
    out["zoom_map"] = zoom(np.arange(28 * 28, dtype=np.float64).reshape(1, 28, 28), (1, 8, 8), order=0)[0]
    out["gauss"] = gaussian_filter(wam, sigma=2)
    np.savez_compressed(os.path.join(HERE, "eval_goldens.npz"), **out)
    print({k: (v.shape, v.dtype) for k, v in out.items()})


if __name__ == "__main__":
    main()
