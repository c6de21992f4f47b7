"""World-2 run of the WAM classes with dist=... (one process per rank, both on cuda:0, gloo).

Launched by tests/conftest.py BEFORE the pytest process touches the GPU (a process that has
initialised the GPU must not start programs itself):

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port P tests/dist_worker.py OUT.json

Every rank computes each case twice -- unsharded (dist=None) and sharded (dist=True, the given
dist_axis) -- and rank 0 writes {case: max |sharded - unsharded| / max(1, max |unsharded|)} plus
any exception text to OUT.json. Cases cover SURVEY 8(e): ragged sample / step splits, batch
(image) sharding with the all-reduce MAX of the batch-global maxima, int-y loss scaling with
unnormalised maps, 1D with fewer samples than ranks (an empty range), 3D legacy weights, IG, and
uneven image splits whose sample range is cut into several chunks (N=23 images, 25 samples).
"""
import json
import os
import sys
import traceback

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def cases():
    import testmodels
    rs = np.random.RandomState(31)
    x2 = torch.tensor(rs.standard_normal((3, 3, 224, 224)).astype(np.float32))
    x96 = torch.tensor(rs.standard_normal((3, 3, 96, 96)).astype(np.float32))
    x1 = torch.tensor(rs.standard_normal((3, 4000)).astype(np.float32))
    x3 = torch.tensor((rs.standard_normal((2, 1, 16, 16, 16)) > 0).astype(np.float32))
    x23 = torch.tensor(rs.standard_normal((23, 3, 64, 64)).astype(np.float32))
    y23 = [int(v) for v in rs.randint(0, 10, 23)]
    m2, m1, m3 = testmodels.TinySmooth2D, testmodels.TinyAudio, testmodels.TinyVoxel
    # uneven image split (12 / 11) with the default (auto) axis and chunk sizes: the ranks must cut
    # the 25 samples / steps at the same points (rank-local group sizes paired
    # band-maximum tensors of different sizes in the all-reduce MAX)
    yield ("2d_smooth_numpy_auto_uneven_23", "2D", m2, x23, y23,
           dict(wavelet="haar", J=3, n_samples=25, frame="native"))
    yield ("2d_smooth_philox_auto_uneven_23", "2D", m2, x23, y23,
           dict(wavelet="db4", J=2, n_samples=25, noise="philox", frame="native"))
    yield ("2d_ig_auto_uneven_23", "2D", m2, x23, y23,
           dict(wavelet="haar", J=2, method="integratedgrad", n_samples=25, frame="native"))
    # a trainable head forward() never uses: .grad stays None on every rank
    yield ("2d_smooth_unused_head_samples", "2D", testmodels.TinySmooth2DAux, x2, [1, 4, 2],
           dict(wavelet="haar", J=2, n_samples=3, dist_axis="samples"))
    yield ("2d_smooth_numpy_samples", "2D", m2, x2, [1, 4, 2],
           dict(wavelet="haar", J=3, n_samples=5, dist_axis="samples"))
    yield ("2d_smooth_philox_images", "2D", m2, x2, [1, 4, 2],
           dict(wavelet="db4", J=3, n_samples=4, noise="philox", frame="native", dist_axis="images"))
    yield ("2d_smooth_numpy_images_int_y_unnormalised", "2D", m2, x2, 5,
           dict(wavelet="haar", J=2, n_samples=3, normalize_coeffs=False, dist_axis="images"))
    yield ("2d_ig_samples", "2D", m2, x96, [0, 1, 2],
           dict(wavelet="db4", J=2, method="integratedgrad", n_samples=5, frame="native", dist_axis="samples"))
    yield ("2d_ig_images", "2D", m2, x96, [0, 1, 2],
           dict(wavelet="sym4", J=2, method="integratedgrad", n_samples=4, frame="native", dist_axis="images"))
    yield ("1d_smooth_one_sample", "1D", m1, x1, [1, 2, 3],
           dict(wavelet="db6", J=3, n_samples=1, sample_rate=16000))
    yield ("1d_smooth", "1D", m1, x1, [1, 2, 3], dict(wavelet="db6", J=3, n_samples=3, sample_rate=16000))
    yield ("1d_ig", "1D", m1, x1, 4, dict(wavelet="haar", J=3, method="integratedgrad", n_samples=3,
                                          sample_rate=16000))
    yield ("3d_smooth_legacy_weights", "3D", m3, x3, [1, 2], dict(wavelet="haar", J=2, n_samples=3,
                                                                  stdev_spread=0.05))
    yield ("3d_ig", "3D", m3, x3, [1, 2], dict(wavelet="haar", J=2, method="integratedgrad", n_samples=3))


def flat(r):
    if isinstance(r, tuple):  # 1D: (melspec grads, [coefficient grads])
        return np.concatenate([np.asarray(r[0]).ravel()] + [np.asarray(c).ravel() for c in r[1]])
    return np.asarray(r).ravel()


def main():
    out_path = sys.argv[1]
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    import wam_amd
    res = {}
    for name, dim, model, x, y, kw in cases():
        try:
            cls = getattr(wam_amd, "WaveletAttribution" + dim)
            m_ref, m_sh = model().cuda(), model().cuda()
            ref = flat(cls(m_ref, **kw)(x, y))
            got = flat(cls(m_sh, dist=True, **kw)(x, y))
            err = float(np.abs(got - ref).max() / max(1.0, np.abs(ref).max())) if got.shape == ref.shape else 1e9
            # the model's .grad after the call: per-rank increments summed over the ranks
            # (engine.param_grad_sum) must equal the single-process call's
            gerr = 0.0
            for a, b in zip(m_sh.parameters(), m_ref.parameters()):
                if (a.grad is None) != (b.grad is None):
                    gerr = 1e9
                elif a.grad is not None:
                    ga, gb = a.grad.double().cpu(), b.grad.double().cpu()
                    gerr = max(gerr, float((ga - gb).abs().max() / max(1e-30, float(gb.abs().max()))))
            res[name] = {"err": err, "shape_ok": got.shape == ref.shape, "grad_err": gerr}
        except Exception:
            res[name] = {"error": traceback.format_exc()}
        dist.barrier()
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
