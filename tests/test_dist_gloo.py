"""Multi-process (world_size 2, gloo, CPU) coverage of the sharded path.

Each rank runs wam_amd.engine's sharding (Shard.range over noise samples / IG steps, the numpy
noise stream positioned for its slice, ig_weights / legacy3d_weights) with the oracle standing
in for the per-sample GPU pass, then all-reduces its partial accumulator exactly like the
classes do (Shard.all_reduce_sum). The combined result must equal the single-process reference.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import testmodels
        from oracle import wam_ref
        from wam_amd import engine

        shard = engine.Shard(True)
        assert (shard.rank, shard.world) == (rank, world)
        res = {}
        # --- 2D SmoothGrad: samples sharded, per-sample max stays local, SUM of mosaics
        rs = np.random.RandomState(0)
        x = torch.tensor(rs.standard_normal((2, 3, 224, 224)).astype(np.float32))
        model = testmodels.TinySmooth2D()
        n = 5
        lo, hi = shard.range(n)
        sig = [float(np.float32(0.25) * (x[i].max() - x[i].min())) for i in range(2)]
        acc = torch.zeros(2, 224, 224, dtype=torch.float64)
        for s, noise in engine.legacy_noise(sig, (3, 224, 224), 42, list(range(lo, hi))):
            noisy = x + torch.tensor(noise)
            _, g = wam_ref.single_pass_2d(model, noisy, [1, 2], "haar", 3, "reflect")
            acc += torch.tensor(wam_ref.mosaic_2d(g, True, (224, 224), (224, 224)))
        shard.all_reduce_sum(acc)
        res["smooth"] = (acc / n).numpy()
        # --- IG weighted form over sharded steps
        G = torch.tensor(np.random.RandomState(1).standard_normal((7, 50)).astype(np.float32))
        k0, k1 = shard.range(7)
        w = torch.tensor(engine.ig_weights(k0, k1 - k0, 7))
        part = (w[:, None] * G[k0:k1]).sum(0)
        shard.all_reduce_sum(part)
        res["ig"] = part.numpy()
        # --- legacy 3D averaging weights over sharded samples
        C = G.abs()
        s0, s1 = shard.range(7)
        w3 = torch.tensor(engine.legacy3d_weights(s0, s1 - s0, 7))
        part3 = (w3[:, None] * C[s0:s1]).sum(0)
        shard.all_reduce_sum(part3)
        res["cube"] = part3.numpy()
        # --- 2D SmoothGrad, batch (image) axis: ragged image ranges, each rank's per-sample band
        # maxima combined by an all-reduce MAX before normalising, rows gathered at the end (the
        # classes' dist_axis='images'; the loss seed of a rank's rows: engine.seed_gradient batch=)
        x3 = torch.tensor(np.random.RandomState(4).standard_normal((3, 3, 64, 64)).astype(np.float32))
        i0, i1 = shard.range(3)
        sig3 = [float(np.float32(0.25) * (x3[i].max() - x3[i].min())) for i in range(3)]
        acc3 = torch.zeros(i1 - i0, 64, 64, dtype=torch.float64)
        for s, noise in engine.legacy_noise(sig3, (3, 64, 64), 42, list(range(3))):
            noisy = (x3 + torch.tensor(noise))[i0:i1]
            _, g = wam_ref.single_pass_2d(model, noisy, [1, 2, 0][i0:i1], "db2", 2, "reflect")
            bands = [np.abs(g[0].mean(axis=1))] + [np.abs(t.mean(axis=1)) for lv in g[1:] for t in lv]
            # the oracle's loss is the mean over this rank's rows (1/n_local per item); the whole
            # batch's loss scales every item by 1/N (what seed_gradient(batch=) seeds)
            bands = [b * np.float32((i1 - i0) / 3.0) for b in bands]
            mx = torch.tensor([float(b.max()) for b in bands], dtype=torch.float32)
            shard.all_reduce_max(mx)
            normed = [b / np.float32(m) for b, m in zip(bands, mx.numpy())]
            gn = [normed[0][:, None]] + [tuple(normed[1 + 3 * k + j][:, None] for j in range(3))
                                         for k in range(len(g) - 1)]
            acc3 += torch.tensor(wam_ref.mosaic_2d(gn, False, (64, 64), (64, 64)))
        res["smooth_images"] = (shard.all_gather_rows(acc3, 3) / 3).numpy()
        # --- parameter gradients of a sharded call: per-rank increments summed once (every rank
        # in the same order; rank 1 has no samples of a 1-sample call and contributes zeros)
        pm = testmodels.TinySmooth2D()
        xg = torch.tensor(np.random.RandomState(6).standard_normal((3 * 2, 3, 16, 16)).astype(np.float32))
        for n_smp in (3, 1):
            for p_ in pm.parameters():
                p_.grad = None
            a0, a1 = shard.range(n_smp)
            with engine.param_grad_sum(engine.trainable_params(pm), shard):
                if a1 > a0:
                    engine.input_gradient(pm, xg[2 * a0:2 * a1], [1, 2], a1 - a0, 2)
            res["pgrad%d" % n_smp] = [p_.grad.clone().numpy() for p_ in pm.parameters()]
        # a trainable parameter no rank reaches (an unused head) keeps .grad None, as the
        # single-process loss.backward() leaves it (not zeros: optimizers would step on zeros)
        pa = testmodels.TinySmooth2DAux()
        a0, a1 = shard.range(3)
        with engine.param_grad_sum(engine.trainable_params(pa), shard):
            engine.input_gradient(pa, xg[2 * a0:2 * a1], [1, 2], a1 - a0, 2)
        res["aux_grad_none"] = pa.aux.weight.grad is None and pa.aux.bias.grad is None
        res["aux_conv_grad"] = pa.conv.weight.grad.clone().numpy()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_matches_single_process():
    from oracle import wam_ref
    import testmodels
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rs = np.random.RandomState(0)
    x = torch.tensor(rs.standard_normal((2, 3, 224, 224)).astype(np.float32))
    ref = wam_ref.smooth_2d(testmodels.TinySmooth2D(), x, [1, 2], wavelet="haar", J=3, n_samples=5)
    G = np.random.RandomState(1).standard_normal((7, 50)).astype(np.float32)
    avg = np.zeros(50, dtype=np.float32)
    for s in range(7):
        avg = (avg + np.abs(G[s])) / np.float32(7)
    for r in range(world):
        assert np.abs(out[r]["smooth"] - ref).max() < 1e-12   # same per-sample maps, fp64 sums
        assert np.allclose(out[r]["ig"], np.trapz(G, axis=0), rtol=1e-5, atol=1e-6)
        assert np.allclose(out[r]["cube"], avg, rtol=1e-5, atol=1e-30)
        assert np.array_equal(out[0]["smooth"], out[r]["smooth"])
        ref3 = wam_ref.smooth_2d(testmodels.TinySmooth2D(), torch.tensor(np.random.RandomState(4).standard_normal(
            (3, 3, 64, 64)).astype(np.float32)), [1, 2, 0], wavelet="db2", J=2, n_samples=3, frame="native")
        for n_smp in (3, 1):
            pm = testmodels.TinySmooth2D()
            xg = torch.tensor(np.random.RandomState(6).standard_normal((3 * 2, 3, 16, 16)).astype(np.float32))
            from wam_amd import engine
            engine.input_gradient(pm, xg[:2 * n_smp], [1, 2], n_smp, 2)
            for got, p_ in zip(out[r]["pgrad%d" % n_smp], pm.parameters()):
                assert np.allclose(got, p_.grad.numpy(), rtol=1e-5, atol=1e-7)
        assert out[r]["aux_grad_none"]
        pa = testmodels.TinySmooth2DAux()
        engine.input_gradient(pa, xg[:6], [1, 2], 3, 2)
        assert np.allclose(out[r]["aux_conv_grad"], pa.conv.weight.grad.numpy(), rtol=1e-5, atol=1e-7)
        assert out[r]["smooth_images"].shape == ref3.shape
        assert np.abs(out[r]["smooth_images"] - ref3).max() < 1e-6
