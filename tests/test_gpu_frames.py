"""The mosaic accumulation in coefficient order (wam_frame_accumulate_coef, the path the classes
use) vs the per-pixel gather form (wam_frame_accumulate): bit-identical fp64 frames (same per-pixel
sum order), for the legacy and native c2 mosaics, normalised and not."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wav,frame", [("db4", "native"), ("haar", "legacy"), ("haar", "native")])
@pytest.mark.parametrize("normalize", [True, False])
def test_coef_order_equals_gather(wav, frame, normalize):
    from wam_amd import frames, plan as P
    from wam_amd._lib import check, lib, ptr, stream_of
    p = P.get_plan(2, (224, 224), 3, wav, "reflect", "cuda")
    n, groups = 5, 11
    gmap, (rh, rw) = frames.smooth_frame(p, n, frame, "cuda")
    torch.manual_seed(4)
    maps = torch.rand(groups * n * p.coeff_numel, device="cuda")
    bmax = torch.rand(groups, p.nbands, device="cuda") + 0.5
    base = torch.randn(n, rh, rw, dtype=torch.float64, device="cuda")
    a, b = base.clone(), base.clone()
    P.frame_accumulate(groups, n, gmap, maps, p.coeff_numel, bmax, p.nbands, normalize, a)
    assert P._inverse_map(gmap, p.coeff_numel) is not None  # the classes' path is the coefficient order
    src, band = gmap
    check(lib.wam_frame_accumulate(groups, n, src.numel(), ptr(src), ptr(band), ptr(maps), p.coeff_numel, ptr(bmax),
                                   p.nbands, int(normalize), ptr(b), stream_of(b.device)))
    assert torch.equal(a, b)
