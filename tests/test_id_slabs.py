"""GPU suite: the single-frame render over 4-byte id slabs (the product
default for sparse frames; raster_render_ids_kernel, two
one-tile waves per workgroup, against the generic kernel: A/B knob 38 = 1)
against the render over 48-byte
slab records (A/B knob 24 = 1, diagnostic library) and the banded kernel
(knob 0 = 2, records).  Same entries per tile, same id order, same blend: the
images must be bit-identical, including tiles past 256 entries (the id
slabs: their first 256 ids rebuilt from the bboxes; the record slabs: sorted
from the slab and its overflow ids up to 1024 entries, rebuilt past that), ragged image sizes and a frame with no
intersections (rasterize_sum.py:121-127's background) -- and within 1e-5 of
the C oracle's render of the same activations.  The calls go through
render_frame_sum, i.e. the ordered projection after the first call."""
import numpy as np
import pytest
import torch

from conftest import knobs

pytestmark = pytest.mark.gpu


def _frame(n, seed, chol, dev, cluster=0.0):
    g = torch.Generator().manual_seed(seed)
    xyz = torch.atanh(2 * (torch.rand(n, 2, generator=g) - 0.5) * 0.999)
    if cluster > 0:  # a share of the splats piled onto a few tiles
        k = int(n * cluster)
        xyz[:k] = torch.atanh(0.02 * (torch.rand(k, 2, generator=g) - 0.5))
    chol = torch.rand(n, 3, generator=g) * chol
    feat = torch.rand(n, 3, generator=g)
    return xyz.to(dev), chol.to(dev), feat.to(dev)


@pytest.mark.parametrize("n,H,W,chol,cluster", [
    (10000, 1080, 1920, 1.0, 0.0),
    (50000, 1080, 1920, 3.0, 0.0),
    (20000, 360, 640, 1.0, 0.2),   # tiles past 256 entries
    (20000, 360, 640, 1.0, 0.03),  # past 256 but within the record slabs' overflow ids (1024)
    (3000, 250, 333, 1.0, 0.0),    # ragged edge tiles
    (3000, 200, 300, 1.0, 0.0),    # an odd tile count (247): the last two-tile workgroup's second wave idle
    (500, 128, 128, 0.0, 0.0),     # L = 0 (no bound): no intersections, the background
])
def test_id_slab_render_bit_identical(cuda, oracle, n, H, W, chol, cluster):
    from gsvc_amd.render import render_frame_sum
    xyz, c, f = _frame(n, 7 + n, chol, cuda, cluster)
    bound = torch.tensor([0.5, 0.0, 0.5], device=cuda) if chol > 0 else None
    bg = torch.tensor([0.3, 0.6, 0.9], device=cuda)
    ref = [render_frame_sum(xyz, c, f, H, W, bg, cholesky_bound=bound) for _ in range(2)]
    got = []
    # records; banded; the order at any density; the generic one-wave kernel
    # instead of raster_render_ids_kernel
    for pair in ((24, 1), (0, 2), (27, 1), (38, 1)):
        with knobs(pair):
            got += [render_frame_sum(xyz, c, f, H, W, bg, cholesky_bound=bound) for _ in range(3)]
    torch.cuda.synchronize()
    assert torch.equal(ref[0], ref[1])
    for g in got:
        assert torch.equal(g, ref[0])
    if chol == 0:
        assert torch.equal(ref[0][0], bg.view(3, 1, 1).expand(3, H, W))
    else:
        # and against the C oracle on the GPU's own activations (torch.tanh ==
        # the kernel's tanhf, test_gpu_sync_free.test_tanh_matches_torch)
        means = torch.tanh(xyz).cpu().numpy()
        L = (c + bound).cpu().numpy()
        r = oracle.render_sum(means, L, f.cpu().numpy(), np.ones((n, 1), np.float32), H, W)
        want = np.clip(r["out"], 0, 1).transpose(2, 0, 1) if r["m"] > 0 else None
        if want is not None:
            np.testing.assert_allclose(ref[0][0].cpu().numpy(), want, rtol=0, atol=1e-5)


def test_needle_splats_every_route(cuda, oracle):
    """Near-singular conics (needles: l22 ~ 1e-4, so a*c / det ~ 1e7): the
    reference's float32 sigma cancels along the needle, and alpha reads 1 far
    outside the true ellipse; the kernels' ellipse culling must leave such
    entries alone (cull.h cull_conditioned).  Sparse id slabs, the banded
    kernel and the record slabs bit-identical, and the C oracle within 1e-5
    (round 5: the banded kernel culled a textured-video needle at 2-3 pixels)."""
    from gsvc_amd.render import render_frame_sum
    H, W, n = 256, 384, 3000
    xyz, c, f = _frame(n, 4242, 1.0, cuda)
    g = torch.Generator().manual_seed(9)
    k = 300
    needle = torch.stack([1.0 + 3.0 * torch.rand(k, generator=g),
                          4.0 * (torch.rand(k, generator=g) - 0.5),
                          torch.full((k,), -0.5 + 1e-4)], 1)
    c[:k] = needle.to(cuda)
    bound = torch.tensor([0.5, 0.0, 0.5], device=cuda)
    bg = torch.tensor([0.3, 0.6, 0.9], device=cuda)
    ref = render_frame_sum(xyz, c, f, H, W, bg, cholesky_bound=bound)
    got = []
    for pair in ((24, 1), (0, 2), (0, 1), (38, 1)):  # records; banded; sparse records; generic kernel
        with knobs(pair):
            got.append(render_frame_sum(xyz, c, f, H, W, bg, cholesky_bound=bound))
    torch.cuda.synchronize()
    for x in got:
        assert torch.equal(x, ref)
    means = torch.tanh(xyz).cpu().numpy()
    L = (c + bound).cpu().numpy()
    r = oracle.render_sum(means, L, f.cpu().numpy(), np.ones((n, 1), np.float32), H, W)
    want = np.clip(r["out"], 0, 1).transpose(2, 0, 1)
    np.testing.assert_allclose(ref[0].cpu().numpy(), want, rtol=0, atol=1e-5)


def test_id_slab_batched_render_bit_identical(cuda):
    """Batched frames (gsvc_render_frames_sum) over id slabs (A/B knob 25 = 1)
    against the records: every frame's image bit-identical."""
    from gsvc_amd.render import render_frames_sum
    H, W = 270, 480
    sizes = [3000, 0, 5000, 1200]
    parts = [_frame(n, 100 + k, 1.0, cuda) for k, n in enumerate(sizes)]
    xyz = torch.cat([p[0] for p in parts])
    chol = torch.cat([p[1] for p in parts])
    feat = torch.cat([p[2] for p in parts])
    bound = torch.tensor([0.5, 0.0, 0.5], device=cuda)
    bg = torch.ones(3, device=cuda)
    ref = render_frames_sum(xyz, chol, feat, sizes, H, W, bg, cholesky_bound=bound)
    with knobs((25, 1)):
        got = [render_frames_sum(xyz, chol, feat, sizes, H, W, bg, cholesky_bound=bound)
               for _ in range(3)]
    torch.cuda.synchronize()
    for g in got:
        assert torch.equal(g, ref)


@pytest.mark.parametrize("n,chol", [(50000, 3.0), (50000, 1.5)])
def test_render_split_loop_instance_bit_identical(cuda, n, chol):
    """raster_render_ids_kernel's two instances -- the lane-group loop with the
    cut / generic branch inside (frames of <= 8 entries per tile by the density
    hint) and one loop per variant (denser frames) -- give the same bits: the
    first render of a workspace runs with hint 0, later ones with the frame's M
    once the lazy count has read it back."""
    from gsvc_amd import render as R
    H, W = 1080, 1920
    xyz, c, f = _frame(n, 11 + n, chol, cuda)
    bound = torch.tensor([0.5, 0.0, 0.5], device=cuda)
    bg = torch.tensor([0.3, 0.6, 0.9], device=cuda)
    R._workspaces.clear()
    first = R.render_frame_sum(xyz, c, f, H, W, bg, cholesky_bound=bound)
    fw = R._workspaces[(cuda.index, R._raw_stream(cuda.index))]
    assert fw.hint.value == 0  # the first call: the single-loop instance
    ntiles = ((W + 15) // 16) * ((H + 15) // 16)
    for _ in range(64):
        torch.cuda.synchronize()
        last = R.render_frame_sum(xyz, c, f, H, W, bg, cholesky_bound=bound)
        if fw.hint.value > 8 * ntiles:
            break
    assert fw.hint.value > 8 * ntiles, fw.hint.value
    last = R.render_frame_sum(xyz, c, f, H, W, bg, cholesky_bound=bound)  # the split instance
    torch.cuda.synchronize()
    assert torch.equal(first, last)
