"""The C++ autograd Functions of the drop-in operators (csrc/torch_ops.cpp):
what GSVC's unchanged files run.  They must be the Python Functions'
(project_gaussians_2d.py / rasterize_sum.py, ctypes over the same C ABI) bit
for bit in the forward and in the projection backward, and within the float
atomics' summation order in the rasterizer backward; the general cases keep
the Python Functions.  Reference: project_gaussians_2d.py:59-141,
rasterize_sum.py:89-254."""
import numpy as np
import pytest
import torch

from conftest import knobs


def test_cpu_tensors_raise():
    """No CPU path (CPU suite: the argument check precedes any HIP call)."""
    from gsvc_amd import _lib
    ext = _lib.torch_ops()
    x = torch.zeros(4, 2)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        ext.project_gaussians_2d(x, torch.zeros(4, 3), 16, 16, 1, 1, 1, 0.01)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        ext.rasterize_sum(x, torch.zeros(4, dtype=torch.int32), torch.zeros(4, 3), torch.zeros(4, 3),
                          torch.ones(4, 1), torch.ones(3), 16, 16)


def _inputs(n, H, W, seed, dev, chol=1.0):
    g = torch.Generator().manual_seed(seed)
    means = (2 * torch.rand(n, 2, generator=g) - 1).to(dev)
    L = (torch.rand(n, 3, generator=g) * chol + torch.tensor([0.5, 0, 0.5]) * chol).to(dev)
    col = torch.rand(n, 3, generator=g).to(dev)
    return means, L, col


def _run(means, L, col, H, W, python_path, v_out):
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    m = means.clone().requires_grad_(True)
    l = L.clone().requires_grad_(True)
    c = col.clone().requires_grad_(True)
    o = torch.ones(m.shape[0], 1, device=m.device)
    tb = ((W + 15) // 16, (H + 15) // 16, 1)

    def go():
        xys, depths, radii, conics, nth = project_gaussians_2d(m, l, H, W, tb)
        out = rasterize_gaussians_sum(xys, depths, radii, conics, nth, c, o, H, W, 16, 16,
                                      background=torch.ones(3, device=m.device))
        (out * v_out).sum().backward()
        return out, xys, radii, conics, nth

    if python_path:
        with knobs((0, 1)):  # the diagnostic library: the Python Functions over ctypes
            res = go()
    else:
        res = go()
    torch.cuda.synchronize()
    return [r.detach() for r in res], (m.grad, l.grad, c.grad)


@pytest.mark.gpu
@pytest.mark.parametrize("n,H,W,chol", [(1000, 256, 256, 1.0), (300, 37, 53, 1.0),
                                        (50000, 1080, 1920, 1.0), (20000, 1080, 1920, 6.0)])
def test_cpp_functions_match_python_functions(cuda, n, H, W, chol):
    means, L, col = _inputs(n, H, W, n + H, cuda, chol)
    v_out = torch.randn(H, W, 3, generator=torch.Generator().manual_seed(3)).to(cuda)
    fast, gf = _run(means, L, col, H, W, False, v_out)
    ref, gr = _run(means, L, col, H, W, True, v_out)
    for a, b in zip(fast, ref):
        assert torch.equal(a, b)
    for a, b in zip(gf, gr):
        scale = float(b.abs().max())
        assert float((a - b).abs().max()) <= 1e-5 * max(scale, 1e-30)


def _gsvc_epilogue(out, H, W):
    """GaussianSplats_Represent.py:88-89 as written."""
    return torch.clamp(out, 0, 1).view(-1, H, W, 3).permute(0, 3, 1, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("n,H,W", [(4000, 256, 320), (300, 37, 53), (50000, 1080, 1920)])
def test_cpp_function_planar_output(cuda, monkeypatch, n, H, W):
    """GSVC_SLABS_PLANES (the default): the image as channel planes, strides
    (W, 1, H*W) -- the same values bit for bit as the contiguous [H, W, 3]
    route (GSVC_OP_PLANAR=0), GSVC's clamp + view + permute already contiguous
    (its .contiguous() copies nothing), the M < 1 background in the same
    layout, and the gradients through GSVC's epilogue and L2 loss equal within
    the float atomics' order."""
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    means, L, col = _inputs(n, H, W, 7 + n, cuda)
    gt = torch.rand(1, 3, H, W, generator=torch.Generator().manual_seed(5)).to(cuda)
    tb = ((W + 15) // 16, (H + 15) // 16, 1)

    def go(planar, shift=0.0):
        monkeypatch.setenv("GSVC_OP_PLANAR", "1" if planar else "0")
        m = (means + shift).clone().requires_grad_(True)
        l = L.clone().requires_grad_(True)
        c = col.clone().requires_grad_(True)
        o = torch.ones(n, 1, device=cuda)
        xys, depths, radii, conics, nth = project_gaussians_2d(m, l, H, W, tb)
        out = rasterize_gaussians_sum(xys, depths, radii, conics, nth, c, o, H, W, 16, 16,
                                      background=torch.tensor([0.2, 0.5, 0.7], device=cuda))
        img = _gsvc_epilogue(out, H, W)
        contiguous_already = img.is_contiguous()
        img = img.contiguous()
        torch.nn.functional.mse_loss(img, gt).backward()
        torch.cuda.synchronize()
        return out.detach(), contiguous_already, (m.grad, l.grad, c.grad)

    hwc, c0, g0 = go(False)
    pl, c1, g1 = go(True)
    assert hwc.is_contiguous() and not c0
    assert pl.shape == (H, W, 3) and pl.stride() == (W, 1, H * W) and c1
    assert torch.equal(pl, hwc)
    for a, b in zip(g1, g0):
        scale = float(b.abs().max())
        assert float((a - b).abs().max()) <= 1e-5 * max(scale, 1e-30)
    # every splat off-screen: M = 0, the background in both layouts
    bg_h, _, _ = go(False, shift=50.0)
    bg_p, _, _ = go(True, shift=50.0)
    assert torch.equal(bg_p, bg_h)
    assert torch.equal(bg_p[0, 0], torch.tensor([0.2, 0.5, 0.7], device=cuda))


@pytest.mark.gpu
def test_cpp_function_return_alpha_and_background(cuda):
    """return_alpha (1 - final_Ts: 0 with intersections) and the M < 1 branch
    (every splat off-screen: the background, alpha 1 - 0 = 1)."""
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    H, W = 64, 80
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    means, L, col = _inputs(200, H, W, 5, cuda)
    bg = torch.tensor([0.2, 0.4, 0.6], device=cuda)
    for shift, alpha in ((0.0, 0.0), (50.0, 1.0)):
        xys, depths, radii, conics, nth = project_gaussians_2d(means + shift, L, H, W, tb)
        out, a = rasterize_gaussians_sum(xys, depths, radii, conics, nth, col,
                                         torch.ones(200, 1, device=cuda), H, W, background=bg,
                                         return_alpha=True)
        assert a.shape == (H, W) and torch.all(a == alpha)
        if shift:
            assert torch.equal(out, bg.expand(H, W, 3))


@pytest.mark.gpu
def test_unchanged_caller_train_step_matches_fused(cuda):
    """GaussianVideoFrame with fused_train / fused_render off (GSVC's own op
    sequence over the C++ Functions) takes the same steps as the fused model:
    PSNR per iteration within float-atomics reassociation."""
    from gsvc_amd.frame import make_frame_model, synthetic_gt
    H, W = 128, 192
    gt = synthetic_gt(H, W, 2, cuda)
    a = make_frame_model(H, W, 3000, cuda, seed=7)
    b = make_frame_model(H, W, 3000, cuda, seed=7, fused_train=False, fused_render=False)
    pa = [a.train_iter(gt, it)[1] for it in range(1, 21)]
    pb = [b.train_iter(gt, it)[1] for it in range(1, 21)]
    assert a.fused_steps == 20 and b.fused_steps == 0
    assert np.allclose(pa, pb, rtol=0, atol=2e-3), (pa, pb)
    with torch.no_grad():
        ra, rb = a()["render"], b()["render"]
    assert float((ra - rb).abs().max()) < 1e-3


@pytest.mark.gpu
def test_cpp_functions_partial_gradients(cuda):
    """Gradient materialisation is off in both C++ Functions (no zero-fill
    launches for depths / radii / num_tiles_hit / M): a loss on xys alone, on
    conics alone, or on depths, takes the undefined-gradient branches and
    gives the Python Functions' gradients."""
    from gsplat.project_gaussians_2d import project_gaussians_2d
    H, W = 64, 96
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    means, L, _ = _inputs(500, H, W, 11, cuda)
    w_xy = torch.randn(500, 2, generator=torch.Generator().manual_seed(1)).to(cuda)
    w_c = torch.randn(500, 3, generator=torch.Generator().manual_seed(2)).to(cuda)

    def grads(python_path, which):
        m = means.clone().requires_grad_(True)
        l = L.clone().requires_grad_(True)

        def go():
            xys, depths, radii, conics, nth = project_gaussians_2d(m, l, H, W, tb)
            loss = {"xys": (xys * w_xy).sum(), "conics": (conics * w_c).sum(),
                    "depths": depths.sum() + (xys * w_xy).sum()}[which]
            loss.backward()
        if python_path:
            with knobs((0, 1)):
                go()
        else:
            go()
        torch.cuda.synchronize()
        return m.grad, l.grad

    for which in ("xys", "conics", "depths"):
        for a, b in zip(grads(False, which), grads(True, which)):
            assert a is not None and b is not None
            assert torch.equal(a, b), which


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["planes", "expanded", "transposed"])
def test_cpp_rasterize_backward_takes_strided_gradients(cuda, layout):
    """The rasterizer backward reads the output gradient at its own strides
    (channel planes after GSVC's permute, a broadcast, a transpose) with no
    .contiguous() copy: the gradients equal those of the contiguous gradient
    (within the float atomics' summation order)."""
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    H, W = 72, 104
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    means, L, col = _inputs(800, H, W, 21, cuda)
    g = torch.Generator().manual_seed(4)
    if layout == "planes":
        v = torch.randn(3, H, W, generator=g).to(cuda).permute(1, 2, 0)
    elif layout == "expanded":
        v = torch.randn(3, generator=g).to(cuda).expand(H, W, 3)
    else:
        v = torch.randn(W, H, 3, generator=g).to(cuda).transpose(0, 1)
    assert not v.is_contiguous()

    def grads(v_out):
        m = means.clone().requires_grad_(True)
        l = L.clone().requires_grad_(True)
        c = col.clone().requires_grad_(True)
        xys, depths, radii, conics, nth = project_gaussians_2d(m, l, H, W, tb)
        out = rasterize_gaussians_sum(xys, depths, radii, conics, nth, c,
                                      torch.ones(800, 1, device=cuda), H, W,
                                      background=torch.ones(3, device=cuda))
        out.backward(v_out)
        torch.cuda.synchronize()
        return m.grad, l.grad, c.grad

    for a, b in zip(grads(v), grads(v.contiguous())):
        assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max())


@pytest.mark.gpu
def test_cpp_functions_splat_order_bit_identical(cuda):
    """The op path inserts ids in a splat order sorted by an earlier call
    (GSVC_TRAIN_ORDER / _REFRESH, speed only): the first call (no order yet),
    the ordered calls after it and the refresh 64 calls later all give the
    Python Functions' image and final_idx bit for bit, and the same gradients
    within the atomics' order."""
    from gsplat.project_gaussians_2d import project_gaussians_2d
    from gsplat.rasterize_sum import rasterize_gaussians_sum
    H, W = 360, 640
    n = 7777  # a count no other test uses: this call starts without an order
    means, L, col = _inputs(n, H, W, 5, cuda, 2.0)
    v_out = torch.randn(H, W, 3, generator=torch.Generator().manual_seed(9)).to(cuda)
    ref, gr = _run(means, L, col, H, W, True, v_out)
    tb = ((W + 15) // 16, (H + 15) // 16, 1)
    o = torch.ones(n, 1, device=cuda)
    for call in range(70):
        if call in (0, 1, 2, 63, 64, 65, 69):
            fast, gf = _run(means, L, col, H, W, False, v_out)
            assert torch.equal(fast[0], ref[0]), call
            for a, b in zip(gf, gr):
                assert float((a - b).abs().max()) <= 1e-5 * max(float(b.abs().max()), 1e-30)
        else:
            with torch.no_grad():
                xys, depths, radii, conics, nth = project_gaussians_2d(means, L, H, W, tb)
                rasterize_gaussians_sum(xys, depths, radii, conics, nth, col, o, H, W, 16, 16,
                                        background=torch.ones(3, device=cuda))


@pytest.mark.gpu
@pytest.mark.parametrize("n,chol", [(9000, 0.4), (24000, 0.4), (60000, 0.4)])
def test_cpp_function_banded_id_slabs(cuda, n, chol):
    """A dense frame (> 96 entries per tile on average): once the lazy M hint
    has seen it, the C++ Function's composite takes the banded kernel over the
    id slabs -- two waves per tile, ONE id sort per tile shared through LDS
    and written back for the backward (both waves used to sort from
    the slots wave 0 rewrites).  Every call (the first sparse, the rest
    banded) equals the Python Function (counted binning) bit for bit in the
    image, and its gradients within the atomics' order; 24k splats on 64 tiles
    pass 256 entries per tile (sorted from the wide id slabs, GSVC_SLABS_WIDE:
    1024 ids per tile), 60k pass 1024 (the bbox rebuild)."""
    H = W = 128
    means, L, col = _inputs(n, H, W, 77 + n, cuda, chol)
    v_out = torch.randn(H, W, 3, generator=torch.Generator().manual_seed(5)).to(cuda)
    ref, gr = _run(means, L, col, H, W, True, v_out)
    m = int(ref[4].sum())  # num_tiles_hit: M
    assert m > 96 * 64
    for _ in range(6):
        fast, gf = _run(means, L, col, H, W, False, v_out)
        for a, b in zip(fast, ref):
            assert torch.equal(a, b)
        for a, b in zip(gf, gr):
            assert float((a - b).abs().max()) <= 1e-5 * max(float(b.abs().max()), 1e-30)
