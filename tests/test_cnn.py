"""The HDN / JLN 2-D CNNs on the fp32 matrix cores (fvp/cnn.py, csrc/fvp_conv.hip;
SURVEY.md §8(f) rank 1).

Golden vectors: tests/golden/cnn.npz -- the reference's own P2PNet and
CenterNet (lib/models/cnns_2d.py) with seeded weights (fvp.synthetic.
seeded_state_dict; the trained checkpoints are not available offline) on
seeded inputs, run on CPU by tools/gen_golden.py.  tests/cnn_arch.py restates
the architectures (same attribute names) for the GPU box, pinned here.

Tolerance: fp32 everywhere; the MFMA implicit GEMM sums in a different order
than torch's conv and folds BatchNorm into one scale/shift, so outputs agree to
2e-5 of the output's max magnitude (measured ~3e-6).
"""
import numpy as np
import pytest
import torch

from conftest import golden

REL = 2e-5


def _close(got, ref, what):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    scale = max(float(np.abs(ref).max()), 1e-6)
    err = float(np.abs(got - ref).max()) / scale
    assert err <= REL, f"{what}: max error {err:.3g} of the output scale (> {REL})"


def _nets():
    from fvp import synthetic
    import cnn_arch

    p2p = cnn_arch.P2PNet(15, 15).eval()
    p2p.load_state_dict(synthetic.seeded_state_dict(p2p, 11))
    cn = cnn_arch.CenterNet(15, 1).eval()
    cn.load_state_dict(synthetic.seeded_state_dict(cn, 12))
    rng = np.random.default_rng(13)
    x_p2p = rng.uniform(0.0, 1.0, (2, 15, 64, 64)).astype(np.float32)
    x_cn = rng.uniform(0.0, 1.0, (1, 15, 40, 40, 4)).astype(np.float32)
    return p2p, cn, x_p2p, x_cn


def test_restated_architectures_match_reference_golden():
    d = golden("cnn.npz")
    p2p, cn, x_p2p, x_cn = _nets()
    with torch.no_grad():
        _close(p2p(torch.from_numpy(x_p2p)).numpy(), d["y_p2p"], "P2PNet (CPU restatement)")
        hm, size = cn(torch.from_numpy(x_cn))
    _close(hm.numpy(), d["hm"], "CenterNet hm")
    _close(size.numpy(), d["size"], "CenterNet size")


@pytest.mark.gpu
def test_fvp_cnn_matches_reference(gpu_device):
    from fvp.cnn import FvpCNN

    d = golden("cnn.npz")
    p2p, cn, x_p2p, x_cn = _nets()
    p2p, cn = p2p.to(gpu_device), cn.to(gpu_device)
    y = FvpCNN(p2p)(torch.from_numpy(x_p2p).to(gpu_device))
    xy = torch.from_numpy(x_cn).to(gpu_device).max(dim=4)[0]
    hm, size = FvpCNN(cn).from_xy(xy)
    torch.cuda.synchronize()
    _close(y.cpu().numpy(), d["y_p2p"], "P2PNet on MFMA")
    _close(hm.cpu().numpy(), d["hm"], "CenterNet hm on MFMA")
    _close(size.cpu().numpy(), d["size"], "CenterNet size on MFMA")
    with torch.no_grad():  # and against torch's own GPU convolution of the same module
        _close(y.cpu().numpy(), p2p(torch.from_numpy(x_p2p).to(gpu_device)).cpu().numpy(), "P2PNet vs torch GPU")


@pytest.mark.gpu
@pytest.mark.parametrize("n,cin,cout,hw,res", [(2, 256, 256, (16, 30), None), (3, 64, 32, (7, 9), "pre"),
                                               (2, 48, 96, (5, 13), "post"), (1, 32, 64, (1, 1), None),
                                               (40, 64, 64, (8, 12), None)])
def test_wino_deconv_vs_torch(gpu_device, n, cin, cout, hw, res):
    """ConvTranspose2d(4, 2, 1) + BN + ReLU by Winograd F(2x2, 2x2) per output
    parity (fvp_deconv4s2_wino_nhwc, the PoseResNet head's layers): fp32
    tolerance against torch on ragged class-space tile grids, one and several
    K steps, 32- and 64-column blocks, residual before / after the ReLU."""
    import torch.nn as nn

    from fvp import cnn, synthetic

    seq = nn.Sequential(nn.ConvTranspose2d(cin, cout, 4, stride=2, padding=1, bias=False),
                        nn.BatchNorm2d(cout)).eval()
    seq.load_state_dict(synthetic.seeded_state_dict(seq, cin + 5 * cout))
    seq = seq.to(gpu_device)
    g = torch.Generator().manual_seed(cin + n)
    x = (torch.rand((n, cin) + hw, generator=g) - 0.5).to(gpu_device)
    ho = (2 * hw[0], 2 * hw[1])
    r = torch.rand((n, cout) + ho, generator=g).to(gpu_device) if res else None
    with torch.no_grad():
        ref = seq(x)
        ref = torch.relu(ref + r) if res == "pre" else torch.relu(ref) + r if res == "post" else torch.relu(ref)
    layer = cnn.ConvLayer(seq[0], seq[1], algo=cnn.CONV_WINO)
    ra = cnn.to_nhwc(r) if res else None
    got = cnn.to_nchw(layer(cnn.to_nhwc(x), relu=True, res_pre=ra if res == "pre" else None,
                            res_post=ra if res == "post" else None))
    assert [k for _, k in layer._ws.values()] == ["wino_dc"]
    _close(got.cpu().numpy(), ref.cpu().numpy(), f"wino deconv {cin}->{cout} {hw} {res}")


@pytest.mark.gpu
@pytest.mark.parametrize("n,c,cp,hw", [(3, 15, 16, (64, 64)), (2, 1, 16, (80, 80)), (2, 70, 80, (9, 11)),
                                       (1, 128, 128, (5, 3)), (4, 3, 4, (1, 7)), (2, 5, 6, (10, 13))])
def test_nhwc_to_nchw_layouts(gpu_device, n, c, cp, hw):
    """fvp_nhwc_to_nchw (the LDS-tiled kernel for 16-B aligned pitches <= 128, the
    element kernel otherwise, and a channel offset via cnn.to_nchw_from): exactly
    the permuted channels."""
    from fvp import cnn

    t = torch.randn((n,) + hw + (cp,), generator=torch.Generator().manual_seed(c)).to(gpu_device)
    assert torch.equal(cnn.to_nchw(cnn.Act(t, c)), t[..., :c].permute(0, 3, 1, 2))
    if c > 1:
        assert torch.equal(cnn.to_nchw_from(cnn.Act(t, c), 1, c - 1), t[..., 1:c].permute(0, 3, 1, 2))
    if cp % 4 == 0 and cp > 4:
        # c0 % 4 == 0 takes the tiled kernel on an offset pointer: it must read only
        # channels c0 .. c0 + C - 1 (a whole-pitch read runs c0 floats past the end).
        for c0, cc in ((4, cp - 4), (4, min(5, cp - 4))):
            assert torch.equal(cnn.to_nchw_from(cnn.Act(t, cp), c0, cc), t[..., c0:c0 + cc].permute(0, 3, 1, 2))


@pytest.mark.gpu
def test_centernet_merged_heads_match_separate(gpu_device):
    """FvpCNN runs CenterNet's hm and size heads as one 3x3 (32 -> 64) and one
    block-diagonal 1x1 launch (cnn._merged_heads): the same outputs as the two
    heads run separately, to fp32 tolerance, both contiguous NCHW tensors."""
    from fvp import cnn

    _, cn, _, x_cn = _nets()
    cn = cn.to(gpu_device)
    xy = torch.from_numpy(x_cn).to(gpu_device).max(dim=4)[0].repeat(8, 1, 1, 1)
    f = cnn.FvpCNN(cn)
    assert f.heads is not None
    hm, size = f.from_xy(xy)
    f.heads = None
    hm1, size1 = f.from_xy(xy)
    assert hm.is_contiguous() and size.is_contiguous() and hm.shape == hm1.shape and size.shape == size1.shape
    _close(hm.cpu().numpy(), hm1.cpu().numpy(), "merged hm head")
    _close(size.cpu().numpy(), size1.cpu().numpy(), "merged size head")


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,k,hw,res", [(15, 16, 7, (64, 64), False), (16, 32, 3, (33, 17), True),
                                               (128, 128, 3, (16, 16), True), (32, 15, 1, (20, 20), False),
                                               (1, 20, 3, (64, 64), False), (40, 70, 5, (9, 11), True),
                                               (16, 64, 3, (41, 37), True), (64, 16, 5, (23, 30), False)])
def test_conv_layer_vs_torch(gpu_device, conv_kernel, cin, cout, k, hw, res):
    """Single fused conv + BN + residual + ReLU layers, ragged shapes and channel counts."""
    import torch.nn as nn

    from fvp import cnn, synthetic

    conv = nn.Conv2d(cin, cout, k, padding=(k - 1) // 2)
    bn = nn.BatchNorm2d(cout)
    seq = nn.Sequential(conv, bn).eval()
    seq.load_state_dict(synthetic.seeded_state_dict(seq, cin + cout))
    seq = seq.to(gpu_device)
    g = torch.Generator().manual_seed(k)
    x = torch.rand((3, cin) + hw, generator=g).to(gpu_device)
    r = torch.rand((3, cout) + hw, generator=g).to(gpu_device) if res else None
    with torch.no_grad():
        ref = seq(x)
        ref = torch.relu(ref + r) if res else torch.relu(ref)
    layer = cnn.ConvLayer(seq[0], seq[1], algo=conv_kernel)
    got = cnn.to_nchw(layer(cnn.to_nhwc(x), relu=True, res_pre=cnn.to_nhwc(r) if res else None))
    _close(got.cpu().numpy(), ref.cpu().numpy(), f"conv {cin}->{cout} k{k}")


@pytest.mark.gpu
@pytest.mark.parametrize("n,cin,cout,hw,res", [
    (2, 16, 32, (13, 21), None), (2, 48, 64, (9, 30), "pre"), (2, 32, 96, (17, 17), "post"),
    (2, 128, 128, (16, 16), "pre"), (2, 1, 64, (8, 16), None), (2, 64, 64, (2, 3), "post"),
    (3, 128, 128, (20, 20), "pre"), (2, 64, 64, (40, 40), "post"), (70, 32, 64, (30, 34), "pre"),
    (80, 64, 64, (32, 32), None), (40, 64, 64, (32, 32), "post")])
def test_wino_conv_vs_torch(gpu_device, n, cin, cout, hw, res):
    """Winograd F(2x2, 3x3) (fvp_conv3x3_wino_nhwc) on ragged images (partial
    tile grids, images smaller than one tile, the 5 x 5 and 3 x 10 grids of
    20^2 / 40^2 maps), one and several 16-channel K steps, 32- and 64-column
    blocks (Cout padded to 32 / 64), the 8-wave xi-split blocks of small
    launches and the 4-wave blocks of large ones (fvp_conv3x3_wino_plan), BN
    folded, the residual added before or after the ReLU: fp32 tolerance."""
    import torch.nn as nn

    from fvp import cnn, synthetic

    seq = nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1), nn.BatchNorm2d(cout)).eval()
    seq.load_state_dict(synthetic.seeded_state_dict(seq, 3 * cin + cout))
    seq = seq.to(gpu_device)
    g = torch.Generator().manual_seed(cout)
    x = (torch.rand((n, cin) + hw, generator=g) - 0.5).to(gpu_device)
    r = torch.rand((n, cout) + hw, generator=g).to(gpu_device) if res else None
    with torch.no_grad():
        ref = seq(x)
        ref = torch.relu(ref + r) if res == "pre" else torch.relu(ref) + r if res == "post" else torch.relu(ref)
    layer = cnn.ConvLayer(seq[0], seq[1], algo=cnn.CONV_WINO)
    plan = cnn.wino_plan(n, hw[0], hw[1], layer.Cpo)
    if (n, hw) == (70, (30, 34)):
        assert plan[2:4] == (2, 1), plan  # 64-column 4-wave blocks
    if (n, hw) == (80, (32, 32)):
        assert plan[2:4] == (2, 1), plan
    if (n, hw) == (40, (32, 32)):
        assert plan[2:4] == (1, 1), plan  # 32-column 4-wave blocks
    if n <= 3:
        assert plan[3] == 2, plan  # 8-wave xi-split blocks
    ra = cnn.to_nhwc(r) if res else None
    y = layer(cnn.to_nhwc(x), relu=True, res_pre=ra if res == "pre" else None,
              res_post=ra if res == "post" else None, pool=True)
    got = cnn.to_nchw(y)
    assert [k for _, k in layer._ws.values()] == ["wino"]
    _close(got.cpu().numpy(), ref.cpu().numpy(), f"wino conv {cin}->{cout} {hw} {res}")
    # the fused 2 x 2 max pool: exactly max_pool2d of the conv output the same launch wrote
    assert torch.equal(cnn.to_nchw(y.pooled), torch.nn.functional.max_pool2d(got, 2, 2))


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,k,hw,res", [(64, 128, 3, (256, 250), True), (256, 512, 1, (100, 90), False),
                                               (48, 96, 1, (160, 150), True)])
def test_auto_takes_f32_dma_kernel(gpu_device, cin, cout, k, hw, res):
    """AUTO (the product setting) on launches that fill the chip runs the fp32
    LDS-DMA kernel (FVP_CONV_F32_KC, k-paired MFMA order), or Winograd on 3x3
    "same" layers: fp32 tolerance vs torch."""
    import torch.nn as nn

    from fvp import cnn, synthetic

    seq = nn.Sequential(nn.Conv2d(cin, cout, k, padding=(k - 1) // 2), nn.BatchNorm2d(cout)).eval()
    seq.load_state_dict(synthetic.seeded_state_dict(seq, cin * cout))
    seq = seq.to(gpu_device)
    g = torch.Generator().manual_seed(cin)
    x = torch.rand((3, cin) + hw, generator=g).to(gpu_device) - 0.5
    r = torch.rand((3, cout) + hw, generator=g).to(gpu_device) if res else None
    with torch.no_grad():
        ref = seq(x)
        ref = torch.relu(ref + r) if res else torch.relu(ref)
    layer = cnn.ConvLayer(seq[0], seq[1])
    assert layer.algo == cnn.CONV_AUTO == cnn.DEFAULT_ALGO
    got = cnn.to_nchw(layer(cnn.to_nhwc(x), relu=True, res_pre=cnn.to_nhwc(r) if res else None))
    # (3x3 "same" layers: Winograd F(2x2, 3x3) when the product enables it)
    want = "wino" if (k == 3 and cnn.WINO_AUTO and layer._wino_pays(cnn.to_nhwc(x))) else True
    assert any(kind == want for _, kind in layer._ws.values()), f"AUTO did not pick {want}"
    _close(got.cpu().numpy(), ref.cpu().numpy(), f"conv {cin}->{cout} k{k} (AUTO: {want})")


@pytest.mark.gpu
def test_transposed_conv_and_pool_vs_torch(gpu_device):
    import torch.nn as nn
    import torch.nn.functional as F

    from fvp import cnn, synthetic

    up = nn.Sequential(nn.ConvTranspose2d(64, 32, 2, stride=2), nn.BatchNorm2d(32)).eval()
    up.load_state_dict(synthetic.seeded_state_dict(up, 3))
    up = up.to(gpu_device)
    g = torch.Generator().manual_seed(4)
    x = torch.rand((2, 64, 9, 7), generator=g).to(gpu_device)
    skip = torch.rand((2, 32, 18, 14), generator=g).to(gpu_device)
    with torch.no_grad():
        ref = torch.relu(up(x)) + skip
    layer = cnn.ConvLayer(up[0], up[1])
    got = cnn.to_nchw(layer(cnn.to_nhwc(x), relu=True, res_post=cnn.to_nhwc(skip)))
    _close(got.cpu().numpy(), ref.cpu().numpy(), "ConvTranspose2d + BN + ReLU + skip")
    p = torch.rand((2, 48, 10, 12), generator=g).to(gpu_device)
    assert torch.equal(cnn.to_nchw(cnn.maxpool2(cnn.to_nhwc(p))), F.max_pool2d(p, 2, 2))


@pytest.mark.gpu
def test_fvp_cnn_large_batch_tiles_vs_torch(gpu_device, conv_kernel):
    """Enough images that every layer takes the large tiles (>= 2 blocks per CU)."""
    from fvp.cnn import FvpCNN

    p2p, cn, _, _ = _nets()
    p2p = p2p.to(gpu_device)
    x = torch.rand((24, 15, 64, 64), generator=torch.Generator().manual_seed(5)).to(gpu_device)
    with torch.no_grad():
        ref = p2p(x)
    got = FvpCNN(p2p, algo=conv_kernel)(x)
    _close(got.cpu().numpy(), ref.cpu().numpy(), "P2PNet, 24 images")


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,k,hw,up", [(15, 16, 7, (64, 64), False), (32, 32, 3, (33, 17), False),
                                              (128, 128, 3, (16, 16), False), (64, 32, 2, (9, 7), True)])
def test_bf16_conv_layer_vs_torch(gpu_device, cin, cout, k, hw, up):
    """Opt-in bf16 operands (fp32 accumulation): within 2e-2 of the output scale
    of torch's fp32 convolution (bf16 keeps 8 mantissa bits)."""
    import torch.nn as nn

    from fvp import cnn, synthetic

    conv = nn.ConvTranspose2d(cin, cout, 2, stride=2) if up else nn.Conv2d(cin, cout, k, padding=(k - 1) // 2)
    seq = nn.Sequential(conv, nn.BatchNorm2d(cout)).eval()
    seq.load_state_dict(synthetic.seeded_state_dict(seq, cin * 7 + cout))
    seq = seq.to(gpu_device)
    x = torch.rand((3, cin) + hw, generator=torch.Generator().manual_seed(k)).to(gpu_device)
    with torch.no_grad():
        ref = torch.relu(seq(x))
    layer = cnn.ConvLayer(seq[0], seq[1], torch.bfloat16)
    got = cnn.to_nchw(layer(cnn.to_nhwc(x), relu=True))
    err = float((got - ref).abs().max()) / float(ref.abs().max())
    assert err <= 2e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cpi,k,stride,hw", [(3, 4, 7, 2, (67, 45)), (3, 8, 3, 1, (20, 33)),
                                                 (10, 12, 5, 2, (31, 30)), (4, 4, 1, 1, (9, 9))])
def test_bf16_small_channel_conv_vs_torch(gpu_device, cin, cpi, k, stride, hw):
    """bf16 operands on a 4 / 8 / 12-channel fp32 input (the RGB stem,
    resnet.py:105-107): one K chunk spans several taps; within 2e-2 of the
    output scale of torch's fp32 convolution."""
    import torch.nn as nn

    from fvp import cnn, synthetic

    seq = nn.Sequential(nn.Conv2d(cin, 64, k, stride=stride, padding=k // 2, bias=False), nn.BatchNorm2d(64)).eval()
    seq.load_state_dict(synthetic.seeded_state_dict(seq, cin * 11 + k))
    seq = seq.to(gpu_device)
    x = torch.rand((2, cin) + hw, generator=torch.Generator().manual_seed(k)).to(gpu_device)
    with torch.no_grad():
        ref = torch.relu(seq(x))
    layer = cnn.ConvLayer(seq[0], seq[1], torch.bfloat16, cpi=cpi)
    assert layer.bf16
    got = cnn.to_nchw(layer(cnn.to_nhwc(x, cpi), relu=True))
    err = float((got - ref).abs().max()) / float(ref.abs().max())
    assert err <= 2e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,k,stride,hw,deconv,res", [(64, 64, 3, 1, (33, 47), False, False),
                                                             (128, 256, 3, 2, (30, 17), False, True),
                                                             (256, 64, 1, 1, (20, 21), False, True),
                                                             (64, 512, 1, 2, (19, 23), False, False),
                                                             (256, 128, 4, 2, (9, 11), True, False),
                                                             (192, 96, 3, 1, (7, 130), False, False),
                                                             (32, 64, 3, 1, (64, 64), False, True),
                                                             (96, 32, 3, 2, (21, 19), False, False),
                                                             (32, 32, 1, 1, (17, 40), False, True),
                                                             (64, 16, 3, 1, (33, 29), False, True),
                                                             (256, 15, 1, 1, (20, 21), False, False)])
def test_bf16_dma_conv_matches_register_staged(gpu_device, cin, cout, k, stride, hw, deconv, res):
    """bf16 activations with Cpi % 32 == 0 run the LDS-DMA kernel
    (conv_dma_kernel, 64- or 32-deep K steps); CONV_PER_TAP_NOSPLIT keeps such layers on the
    register-staged conv_bf16_kernel.  Both walk k in the same order with the
    same MFMA instruction, so the outputs are bit-identical; and within 2e-2 of
    the output scale of torch's fp32 convolution of the bf16-rounded input."""
    import torch.nn as nn

    from fvp import cnn, synthetic

    conv = (nn.ConvTranspose2d(cin, cout, 4, stride=2, padding=1) if deconv
            else nn.Conv2d(cin, cout, k, stride=stride, padding=k // 2, bias=False))
    seq = nn.Sequential(conv, nn.BatchNorm2d(cout)).eval()
    seq.load_state_dict(synthetic.seeded_state_dict(seq, cin + 3 * cout + k))
    seq = seq.to(gpu_device)
    gen = torch.Generator().manual_seed(cin + k)
    x = torch.rand((3, cin) + hw, generator=gen).to(gpu_device).to(torch.bfloat16).float()
    layer = cnn.ConvLayer(seq[0], seq[1], torch.bfloat16)
    layer.act_bf16 = True
    xn = cnn.to_nhwc(x)
    xa = cnn.Act(xn.t.to(torch.bfloat16), xn.C)
    Ho, Wo = layer.out_hw(*hw)
    r = None
    if res:
        rt = torch.zeros((3, Ho, Wo, layer.Cpo), dtype=torch.bfloat16, device=gpu_device)
        rt[..., :cout] = torch.randn((3, Ho, Wo, cout), generator=gen).to(gpu_device).to(torch.bfloat16)
        r = cnn.Act(rt, cout)
    y_dma = layer(xa, relu=True, res_post=r)
    reg = cnn.ConvLayer(seq[0], seq[1], torch.bfloat16, algo=cnn.CONV_PER_TAP_NOSPLIT)
    reg.act_bf16 = True
    y_reg = reg(xa, relu=True, res_post=r)
    assert torch.equal(y_dma.t, y_reg.t)
    with torch.no_grad():
        ref = torch.relu(seq(x))
        if res:
            ref = ref + r.t[..., :cout].float().permute(0, 3, 1, 2)
    got = y_dma.t[..., :cout].float().permute(0, 3, 1, 2)
    err = float((got - ref).abs().max()) / float(ref.abs().max())
    assert err <= 2e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("cin,hw", [(15, (64, 64)), (15, (37, 50)), (3, (80, 80)), (16, (9, 70))])
def test_bf16_front7_vs_torch(gpu_device, cin, hw):
    """fvp_conv_front7_bf16 (the bf16 nets' Basic2DBlock(J, 16, 7) from the NCHW
    maps): within 2e-2 of the output scale of torch's fp32 Basic2DBlock on the
    bf16-rounded input, ragged tiles included."""
    import cnn_arch
    from fvp import cnn, synthetic

    p2p = cnn_arch.P2PNet(cin, 15).eval()
    p2p.load_state_dict(synthetic.seeded_state_dict(p2p, 40 + cin))
    p2p = p2p.to(gpu_device)
    f = cnn.FvpCNN(p2p, torch.bfloat16)
    assert f.front7 is not None
    x = torch.rand((3, cin) + hw, generator=torch.Generator().manual_seed(cin)).to(gpu_device)
    x = x.to(torch.bfloat16).float()
    fn, wp, c = f.front7
    assert fn == "fvp_conv_front7_bf16"
    out = torch.empty((3,) + hw + (16,), dtype=torch.bfloat16, device=gpu_device)
    from fvp import _lib
    from fvp.ops import _ptr, _stream

    _lib.call("fvp_conv_front7_bf16", _ptr(x), 3, cin, hw[0], hw[1], _ptr(wp), _ptr(c.scale), _ptr(c.shift),
              _ptr(out), _stream(out))
    with torch.no_grad():
        ref = p2p.front_layers[0](x)
    got = out.float().permute(0, 3, 1, 2)
    err = float((got - ref).abs().max()) / float(ref.abs().max())
    assert err <= 2e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("n,cin,hw", [(3, 15, (64, 64)), (2, 15, (37, 50)), (8, 3, (80, 80)), (2, 16, (9, 70)),
                                      (3, 1, (5, 3)), (80, 15, (64, 64))])
def test_f32_front7_vs_torch(gpu_device, n, cin, hw):
    """fvp_conv_front7_f32 (the fp32 nets' Basic2DBlock(J, 16, 7) from the NCHW
    maps, AUTO's front layer): fp32 tolerance against torch's Basic2DBlock,
    ragged 8 x 16 tiles, images smaller than a tile, fewer than 16 planes and a
    launch whose persistent blocks walk several tiles each (80 x 64^2: 2,560
    tiles)."""
    import cnn_arch
    from fvp import _lib, cnn, synthetic
    from fvp.ops import _ptr, _stream

    p2p = cnn_arch.P2PNet(cin, 15).eval()
    p2p.load_state_dict(synthetic.seeded_state_dict(p2p, 50 + cin))
    p2p = p2p.to(gpu_device)
    f = cnn.FvpCNN(p2p)
    fn, wp, c = f.front7
    assert fn == "fvp_conv_front7_f32"
    x = torch.rand((n, cin) + hw, generator=torch.Generator().manual_seed(cin + n)).to(gpu_device)
    out = torch.empty((n,) + hw + (16,), device=gpu_device)
    _lib.call(fn, _ptr(x), n, cin, hw[0], hw[1], _ptr(wp), _ptr(c.scale), _ptr(c.shift), _ptr(out), _stream(out))
    with torch.no_grad():
        ref = p2p.front_layers[0](x)
    _close(out.permute(0, 3, 1, 2).cpu().numpy(), ref.cpu().numpy(), f"front7 f32 {n} {cin} {hw}")


@pytest.mark.gpu
def test_bf16_p2pnet_vs_reference(gpu_device):
    """Whole P2PNet with bf16 operands against the reference's fp32 golden:
    within 5e-2 of the output scale (errors compound over 20 convolutions)."""
    from fvp.cnn import FvpCNN

    d = golden("cnn.npz")
    p2p, _, x_p2p, _ = _nets()
    y = FvpCNN(p2p.to(gpu_device), torch.bfloat16)(torch.from_numpy(x_p2p).to(gpu_device))
    err = float(np.abs(y.cpu().numpy() - d["y_p2p"]).max()) / float(np.abs(d["y_p2p"]).max())
    assert err <= 5e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,hw", [(32, 15, (64, 64)), (15, 1, (9, 13)), (50, 64, (5, 7)), (16, 33, (3, 3))])
def test_head_1x1_writes_nchw_vs_torch(gpu_device, cin, cout, hw):
    """fvp_conv1x1_nchw (P2PNet's output layer straight into NCHW, FvpCNN._head_nchw)
    against torch's conv2d of the same weights, and the GEMM + layout-pass path."""
    import torch.nn as nn

    from fvp import cnn, synthetic

    conv = nn.Conv2d(cin, cout, 1).eval()
    conv.load_state_dict(synthetic.seeded_state_dict(conv, cin + cout))
    conv = conv.to(gpu_device)
    x = torch.rand((3, cin) + hw, generator=torch.Generator().manual_seed(cout)).to(gpu_device)
    with torch.no_grad():
        ref = conv(x)
    layer = cnn.ConvLayer(conv, None)
    a = cnn.to_nhwc(x, layer.Cpi)
    f = cnn.FvpCNN.__new__(cnn.FvpCNN)
    f.out = layer
    got = f._head_nchw(a)
    gemm = cnn.to_nchw(layer(a, relu=False))
    torch.cuda.synchronize()
    _close(got.cpu().numpy(), ref.cpu().numpy(), f"1x1 head {cin}->{cout}")
    _close(got.cpu().numpy(), gemm.cpu().numpy(), f"1x1 head vs GEMM {cin}->{cout}")


@pytest.mark.gpu
def test_graphed_centernet_equals_eager(gpu_device):
    """CenterNet replayed from a hipGraph per batch shape (GraphedCNN.from_xy,
    FvpOptions.center_graphs): bit-identical to the eager launches, new inputs
    copied in, both outputs cloned out (not aliased across calls)."""
    from fvp import cnn

    _, cn, _, _ = _nets()
    cn = cn.to(gpu_device)
    eager = cnn.FvpCNN(cn)
    g = cnn.GraphedCNN(cnn.FvpCNN(cn))
    gen = torch.Generator().manual_seed(9)
    outs = []
    for b in (8, 8, 3, 8):
        xy = torch.rand((b, 15, 80, 80), generator=gen).to(gpu_device)
        outs.append((g.from_xy(xy), eager.from_xy(xy)))
    torch.cuda.synchronize()
    for (gh, gs), (eh, es) in outs:
        assert torch.equal(gh, eh) and torch.equal(gs, es)
    assert len(g._graphs) == 2 and g.eager_calls == 0


@pytest.mark.gpu
@pytest.mark.parametrize("n,cin,cout,h,w,j", [(3, 64, 32, 32, 32, 15), (2, 48, 20, 3, 64, 16), (1, 128, 32, 2, 32, 1)])
def test_p2p_tail_one_launch_vs_torch(gpu_device, n, cin, cout, h, w, j):
    """fvp_up2_head_nchw (FvpCNN._tail_nchw): P2PNet's last Upsample2DBlock + skip_x1 +
    output layer in one launch, against torch's modules of the same weights, and
    against the two-launch path (the deconvolution GEMM, then fvp_conv1x1_nchw)."""
    import types

    import torch.nn as nn

    import cnn_arch
    from fvp import cnn, synthetic

    up = cnn_arch.Upsample2DBlock(cin, cout, 2, 2).eval()
    head = nn.Conv2d(cout, j, 1).eval()
    for m, seed in ((up, cin), (head, j)):
        m.load_state_dict(synthetic.seeded_state_dict(m, seed))
    with torch.no_grad():  # non-trivial BN statistics
        bn = up.block[1]
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 1.5)
    up, head = up.to(gpu_device), head.to(gpu_device)
    g = torch.Generator().manual_seed(n * 7 + cin)
    x = (torch.rand((n, cin, h, w), generator=g) - 0.3).to(gpu_device)
    skip = torch.rand((n, cout, 2 * h, 2 * w), generator=g).to(gpu_device)
    with torch.no_grad():
        ref = head(up(x) + skip)
    f = cnn.FvpCNN.__new__(cnn.FvpCNN)
    f.module = types.SimpleNamespace(encoder_decoder=types.SimpleNamespace(decoder_upsample1=up), output_layer=head)
    f.encdec = types.SimpleNamespace(parts={"decoder_upsample1": cnn._Plan(up)})
    f.out = cnn.ConvLayer(head, None)
    f.tail = f._compile_tail()
    assert f.tail is not None
    c = f.tail[1]
    xa, sa = cnn.to_nhwc(x, c.Cpi), cnn.to_nhwc(skip, 32)
    got = f._tail_nchw(xa, sa)
    assert got is not None and got.shape == (n, j, 2 * h, 2 * w)
    two = f._head_nchw(f.encdec.parts["decoder_upsample1"](xa, res_post=sa))
    torch.cuda.synchronize()
    _close(got.cpu().numpy(), ref.cpu().numpy(), f"up2 + head {cin}->{cout}->{j}")
    _close(got.cpu().numpy(), two.cpu().numpy(), f"up2 + head vs two launches {cin}->{cout}->{j}")
    # the whole P2PNet takes this path (64^2 planes: 32-pixel rows into the last upsample)
    p2p = cnn_arch.P2PNet(15, 15).eval().to(gpu_device)
    assert cnn.FvpCNN(p2p).tail is not None
