"""The PoseResNet heatmap backbone on the fvp MFMA convolutions and the
channels-last voxelize that reads its output in place (fvp/backbone.py,
csrc/fvp_conv.hip modes 0/3, fvp_voxelize_cl; SURVEY.md §8(f) rank 4,
lib/models/resnet.py:98-215, faster_voxelpose.py:73-75).

Golden vectors: tests/golden/backbone.npz -- the reference's own ResNet built by
its resnet.get (ResNet-50 with the default deconvolution head and 1x1 final
conv; ResNet-18 with a 3x3 final conv on a 70x90 image, so every stride-2
stage sees odd sizes) with seeded weights (fvp.synthetic.seeded_state_dict; the
pretrained backbone is not available offline) on seeded images, run on CPU by
tools/gen_golden.py.  tests/cnn_arch.PoseResNet restates the architecture
with the same attribute names for the GPU box and is pinned here bit-exactly.

Tolerance: fp32 MFMA implicit GEMMs sum in a different order than torch's CPU
convolutions and fold BatchNorm into one scale/shift; through 50+ layers the
heatmaps agree to REL = 1e-4 of their max magnitude (the error is reported).
The voxelize on channels-last heatmaps is compared bit-exactly with the planar
path (same values, same arithmetic).
"""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from conftest import golden

REL = 1e-4


def _rel_err(got, ref):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    return float(np.abs(got - ref).max()) / max(float(np.abs(ref).max()), 1e-6)


def _net(tag):
    from fvp import synthetic
    import cnn_arch

    d = golden("backbone.npz")
    layers, J, fk, seed = (int(v) for v in d[f"{tag}_cfg"])
    m = cnn_arch.PoseResNet(layers, J, final_kernel=fk).eval()
    m.load_state_dict(synthetic.seeded_state_dict(m, seed))
    return m, d[f"{tag}_images"], d[f"{tag}_heatmaps"]


@pytest.mark.parametrize("tag", ["r50", "r18"])
def test_restated_pose_resnet_matches_reference_golden(tag):
    m, x, y = _net(tag)
    with torch.no_grad():
        got = m(torch.from_numpy(x)).numpy()
    assert got.shape == y.shape
    assert _rel_err(got, y) <= 1e-6, tag


def test_conv_geometry_host():
    """Output sizes follow torch's floor formula; bad geometries are rejected before any launch."""
    import ctypes

    from fvp import _lib

    lib = _lib.load()
    hw = (ctypes.c_int * 2)()
    assert lib.fvp_conv2d_geom(512, 960, 4, 7, 7, 0, 2, 2, 3, 3, hw) == 0 and list(hw) == [256, 480]
    assert lib.fvp_conv2d_geom(35, 45, 64, 3, 3, 0, 2, 2, 1, 1, hw) == 0 and list(hw) == [18, 23]
    assert lib.fvp_conv2d_geom(15, 30, 2048, 2, 2, 3, 0, 0, 0, 0, hw) == 0 and list(hw) == [30, 60]
    assert lib.fvp_conv2d_geom(8, 8, 20, 3, 3, 0, 1, 1, 1, 1, hw) == 1002       # Cpi 20: not 4/8/12 or 16k
    assert lib.fvp_conv2d_geom(8, 8, 16, 3, 3, 0, 1, 1, 3, 1, hw) == 1002       # padding >= kernel
    assert lib.fvp_conv2d_geom(8, 8, 16, 3, 3, 3, 1, 1, 1, 1, hw) == 1002       # mode 3 needs 2x2 taps
    assert lib.fvp_conv2d_geom(2, 2, 16, 7, 7, 0, 1, 1, 0, 0, hw) == 1002       # kernel larger than the input
    assert lib.fvp_maxpool_pad_nhwc(1, 1, 8, 8, 16, 3, 2, 2, 1, None) == 1002  # 2P > K
    # bf16 entry points: argument checks before any launch
    assert lib.fvp_maxpool_pad_nhwc_bf16(1, 1, 8, 8, 12, 3, 2, 1, 1, None) == 1002  # C % 8
    assert lib.fvp_maxpool_pad_nhwc_bf16(None, 1, 8, 8, 16, 3, 2, 1, 1, None) == 1001
    assert lib.fvp_maxpool_nhwc_bf16(1, 1, 8, 8, 12, 2, 2, 1, None) == 1002         # C % 8
    assert lib.fvp_maxpool_nhwc_bf16(1, 1, 8, 8, 16, 3, 2, 1, None) == 1002         # KH > 2
    assert lib.fvp_conv_stem7_bf16(1, 1, 5, 64, 64, 1, 1, 1, 1, None) == 1002      # > 4 input channels
    assert lib.fvp_conv_stem7_bf16(1, 0, 3, 64, 64, 1, 1, 1, 1, None) == 1002      # N = 0
    assert lib.fvp_conv_stem7_bf16(None, 1, 3, 64, 64, 1, 1, 1, 1, None) == 1001
    assert lib.fvp_conv_stem7_f32(16, 1, 4, 64, 64, 16, 16, 16, 16, None) == 1002   # > 3 input channels (fp32)
    assert lib.fvp_conv_stem7_f32(16, 1, 3, 64, 64, 16, 16, 16, 20, None) == 1002   # out not 16-B aligned
    assert lib.fvp_conv_stem7_f32(None, 1, 3, 64, 64, 16, 16, 16, 16, None) == 1001
    assert lib.fvp_conv_front7_bf16(1, 1, 17, 64, 64, 1, 1, 1, 1, None) == 1002     # > 16 input planes
    assert lib.fvp_conv_front7_bf16(None, 1, 15, 64, 64, 1, 1, 1, 1, None) == 1001
    assert lib.fvp_conv_front7_f32(1, 1, 17, 64, 64, 1, 1, 1, 1, None) == 1002
    assert lib.fvp_conv_front7_f32(None, 1, 15, 64, 64, 1, 1, 1, 1, None) == 1001
    # the one-launch 1-D net: NULLs, a slot too small for the input, an lg it has no kernel for
    assert lib.fvp_conv1d_net(None, 80, 15, 20, 1, 25, 1, 1424, 6, 12288, 0, 1, 20, 4, 1, None) == 1001
    assert lib.fvp_conv1d_net(1, 80, 15, 20, 1, 25, 1, 100, 6, 12288, 0, 1, 20, 4, 1, None) == 1002
    assert lib.fvp_conv1d_net(1, 80, 15, 20, 1, 25, 1, 1424, 6, 12288, 0, 1, 20, 3, 1, None) == 1002
    assert lib.fvp_conv1d_net(1, 80, 15, 20, 1, 25, 1, 1424, 6, 12288, 6, 1, 20, 4, 1, None) == 1002
    assert lib.fvp_conv1d_net(1, 80, 15, 20, 1, 25, 1, 1424, 6, 6000, 0, 1, 20, 4, 1, None) == 1002   # chunk % 4096
    assert lib.fvp_conv1d_net(1, 80, 15, 20, 1, 25, 1, 1424, 6, 16384, 0, 1, 20, 4, 1, None) == 1002  # > 3 stages
    assert lib.fvp_conv1d_net_lds_bytes(2832, 6, 8192, 4) == (2 * 8192 + 4096 + 2832 * 6) * 4
    # the 1x1 head writing NCHW: NULLs, Cout > 64, a pitch too small for the float4s read, misalignment
    head = lambda p, cpi, cin, cout: lib.fvp_conv1x1_nchw(p, 1, 8, 8, cpi, cin, 16, cout, cout, 16, 16, 0, 16, None)
    assert head(None, 16, 16, 15) == 1001
    assert head(16, 16, 16, 65) == 1002
    assert head(16, 16, 20, 15) == 1002   # Cin > pitch
    assert head(16, 20, 20, 15) == 1002   # 8 float4s per pixel but a 20-float pitch
    assert head(16, 18, 16, 15) == 1002   # pitch % 4
    assert head(20, 16, 16, 15) == 1002   # input not 16-B aligned
    # the JLN's nonzero / scatters: NULLs and sizes before any launch
    assert lib.fvp_mask_nonzero(None, 2, 2, 16, 16, None) == 1001
    assert lib.fvp_mask_nonzero(16, 2, 0, 16, 16, None) == 1002
    assert lib.fvp_mask_nonzero(16, 1 << 13, 1 << 12, 16, 16, None) == 1002
    assert lib.fvp_scatter_poses(None, 0, 1, 1, 1, None, None, None, None, None, None, 7, 7, 4, None) == 0  # P = 0
    assert lib.fvp_scatter_poses(16, 3, 1, 2, 15, 16, 16, 16, 16, 16, None, 7, 7, 4, None) == 1002          # P > B K
    assert lib.fvp_scatter_poses(16, 1, 1, 2, 15, 16, 16, None, 16, 16, 16, 14, 7, 4, None) == 1001         # confs
    # P2PNet's fused tail: NULLs, W % 32, Cpi % 16 / > 128, skip channels, J > 16
    tail = lambda p, w, cpi, cps, cs, j: lib.fvp_up2_head_nchw(p, 1, 4, w, cpi, 16, 16, 16, 16, cps, cs, 16, 16, 16,
                                                               j, 16, None)
    assert tail(None, 32, 64, 32, 32, 15) == 1001
    assert tail(16, 48, 64, 32, 32, 15) == 1002
    assert tail(16, 32, 40, 32, 32, 15) == 1002
    assert tail(16, 32, 144, 32, 32, 15) == 1002
    assert tail(16, 32, 64, 16, 32, 15) == 1002   # skip pitch < its channels
    assert tail(16, 32, 64, 64, 33, 15) == 1002   # > 32 upsampled channels
    assert tail(16, 32, 64, 32, 32, 17) == 1002
    assert tail(20, 32, 64, 32, 32, 15) == 1002   # input not 16-B aligned
    # FVP_CONV_F32_KC (fp32 LDS-DMA kernel): not with bf16 operands, Cpi % 16 only
    conv = lambda cpi, flags: lib.fvp_conv2d_nhwc_ex(1, 1, 8, 8, cpi, 1, 3, 3, 16, 128, 1, 1, None, None, 0,
                                                      0, 1, 1, 1, 1, flags, 0, 1, None, 0, None)
    assert conv(16, 8 | 1) == 1002
    assert conv(4, 8) == 1002
    assert conv(16, 16) == 1002  # unknown flag


def test_backbone_compile_rejects_train_mode():
    from fvp import _lib
    from fvp.backbone import FvpPoseResNet
    import cnn_arch

    with pytest.raises(_lib.FvpError):
        FvpPoseResNet(cnn_arch.PoseResNet(18, 15).train())


# ------------------------------------------------------------------------- GPU
def _conv_case(dev, conv, bn, x, algo=None):
    from fvp.cnn import ConvLayer, to_nchw, to_nhwc

    conv, bn = conv.to(dev).eval(), (bn.to(dev).eval() if bn is not None else None)
    with torch.no_grad():
        if bn is not None:  # non-trivial BN statistics
            bn.running_mean.uniform_(-0.2, 0.2)
            bn.running_var.uniform_(0.5, 1.5)
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
        ref = conv(x) if bn is None else bn(conv(x))
        cin = conv.in_channels
        cpi = 4 if cin <= 4 else None
        layer = ConvLayer(conv, bn, cpi=cpi, algo=algo)
        got = to_nchw(layer(to_nhwc(x, layer.Cpi), relu=False))
    torch.cuda.synchronize()
    return got.cpu().numpy(), ref.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,k,s,p,hw", [
    (3, 64, 7, 2, 3, (70, 90)),      # resnet.py:105 stem on the RGB input (4-channel pitch)
    (64, 64, 3, 2, 1, (35, 45)),     # Bottleneck conv2 with stride (:64), odd sizes
    (256, 512, 1, 2, 0, (17, 23)),   # downsample 1x1/s2 (:134)
    (128, 128, 3, 1, 1, (24, 40)),   # stride-1 3x3 (halo-eligible)
    (1024, 256, 1, 1, 0, (9, 12)),   # Bottleneck 1x1 reduce, long K walk (split-K)
    (256, 17, 3, 1, 1, (24, 24)),    # 3x3 final layer (FINAL_CONV_KERNEL 3)
])
def test_strided_conv_matches_torch(gpu_device, conv_kernel, cin, cout, k, s, p, hw):
    torch.manual_seed(cin + k + s)
    conv = nn.Conv2d(cin, cout, k, s, p, bias=cout == 17)
    bn = None if cout == 17 else nn.BatchNorm2d(cout)
    x = torch.randn((2, cin) + hw, device=gpu_device)
    got, ref = _conv_case(gpu_device, conv, bn, x, conv_kernel)
    assert got.shape == ref.shape
    assert _rel_err(got, ref) <= 2e-5


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,relu,nhw", [(512, 128, True, (3, 10, 14)), (1024, 256, True, (3, 10, 14)),
                                               (2048, 512, False, (3, 10, 14)), (64, 256, False, (1, 1024, 1024)),
                                               (256, 64, True, (2, 512, 1024))])
def test_blas_1x1_matches_torch(gpu_device, cin, cout, relu, nhw):
    """AUTO's library-GEMM path for the 1x1 layers without a residual (resnet.py:60-62
    reducing conv1, :132-137 the first stage's downsample): BN scale folded into the
    weights, bias (+ ReLU) in the GEMM epilogue; K >= 512, or >= 2^20 pixels."""
    from fvp import cnn

    torch.manual_seed(cin + cout)
    conv, bn = nn.Conv2d(cin, cout, 1, bias=False).to(gpu_device).eval(), nn.BatchNorm2d(cout).to(gpu_device).eval()
    n, h, w = nhw
    x = torch.randn((n, cin, h, w), device=gpu_device)
    with torch.no_grad():
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 1.5)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
        ref = bn(conv(x))
        ref = torch.relu(ref) if relu else ref
        layer = cnn.ConvLayer(conv, bn)
        xa = cnn.to_nhwc(x, layer.Cpi)
        out = torch.empty((n, h, w, cout), device=gpu_device)
        assert layer.blas_w is not None and layer._blas(xa, relu, None, None, out, False) == cnn.BLAS_1X1
        got = cnn.to_nchw(layer(xa, relu=relu))
    assert _rel_err(got.cpu().numpy(), ref.cpu().numpy()) <= 2e-5


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,hw", [(2048, 256, (3, 4)), (256, 256, (12, 16)), (48, 32, (5, 7))])
def test_deconv4_matches_torch(gpu_device, conv_kernel, cin, cout, hw):
    """ConvTranspose2d(4, 2, 1) (resnet.py:173-180) as four parity GEMMs."""
    torch.manual_seed(cin + cout)
    conv = nn.ConvTranspose2d(cin, cout, 4, 2, 1, 0, bias=False)
    x = torch.randn((2, cin) + hw, device=gpu_device)
    got, ref = _conv_case(gpu_device, conv, nn.BatchNorm2d(cout), x, conv_kernel)
    assert got.shape == ref.shape == (2, cout, 2 * hw[0], 2 * hw[1])
    assert _rel_err(got, ref) <= 2e-5


@pytest.mark.gpu
@pytest.mark.parametrize("k,s,p", [(3, 2, 1), (3, 1, 1), (2, 2, 0)])  # (3, 2, 1): the stem's 32-bit kernel
def test_maxpool_pad_matches_torch(gpu_device, k, s, p):
    from fvp.cnn import maxpool_pad, to_nchw, to_nhwc

    x = torch.randn((2, 64, 35, 45), device=gpu_device)
    x[0, 3, 0, 0] = float("nan")
    x[1, 5] = -float("inf")
    got = to_nchw(maxpool_pad(to_nhwc(x), k, s, p))
    ref = F.max_pool2d(x, k, s, p)
    torch.cuda.synchronize()
    assert got.shape == ref.shape
    assert torch.equal(torch.nan_to_num(got, 7.0), torch.nan_to_num(ref, 7.0))
    assert torch.equal(torch.isnan(got), torch.isnan(ref))


@pytest.mark.gpu
def test_maxpool_pad_bf16_matches_torch(gpu_device):
    """bf16 NHWC max pool (the bf16 backbone's, after its bf16 stem): exact."""
    from fvp.cnn import Act, maxpool_pad

    x = torch.randn((2, 37, 43, 64), device=gpu_device).to(torch.bfloat16)
    x[0, 0, 0, 3] = float("nan")
    x[1, :, :, 5] = -float("inf")
    got = maxpool_pad(Act(x, 64), 3, 2, 1).t
    assert got.dtype == torch.bfloat16
    ref = F.max_pool2d(x.float().permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1).to(torch.bfloat16)
    torch.cuda.synchronize()
    assert got.shape == ref.shape
    assert torch.equal(torch.nan_to_num(got.float(), 7.0), torch.nan_to_num(ref.float(), 7.0))
    assert torch.equal(torch.isnan(got), torch.isnan(ref))


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["r50", "r18"])
def test_fvp_pose_resnet_matches_reference(gpu_device, tag):
    from fvp.backbone import FvpPoseResNet

    m, x, y = _net(tag)
    m = m.to(gpu_device)
    bb = FvpPoseResNet(m)
    xt = torch.from_numpy(x).to(gpu_device)
    got = bb(xt)
    torch.cuda.synchronize()
    err = _rel_err(got.cpu().numpy(), y)
    print(f"{tag}: max |fvp - reference| = {err:.3g} of the heatmap scale")
    assert got.shape == y.shape and err <= REL
    with torch.no_grad():  # and torch's own GPU forward of the same module
        assert _rel_err(got.cpu().numpy(), m(xt).cpu().numpy()) <= REL
    # the NHWC output holds the same values, joints in channels 0..J-1, zeros after
    act = bb.forward_nhwc(xt)
    J = y.shape[1]
    assert act.Cp >= J and torch.equal(act.t[..., :J].permute(0, 3, 1, 2), got)
    assert int(torch.count_nonzero(act.t[..., J:])) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("cin,hw", [(3, (512, 960)), (3, (37, 70)), (4, (21, 33)), (1, (64, 100))])
def test_stem7_bf16_vs_torch(gpu_device, cin, hw):
    """fvp_conv_stem7_bf16 (7x7/s2/p3 -> 64 + BN + ReLU from NCHW images, bf16
    operands): within 2e-2 of the output scale of torch's fp32 conv of the
    bf16-rounded input, ragged tiles included."""
    import cnn_arch
    from fvp import synthetic
    from fvp.backbone import FvpPoseResNet

    m = cnn_arch.PoseResNet(18, 15).eval()
    m.conv1 = nn.Conv2d(cin, 64, 7, 2, 3, bias=False)
    m.load_state_dict(synthetic.seeded_state_dict(m, 3 + cin))
    m = m.to(gpu_device)
    bb = FvpPoseResNet(m, torch.bfloat16)
    assert bb.stem7 is not None
    x = torch.rand((2, cin) + hw, generator=torch.Generator().manual_seed(cin)).to(gpu_device)
    x = x.to(torch.bfloat16).float()
    got = bb._stem7(x).t.float().permute(0, 3, 1, 2)
    with torch.no_grad():
        ref = torch.relu(m.bn1(m.conv1(x)))
    assert got.shape == ref.shape
    err = float((got - ref).abs().max()) / float(ref.abs().max())
    assert err <= 2e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("cin,hw", [(3, (512, 960)), (3, (37, 70)), (2, (21, 33)), (1, (64, 100))])
def test_stem7_f32_vs_torch(gpu_device, cin, hw):
    """fvp_conv_stem7_f32 (the fp32 backbone's 7x7/s2/p3 -> 64 + BN + ReLU from
    NCHW images, K = the 147 real (tap, channel) pairs): within 2e-5 of the
    output scale of torch's fp32 conv, ragged tiles included; an Inf pixel
    reaches no output outside the windows that hold it (the padded K row reads
    no image data)."""
    import cnn_arch
    from fvp import synthetic
    from fvp.backbone import FvpPoseResNet

    m = cnn_arch.PoseResNet(18, 15).eval()
    m.conv1 = nn.Conv2d(cin, 64, 7, 2, 3, bias=False)
    m.load_state_dict(synthetic.seeded_state_dict(m, 5 + cin))
    m = m.to(gpu_device)
    bb = FvpPoseResNet(m)
    assert bb.stem7_f32 is not None
    x = torch.rand((2, cin) + hw, generator=torch.Generator().manual_seed(cin)).to(gpu_device)
    if hw == (37, 70):
        x[1, cin - 1, 20, 41] = float("inf")
    got = bb._stem7_f32(x).t.permute(0, 3, 1, 2).cpu()
    with torch.no_grad():  # on the CPU: MIOpen's conv spreads an Inf beyond the windows that hold it
        ref = torch.relu(m.bn1.cpu()(m.conv1.cpu()(x.cpu())))
    assert got.shape == ref.shape
    fin = torch.isfinite(ref)
    assert int((~fin).sum()) <= 4 * 4 * 64  # only the windows over the Inf pixel
    err = float((got - ref)[fin].abs().max()) / float(ref[fin].abs().max())
    assert err <= 2e-5, err


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["r50", "r18"])
def test_fvp_pose_resnet_bf16(gpu_device, tag):
    """bf16 operands and activations (opt-in): within 5e-2 of the heatmap scale
    of the reference's fp32 output (ResNet-50's Bottleneck layers run the
    LDS-DMA kernel, the stem the small-channel bf16 path)."""
    from fvp.backbone import FvpPoseResNet

    m, x, y = _net(tag)
    got = FvpPoseResNet(m.to(gpu_device), torch.bfloat16)(torch.from_numpy(x).to(gpu_device))
    torch.cuda.synchronize()
    err = _rel_err(got.cpu().numpy(), y)
    print(f"bf16 {tag}: {err:.3g} of the heatmap scale")
    assert err <= 5e-2


def _c2_layer(dev):
    from fvp.config import make_cfg
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    w = WORKLOADS["c2"]
    layer = ProjectLayer(make_cfg(w, str(dev)))
    layer.verbose = False
    cams, seq = w.cameras()
    from fvp import geometry

    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float32,
                         device=dev)
    return w, layer, cams, seq, rt


@pytest.mark.gpu
@pytest.mark.parametrize("on_the_fly", [False, True])
@pytest.mark.parametrize("J,cp", [(15, 16), (15, 32), (17, 32), (5, 16), (3, 4)])
def test_voxelize_channels_last_bit_exact(gpu_device, on_the_fly, J, cp):
    """fvp_voxelize_cl(_cams) on [B,V,H,W,cp] == fvp_voxelize(_cams) on the same planar values."""
    from fvp.heatmaps import ChannelsLastHeatmaps, attach

    w, layer, cams, seq, rt = _c2_layer(gpu_device)
    layer.on_the_fly = on_the_fly
    g = torch.Generator(device="cpu").manual_seed(J * 100 + cp)
    B, V = 3, 5
    H, W = w.heatmap_size[1], w.heatmap_size[0]
    planar = torch.rand((B, V, J, H, W), generator=g).to(gpu_device)
    cl = torch.zeros((B, V, H, W, cp), device=gpu_device)
    cl[..., :J] = planar.permute(0, 1, 3, 4, 2)
    cl[..., J:] = 123.0  # channels past J are ignored
    meta = {"seq": [seq] * B}
    cube_ref, xy_ref = layer.forward_fused(planar, meta, cams, rt)
    cube, xy = layer.forward_fused(ChannelsLastHeatmaps(cl, J), meta, cams, rt)
    torch.cuda.synchronize()
    assert torch.equal(cube, cube_ref) and torch.equal(xy, xy_ref)
    # through the reference interface: a planar tensor carrying its channels-last copy
    cube2 = layer(attach(planar.clone(), ChannelsLastHeatmaps(cl, J)), meta, cams, rt)
    assert torch.equal(cube2, cube_ref)


@pytest.mark.gpu
def test_attached_copy_is_dropped_after_in_place_write(gpu_device):
    from fvp.heatmaps import ChannelsLastHeatmaps, attach, channels_last_of

    planar = torch.zeros((1, 2, 3, 4, 5), device=gpu_device)
    cl = ChannelsLastHeatmaps(torch.zeros((1, 2, 4, 5, 4), device=gpu_device), 3)
    t = attach(planar, cl)
    assert channels_last_of(t) is cl
    assert channels_last_of(t.clone()) is None and channels_last_of(t[:1]) is None
    t.add_(1.0)
    assert channels_last_of(t) is None


@pytest.mark.gpu
def test_views_to_cube_equals_planar_path(gpu_device):
    """views -> backbone (channels-last, no transpose) -> voxelize == views ->
    backbone NCHW heatmaps -> reference-layout voxelize, bit for bit."""
    from fvp.backbone import FvpPoseResNet
    import cnn_arch
    from fvp import synthetic

    w, layer, cams, seq, rt = _c2_layer(gpu_device)
    m = cnn_arch.PoseResNet(18, 15).eval()
    m.load_state_dict(synthetic.seeded_state_dict(m, 3))
    bb = FvpPoseResNet(m.to(gpu_device))
    B, V = 2, 5
    H, W = w.heatmap_size[1], w.heatmap_size[0]
    views = torch.randn((B, V, 3, 4 * H, 4 * W), generator=torch.Generator().manual_seed(5)).to(gpu_device)
    cl = bb.heatmaps_cl(views)
    assert cl.shape == (B, V, 15, H, W)
    # the reference's per-view loop + stack (faster_voxelpose.py:75): same values up to the
    # launch-size-dependent split-K summation order
    stacked = torch.stack([bb(views[:, c]) for c in range(V)], dim=1)
    planar = cl.planar()
    assert _rel_err(planar.cpu().numpy(), stacked.cpu().numpy()) <= 1e-5
    meta = {"seq": [seq] * B}
    a = layer.forward_fused(cl, meta, cams, rt)
    b = layer.forward_fused(planar.clone(), meta, cams, rt)  # (a clone: the planar path)
    torch.cuda.synchronize()
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


# ------------------------------------------------------------------ drop-in
def _fake_reference(mods_cls):
    """Stand-ins for models.resnet / models.faster_voxelpose with the reference's
    forward flow on the views path (faster_voxelpose.py:73-86)."""
    import types

    rn = types.ModuleType("models.resnet")
    rn.ResNet = mods_cls

    class FasterVoxelPoseNet(nn.Module):
        def __init__(self, project_layer):
            super().__init__()
            self.project_layer = project_layer
            self.seen = None

        def forward(self, backbone=None, views=None, meta=None, targets=None, input_heatmaps=None, cameras=None,
                    resize_transform=None):
            if views is not None:
                input_heatmaps = torch.stack([backbone(views[:, c]) for c in range(views.shape[1])], dim=1)
            from fvp.heatmaps import channels_last_of
            self.seen = channels_last_of(input_heatmaps)  # what the HDN / JLN are handed
            cube = self.project_layer(input_heatmaps, meta, cameras, resize_transform)
            return cube, input_heatmaps

    fv = types.ModuleType("models.faster_voxelpose")
    fv.FasterVoxelPoseNet = FasterVoxelPoseNet
    return {"models.resnet": rn, "models.faster_voxelpose": fv}, FasterVoxelPoseNet


def _restore(cls):
    if hasattr(cls, "_fvp_original_forward"):
        cls.forward = cls._fvp_original_forward
        del cls._fvp_original_forward
    if "fvp_options" in cls.__dict__:  # install()'s per-class options
        del cls.fvp_options


def test_install_backbone_patches_and_falls_back_on_cpu():
    from fvp import integration
    import cnn_arch

    class ResNet(cnn_arch.PoseResNet):  # a subclass: patching it leaves cnn_arch untouched
        pass

    mods, FVP = _fake_reference(ResNet)
    try:
        patched = integration.install(fused=True, modules=mods, backbone=True)
        assert ResNet.forward is integration.fvp_resnet_forward
        assert FVP.forward is integration.fused_fvp_forward
        assert "models.resnet.ResNet.forward" in patched
        m = ResNet(18, 5).eval()
        x = torch.randn(1, 3, 64, 64)
        with torch.no_grad():  # CPU tensors: the reference's own forward
            assert torch.equal(m(x), cnn_arch.PoseResNet.forward(m, x))
    finally:
        _restore(ResNet)
        _restore(FVP)


@pytest.mark.gpu
def test_installed_views_path_matches_reference_flow(gpu_device):
    """install(backbone=True): the model's views path runs the fvp backbone over all
    views at once and the voxelize reads its channels-last output; the cube equals
    the reference flow (per-view backbone, stack, planar voxelize) up to the
    backbone's MFMA summation order, and bit-exactly the planar voxelize of the
    heatmaps the fused path returns."""
    from fvp import integration, synthetic
    from fvp.heatmaps import channels_last_of
    import cnn_arch

    class ResNet(cnn_arch.PoseResNet):
        pass

    w, layer, cams, seq, rt = _c2_layer(gpu_device)
    mods, FVP = _fake_reference(ResNet)
    m = ResNet(18, 15).eval()
    m.load_state_dict(synthetic.seeded_state_dict(m, 4))
    m = m.to(gpu_device)
    model = FVP(layer).eval()
    B, V = 2, 5
    H, W = w.heatmap_size[1], w.heatmap_size[0]
    views = torch.randn((B, V, 3, 4 * H, 4 * W), generator=torch.Generator().manual_seed(6)).to(gpu_device)
    meta = {"seq": [seq] * B}
    with torch.no_grad():
        ref_cube, ref_hm = model(backbone=m, views=views, meta=meta, cameras=cams, resize_transform=rt)
        try:
            integration.install(fused=True, modules=mods, backbone=True)
            cube, hm = model(backbone=m, views=views, meta=meta, cameras=cams, resize_transform=rt)
            assert model.seen is not None  # the HDN got the channels-last copy
            assert channels_last_of(hm) is None  # and it does not outlive the forward
        finally:
            _restore(ResNet)
            _restore(FVP)
        planar = layer(hm.clone(), meta, cams, rt)
    torch.cuda.synchronize()
    assert torch.equal(cube, planar)
    assert _rel_err(hm.cpu().numpy(), ref_hm.cpu().numpy()) <= REL
    assert float((cube - ref_cube).abs().max()) <= 1e-4
