"""The HDN's 1-D C2CNet and the JLN's WeightNet on fvp kernels (fvp/cnn.py;
csrc/fvp_conv.hip, csrc/fvp_jln.hip).

Golden vectors: tests/golden/cnn.npz ``y_c2c`` / ``y_weight`` -- the
reference's own C2CNet (lib/models/cnns_1d.py:182-241) and WeightNet
(lib/models/weight_net.py:48-80) with seeded weights on seeded inputs, run on
CPU by tools/gen_golden.py.  tests/cnn_arch.py restates both (same attribute
names) for the GPU box and is pinned here.

C2CNet runs on the MFMA convolutions as rows of height 1 (Conv1d(k) = a 1 x k
kernel, ConvTranspose1d(2, 2) = a 1 x 1 conv with a 1 x 2 scatter, max_pool1d
= a 1 x 2 pool).  WeightNet is one fused launch per joint map (conv 3x3 1->C,
BN, 2x2 max pool, ReLU, mean, two Linear layers, sigmoid).

Tolerance: fp32; different summation orders and folded BatchNorm give
agreement to 2e-5 of the output scale (as tests/test_cnn.py).
"""
import numpy as np
import pytest
import torch

from conftest import golden

REL = 2e-5


def _close(got, ref, what, rel=REL):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    scale = max(float(np.abs(ref).max()), 1e-6)
    err = float(np.abs(got - ref).max()) / scale
    assert err <= rel, f"{what}: max error {err:.3g} of the output scale (> {rel})"


def _nets():
    """The restated modules and the inputs gen_golden.py drew (same rng order)."""
    from fvp import synthetic
    import cnn_arch

    c2c = cnn_arch.C2CNet(15, 1).eval()
    c2c.load_state_dict(synthetic.seeded_state_dict(c2c, 14))
    wn = cnn_arch.WeightNet(15).eval()
    wn.load_state_dict(synthetic.seeded_state_dict(wn, 15))
    rng = np.random.default_rng(13)
    rng.uniform(0.0, 1.0, (2, 15, 64, 64))      # P2PNet input (tests/test_cnn.py)
    rng.uniform(0.0, 1.0, (1, 15, 40, 40, 4))   # CenterNet input
    x_c2c = rng.uniform(0.0, 1.0, (6, 15, 20)).astype(np.float32)
    x_wn = rng.normal(0.0, 1.0, (3, 2, 15, 64, 64)).astype(np.float32)
    return c2c, wn, x_c2c, x_wn


def test_restated_c2c_and_weight_net_match_reference_golden():
    d = golden("cnn.npz")
    c2c, wn, x_c2c, x_wn = _nets()
    with torch.no_grad():
        _close(c2c(torch.from_numpy(x_c2c)).numpy(), d["y_c2c"], "C2CNet (CPU restatement)")
        _close(wn(torch.from_numpy(x_wn)).numpy(), d["y_weight"], "WeightNet (CPU restatement)")


def test_weight_net_refuses_other_layouts():
    import torch.nn as nn

    import cnn_arch
    from fvp import _lib
    from fvp.cnn import FvpWeightNet

    wn = cnn_arch.WeightNet(15).eval()
    wn.heatmap_feature_net[2] = nn.AvgPool2d(2)
    with pytest.raises(_lib.FvpError, match="WeightNet layout"):
        FvpWeightNet(wn)
    with pytest.raises(_lib.FvpError, match="eval mode"):
        FvpWeightNet(cnn_arch.WeightNet(15).train())


@pytest.mark.gpu
def test_fvp_c2c_and_weight_net_match_reference(gpu_device):
    from fvp.cnn import FvpCNN, FvpWeightNet

    d = golden("cnn.npz")
    c2c, wn, x_c2c, x_wn = _nets()
    c2c, wn = c2c.to(gpu_device), wn.to(gpu_device)
    xc, xw = torch.from_numpy(x_c2c).to(gpu_device), torch.from_numpy(x_wn).to(gpu_device)
    y = FvpCNN(c2c)(xc)
    w = FvpWeightNet(wn)(xw)
    torch.cuda.synchronize()
    assert tuple(y.shape) == (6, 1, 20) and tuple(w.shape) == (6, 15, 1)
    _close(y.cpu().numpy(), d["y_c2c"], "C2CNet on MFMA")
    _close(w.cpu().numpy(), d["y_weight"], "WeightNet fused")
    with torch.no_grad():  # and against torch's own GPU kernels
        _close(y.cpu().numpy(), c2c(xc).cpu().numpy(), "C2CNet vs torch GPU")
        _close(w.cpu().numpy(), wn(xw).cpu().numpy(), "WeightNet vs torch GPU")


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,k,L,res", [(15, 16, 7, 20, False), (16, 32, 3, 20, True), (32, 64, 1, 10, False),
                                              (128, 128, 3, 5, True), (15, 16, 7, 32, False), (40, 70, 5, 13, True)])
def test_conv1d_layer_vs_torch(gpu_device, cin, cout, k, L, res):
    import torch.nn as nn

    from fvp import cnn, synthetic

    seq = nn.Sequential(nn.Conv1d(cin, cout, k, padding=(k - 1) // 2), nn.BatchNorm1d(cout)).eval()
    seq.load_state_dict(synthetic.seeded_state_dict(seq, cin + cout + k))
    seq = seq.to(gpu_device)
    g = torch.Generator().manual_seed(k + L)
    x = torch.rand((80, cin, L), generator=g).to(gpu_device)
    r = torch.rand((80, cout, L), generator=g).to(gpu_device) if res else None
    with torch.no_grad():
        ref = seq(x)
        ref = torch.relu(ref + r) if res else torch.relu(ref)
    layer = cnn.ConvLayer(seq[0], seq[1])
    a = cnn.to_nhwc(x.unsqueeze(2))
    got = cnn.to_nchw(layer(a, relu=True, res_pre=cnn.to_nhwc(r.unsqueeze(2)) if res else None)).squeeze(2)
    _close(got.cpu().numpy(), ref.cpu().numpy(), f"conv1d {cin}->{cout} k{k} L{L}")


@pytest.mark.gpu
def test_transposed_conv1d_and_pool1d_vs_torch(gpu_device):
    import torch.nn as nn
    import torch.nn.functional as F

    from fvp import cnn, synthetic

    up = nn.Sequential(nn.ConvTranspose1d(128, 64, 2, stride=2), nn.BatchNorm1d(64)).eval()
    up.load_state_dict(synthetic.seeded_state_dict(up, 5))
    up = up.to(gpu_device)
    g = torch.Generator().manual_seed(6)
    x = torch.rand((80, 128, 5), generator=g).to(gpu_device)
    skip = torch.rand((80, 64, 10), generator=g).to(gpu_device)
    with torch.no_grad():
        ref = torch.relu(up(x)) + skip
    layer = cnn.ConvLayer(up[0], up[1])
    got = cnn.to_nchw(layer(cnn.to_nhwc(x.unsqueeze(2)), relu=True, res_post=cnn.to_nhwc(skip.unsqueeze(2))))
    _close(got.squeeze(2).cpu().numpy(), ref.cpu().numpy(), "ConvTranspose1d + BN + ReLU + skip")
    for L in (20, 11):  # even and odd (floor) lengths
        p = torch.rand((7, 48, L), generator=g).to(gpu_device)
        got = cnn.to_nchw(cnn.maxpool2(cnn.to_nhwc(p.unsqueeze(2)), dim=1)).squeeze(2)
        assert torch.equal(got, F.max_pool1d(p, 2, 2))


@pytest.mark.gpu
@pytest.mark.parametrize("N,L", [(80, 20), (80, 32), (40, 64), (1, 20), (320, 20)])
def test_c2c_large_batch_vs_torch(gpu_device, N, L):
    """N columns (80 = 8 frames x K=10) at the C2 / C3 (Z=20), C4 (Z=32) and C5
    (Z=64) column lengths, through the one-launch net (fvp_conv1d_net, the AUTO
    path; Z = 64 with 8,192-float weight chunks) and the per-layer kernels: both
    against torch's C2CNet."""
    from fvp import cnn
    from fvp.cnn import FvpCNN

    c2c, _, _, _ = _nets()
    c2c = c2c.to(gpu_device)
    x = torch.rand((N, 15, L), generator=torch.Generator().manual_seed(L + N)).to(gpu_device)
    with torch.no_grad():
        ref = c2c(x)
    net = FvpCNN(c2c)
    y = net(x)
    n1 = net.net1d[(15, L)]
    assert n1 is not None, "the one-launch path was not taken"
    assert n1.wchunk == (8192 if L == 64 else 12288)  # (Z = 64: smaller weight chunks make room)
    _close(y.cpu().numpy(), ref.cpu().numpy(), f"C2CNet one launch, {N} columns of {L}")
    per_layer = FvpCNN(c2c, algo=cnn.CONV_PER_TAP)(x)
    _close(per_layer.cpu().numpy(), ref.cpu().numpy(), f"C2CNet per layer, {N} columns of {L}")


def test_one_launch_c2c_refuses_lengths_the_reference_cannot_run():
    """Z % 4 != 0: two pools then two upsamples do not restore Z, and the reference
    fails at ``x + skip_x2`` (cnns_1d.py:223-233).  The one-launch net must not be
    planned for such a length (it would read the skip buffer at the wrong pitch)."""
    from fvp.cnn import Net1D

    c2c, _, _, _ = _nets()
    for L in (30, 18, 22, 2):
        assert Net1D.build(c2c, 15, L) is None
        with pytest.raises(RuntimeError):  # and the reference itself refuses it
            with torch.no_grad():
                c2c(torch.zeros((1, 15, L)))


@pytest.mark.gpu
def test_c2c_odd_length_raises_like_the_reference(gpu_device):
    from fvp.cnn import FvpCNN

    c2c, _, _, _ = _nets()
    net = FvpCNN(c2c.to(gpu_device))
    with pytest.raises((AssertionError, RuntimeError)):
        net(torch.rand((4, 15, 30), device=gpu_device))
    assert net.net1d.get((15, 30)) is None


@pytest.mark.gpu
@pytest.mark.parametrize("feat,hidden,hw,P", [(32, 64, (64, 64), 10), (16, 32, (33, 18), 3), (64, 100, (40, 40), 2)])
def test_weight_net_shapes_vs_torch(gpu_device, feat, hidden, hw, P):
    """Channel counts of both template widths, odd map sizes (floor pooling)."""
    from fvp import synthetic
    from fvp.cnn import FvpWeightNet
    import cnn_arch

    wn = cnn_arch.WeightNet(15, hw, feat, hidden).eval()
    wn.load_state_dict(synthetic.seeded_state_dict(wn, feat + hidden))
    wn = wn.to(gpu_device)
    x = torch.randn((3, P, 15) + hw, generator=torch.Generator().manual_seed(P)).to(gpu_device)
    with torch.no_grad():
        ref = wn(x)
    got = FvpWeightNet(wn)(x)
    assert got.shape == ref.shape
    _close(got.cpu().numpy(), ref.cpu().numpy(), f"WeightNet C={feat} Hd={hidden} {hw}")


@pytest.mark.gpu
def test_bf16_c2c_vs_reference(gpu_device):
    from fvp.cnn import FvpCNN

    d = golden("cnn.npz")
    c2c, _, x_c2c, _ = _nets()
    y = FvpCNN(c2c.to(gpu_device), torch.bfloat16)(torch.from_numpy(x_c2c).to(gpu_device))
    _close(y.cpu().numpy(), d["y_c2c"], "C2CNet bf16", rel=5e-2)


@pytest.mark.gpu
def test_graphed_c2c_equals_eager(gpu_device):
    """fvp.cnn.GraphedCNN (C2CNet replayed from a hipGraph per input shape):
    bit-identical to the eager launches for every call, new inputs copied in,
    several shapes (more than the cache keeps: those run eagerly, counted),
    outputs not aliased."""
    from fvp import cnn

    c2c, _, _, _ = _nets()
    c2c = c2c.to(gpu_device)
    # the per-layer kernels (a launch-bound chain: what the graphs are for); the one-launch
    # net (AUTO) runs eagerly inside GraphedCNN -- a graph of one kernel only adds copies
    eager = cnn.FvpCNN(c2c, algo=cnn.CONV_PER_TAP)
    g = cnn.GraphedCNN(cnn.FvpCNN(c2c, algo=cnn.CONV_PER_TAP), max_shapes=2)
    one = cnn.GraphedCNN(cnn.FvpCNN(c2c))
    x1 = torch.rand((80, 15, 20), generator=torch.Generator().manual_seed(4)).to(gpu_device)
    assert torch.equal(one(x1), cnn.FvpCNN(c2c)(x1)) and not one._graphs and one.eager_calls == 0
    gen = torch.Generator().manual_seed(3)
    outs = []
    for n, L in ((80, 20), (80, 20), (30, 32), (8, 20), (80, 20), (30, 32)):
        x = torch.rand((n, 15, L), generator=gen).to(gpu_device)
        got = g(x)
        outs.append((got, eager(x)))
    torch.cuda.synchronize()
    for got, ref in outs:  # earlier results survive later replays
        assert torch.equal(got, ref)
    assert len(g._graphs) == 2 and g.eager_calls == 1  # (8, 20): the third shape, past max_shapes


def test_cached_signature_tracks_every_change():
    """fvp.cnn.cached rebuilds its wrapper when the module's weights change: the
    fast walk (_tensor_sig) must see in-place writes, load_state_dict, a
    reassigned Parameter, a replaced submodule and BatchNorm statistics, and
    stay equal when nothing changed."""
    import torch.nn as nn

    import cnn_arch
    from fvp import synthetic
    from fvp.cnn import _tensor_sig

    m = cnn_arch.C2CNet(15, 1).eval()
    s0 = _tensor_sig(m)
    assert _tensor_sig(m) == s0 and len(s0) == len(list(m.parameters())) + len(list(m.buffers()))
    with torch.no_grad():
        m.output_hm.weight.add_(1.0)  # in place: version
    s1 = _tensor_sig(m)
    assert s1 != s0
    m.load_state_dict(synthetic.seeded_state_dict(m, 3))
    s2 = _tensor_sig(m)
    assert s2 != s1
    m.output_hm.weight = nn.Parameter(m.output_hm.weight.detach().clone())  # reassigned: storage
    s3 = _tensor_sig(m)
    assert s3 != s2
    bn = next(x for x in m.modules() if isinstance(x, nn.BatchNorm1d))
    bn.running_mean.add_(0.5)
    s4 = _tensor_sig(m)
    assert s4 != s3
    m.output_hm = nn.Conv1d(32, 1, 1)  # a replaced submodule: the walk is re-listed
    s5 = _tensor_sig(m)
    assert s5 != s4 and len(s5) == len(list(m.parameters())) + len(list(m.buffers()))
    assert _tensor_sig(m) == s5
