"""Drop-in integration (fvp/integration.py): install() rebinds the reference's
names, and the fused HumanDetectionNet.forward returns what the reference's
forward (human_detection_net.py:157-220) returns for the same modules.  The
dense CNNs are out of scope, so seeded stand-ins with the reference's
attribute names are used; the reference flow is restated with plain torch ops
(torch.max / max_pool2d+topk / torch.gather) around them."""
import types

import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from fvp import integration


def test_install_patches_reference_names():
    mods = {}
    for name in ("models.project_whole", "models.project_individual", "models.human_detection_net",
                 "models.joint_localization_net", "core.proposal"):
        m = types.ModuleType(name)
        mods[name] = m
    mods["models.project_whole"].ProjectLayer = object
    mods["models.project_individual"].ProjectLayer = object
    mods["models.human_detection_net"].ProjectLayer = object
    mods["models.human_detection_net"].nms2D = None
    mods["models.joint_localization_net"].ProjectLayer = object
    mods["core.proposal"].nms2D = None

    class HDN:
        def forward(self):
            return "reference"

    mods["models.human_detection_net"].HumanDetectionNet = HDN
    patched = integration.install(fused=True, modules=mods)
    from fvp import project_individual, project_whole, proposal

    assert mods["models.project_whole"].ProjectLayer is project_whole.ProjectLayer
    assert mods["models.human_detection_net"].ProjectLayer is project_whole.ProjectLayer
    assert mods["models.project_individual"].ProjectLayer is project_individual.ProjectLayer
    assert mods["models.joint_localization_net"].ProjectLayer is project_individual.ProjectLayer
    assert mods["core.proposal"].nms2D is proposal.nms2D
    assert mods["models.human_detection_net"].nms2D is proposal.nms2D
    assert HDN.forward is integration.fused_hdn_forward
    assert HDN.fvp_options == integration.FvpOptions()  # install()'s options, per patched class
    assert integration.options_of(HDN()) is HDN.fvp_options
    assert len(patched) == 8


class _CenterNet(nn.Module):
    """Stand-in with CenterNet's attribute names (cnns_2d.py:235-295)."""

    def __init__(self, J):
        super().__init__()
        self.front_layers = nn.Sequential(nn.Conv2d(J, 8, 3, padding=1), nn.ReLU())
        self.encoder_decoder = nn.Conv2d(8, 8, 3, padding=1)
        self.output_hm = nn.Conv2d(8, 1, 1)
        self.output_size = nn.Conv2d(8, 2, 1)
        with torch.no_grad():  # positive weights: peaks of the xy plane stay peaks (tie-free proposals)
            for m in (self.front_layers[0], self.encoder_decoder, self.output_hm):
                m.weight.abs_()

    def forward(self, x):
        x, _ = torch.max(x, dim=4)
        x = self.encoder_decoder(self.front_layers(x))
        return self.output_hm(x), self.output_size(x)


class _Proposal(nn.Module):
    """Test-mode ProposalLayer semantics (human_detection_net.py:36-37,99-124)."""

    def __init__(self, w):
        super().__init__()
        self.scale = torch.tensor(w.space_size) / (torch.tensor(w.voxels_per_axis) - 1)
        self.bias = torch.tensor(w.space_center) - torch.tensor(w.space_size) / 2.0
        self.min_score = w.min_score

    def forward(self, topk_index, topk_confs, match_bbox, meta):
        B, K = topk_confs.shape
        out = torch.zeros(B, K, 7, device=topk_confs.device)
        out[:, :, 0:3] = topk_index.float() * self.scale.to(out.device) + self.bias.to(out.device)
        out[:, :, 4] = topk_confs
        out[:, :, 3] = (topk_confs > self.min_score).float() - 1.0
        out[:, :, 5:7] = match_bbox
        return out


def _reference_flow(net, heatmaps, meta, cameras, rt):
    """human_detection_net.py:177-220 with plain torch ops (reference semantics)."""
    B, J = heatmaps.shape[0], heatmaps.shape[2]
    cubes = net.project_layer(heatmaps, meta, cameras, rt)
    hm2d, bbox = net.center_net(cubes)
    mx = F.max_pool2d(hm2d, 3, 1, 1)
    nms = ((hm2d == mx).float() * hm2d).reshape(B, -1)
    confs, flat = nms.topk(net.max_people)
    idx2d = torch.stack([torch.div(flat, hm2d.shape[2], rounding_mode="trunc"), flat % hm2d.shape[2]], dim=2)
    bbox_f = torch.flatten(bbox, 2, 3).permute(0, 2, 1)
    match = torch.gather(bbox_f, 1, flat.unsqueeze(2).repeat(1, 1, 2))
    f1d = torch.gather(torch.flatten(cubes, 2, 3).permute(0, 2, 1, 3), 1,
                       flat.view(B, -1, 1, 1).repeat(1, 1, J, cubes.shape[4]))
    hm1d = net.c2c_net(torch.flatten(f1d, 0, 1)).view(B, net.max_people, -1)
    c1, i1 = hm1d.detach().topk(1)
    centers = net.proposal_layer(torch.cat([idx2d, i1], dim=2), confs * c1.squeeze(2), match, meta)
    return hm2d, hm1d, centers, bbox_f


@pytest.mark.gpu
def test_fused_hdn_forward_matches_reference_flow(gpu_device):
    from fvp import geometry, synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    torch.manual_seed(0)
    w = WORKLOADS["c3"]
    net = types.SimpleNamespace()
    net.project_layer = ProjectLayer(w.cfg(str(gpu_device)))
    net.project_layer.verbose = False
    net.center_net = _CenterNet(w.num_joints).to(gpu_device).eval()
    net.c2c_net = nn.Conv1d(w.num_joints, 1, 1).to(gpu_device).eval()
    net.proposal_layer = _Proposal(w)
    net.max_people = w.max_people
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, 3)).to(gpu_device)
    meta = {"seq": [seq] * 3}
    with torch.no_grad():
        ref = _reference_flow(net, hm, meta, cams, rt)
        got = integration.fused_hdn_forward(net, hm, meta, cams, rt)
    assert torch.equal(got[0], ref[0])           # CenterNet heatmap: same conv on the same xy plane
    assert torch.equal(got[3], ref[3])           # bbox preds
    from oracle import fvp_oracle as O

    rc, gc = ref[2].cpu().numpy(), got[2].cpu().numpy()
    v2d, _, _ = O.nms2d(ref[0].cpu().numpy(), w.max_people)
    tie_free = 0
    for b in range(3):  # proposals identical wherever the 2-D peak value is tie-free (topk tie order unspecified)
        for k in range(w.max_people):
            if np.sum(v2d[b] == v2d[b, k]) == 1:
                assert np.array_equal(gc[b, k], rc[b, k])
                tie_free += 1
    assert tie_free > 0
    if tie_free == 3 * w.max_people:
        assert torch.equal(got[1], ref[1])


class _WeightNet(nn.Module):
    """Stand-in with WeightNet's I/O (weight_net.py:48-80): [3,P,J,S,S] -> [3P,J,1] in (0,1)."""

    def __init__(self, J):
        super().__init__()
        self.lin = nn.Linear(1, 1)
        self.J = J

    def forward(self, x):
        x = torch.flatten(x, 0, 1)
        return torch.sigmoid(self.lin(x.mean(dim=(2, 3)).reshape(-1, 1))).view(x.shape[0], self.J, 1)


def _jln_reference_flow(net, meta, heatmaps, pc, mask, cams, rt):
    """joint_localization_net.py:122-182 with plain torch ops (reference semantics,
    per-frame loop, SoftArgmaxLayer :32-56, fuse_pose_preds :83-120)."""
    B, K, J = pc.shape[0], pc.shape[1], heatmaps.shape[2]
    all_f = torch.zeros((B, K, J, 3), device=heatmaps.device)
    all_p = torch.zeros((3, B, K, J, 2), device=heatmaps.device)
    for i in range(B):
        if torch.sum(mask[i]) == 0:
            continue
        cubes, offset = net.project_layer(heatmaps, i, meta, pc[i, mask[i]], cams, rt)
        inp = torch.cat([torch.max(cubes, dim=4)[0], torch.max(cubes, dim=3)[0], torch.max(cubes, dim=2)[0]])
        jf = torch.stack(torch.chunk(net.conv_net(inp), 3), dim=0)
        P = jf.shape[1]
        x = F.softmax(net.soft_argmax_layer.beta * jf.reshape(3, P, J, -1, 1), dim=3)
        confs = torch.mean(torch.max(x, dim=3)[0].squeeze(3), dim=(0, 2))
        pose = torch.sum(x * net.project_layer.center_grid.reshape(3, 1, 1, -1, 2), dim=3)
        o = offset.reshape(-1, 1, 3)
        pose[0] += o[:, :, :2]
        pose[1] += o[:, :, ::2]
        pose[2] += o[:, :, 1:]
        wxy, wxz, wyz = torch.chunk(net.weight_net(jf), 3)
        xw = torch.cat([wxy, wxz], 2)
        yw = torch.cat([wxy, wyz], 2)
        zw = torch.cat([wxz, wyz], 2)
        xw, yw, zw = (t / torch.sum(t, dim=2).unsqueeze(2) for t in (xw, yw, zw))
        fused = torch.cat([xw[:, :, :1] * pose[0][:, :, :1] + xw[:, :, 1:] * pose[1][:, :, :1],
                           yw[:, :, :1] * pose[0][:, :, 1:] + yw[:, :, 1:] * pose[2][:, :, :1],
                           zw[:, :, :1] * pose[1][:, :, 1:] + zw[:, :, 1:] * pose[2][:, :, 1:]], dim=2)
        all_f[i, mask[i]] = fused
        all_p[:, i, mask[i]] = pose
        pc[i, mask[i], 4] = confs
    return all_f, all_p


@pytest.mark.gpu
def test_fused_jln_forward_matches_reference_flow(gpu_device):
    """Batched JLN forward (one planes launch, CNNs on all proposals, fvp
    soft-argmax + fusion) vs the reference's per-frame flow.  Tolerance: the
    stand-in CNNs run on a different batch shape (conv rounding) and the
    softmax sums differ in order: poses within 0.5 mm, confidences 1e-4."""
    from fvp import geometry, jln, synthetic
    from fvp.config import AttrDict
    from fvp.project_individual import ProjectLayer
    from fvp.workloads import WORKLOADS

    torch.manual_seed(0)
    w = WORKLOADS["c3"]
    J = w.num_joints
    net = types.SimpleNamespace(training=False)
    net.project_layer = ProjectLayer(w.cfg(str(gpu_device)))
    net.project_layer.verbose = False
    net.conv_net = nn.Conv2d(J, J, 3, padding=1).to(gpu_device).eval()
    net.weight_net = _WeightNet(J).to(gpu_device).eval()
    net.soft_argmax_layer = jln.SoftArgmaxLayer(AttrDict.wrap({"NETWORK": {"BETA": 100}}))
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    B, K = 3, 5
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, B)).to(gpu_device)
    pc = torch.from_numpy(np.stack([synthetic.proposals_for_frame(w, f, K) for f in range(B)])).to(gpu_device)
    mask = torch.ones((B, K), dtype=torch.bool, device=gpu_device)
    mask[1, 3:] = False
    mask[2] = False  # a frame without proposals
    meta = {"seq": [seq] * B}
    pc_ref, pc_got = pc.clone(), pc.clone()
    with torch.no_grad():
        rf, rp = _jln_reference_flow(net, meta, hm, pc_ref, mask, cams, rt)
        gf, gp = jln.fused_jln_forward(net, meta, hm, pc_got, mask, cams, rt)
    torch.cuda.synchronize()
    np.testing.assert_allclose(gp.cpu().numpy(), rp.cpu().numpy(), atol=0.5, rtol=0)
    np.testing.assert_allclose(gf.cpu().numpy(), rf.cpu().numpy(), atol=0.5, rtol=0)
    np.testing.assert_allclose(pc_got.cpu().numpy(), pc_ref.cpu().numpy(), atol=1e-4, rtol=0)
    assert torch.count_nonzero(gf[2]) == 0 and torch.count_nonzero(gf[1, 3:]) == 0


@pytest.mark.gpu
def test_fused_forwards_with_fvp_cnn(gpu_device):
    """install(cnn=True): CenterNet + C2CNet (HDN) and P2PNet + WeightNet (JLN)
    run on the fvp kernels inside the fused forwards; results match the
    torch-conv fused forwards within the CNN tolerance (2e-5 of the output
    scale; the proposals themselves may reorder only where heatmap values tie
    within it)."""
    import cnn_arch

    from fvp import geometry, jln, synthetic
    from fvp.config import AttrDict
    from fvp.project_individual import ProjectLayer as PI
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    w = WORKLOADS["c3"]
    J = w.num_joints
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, 2)).to(gpu_device)
    meta = {"seq": [seq] * 2}
    hdn = types.SimpleNamespace()
    hdn.project_layer = ProjectLayer(w.cfg(str(gpu_device)))
    hdn.project_layer.verbose = False
    hdn.center_net = cnn_arch.CenterNet(J, 1).eval()
    hdn.center_net.load_state_dict(synthetic.seeded_state_dict(hdn.center_net, 12))
    hdn.center_net = hdn.center_net.to(gpu_device)
    hdn.c2c_net = cnn_arch.C2CNet(J, 1).eval()
    hdn.c2c_net.load_state_dict(synthetic.seeded_state_dict(hdn.c2c_net, 14))
    hdn.c2c_net = hdn.c2c_net.to(gpu_device)
    hdn.proposal_layer = _Proposal(w)
    hdn.max_people = w.max_people
    if True:
        with torch.no_grad():
            integration.set_options(hdn, cnn=False)
            ref = integration.fused_hdn_forward(hdn, hm, meta, cams, rt)
            integration.set_options(hdn, cnn=True)
            got = integration.fused_hdn_forward(hdn, hm, meta, cams, rt)
        scale = float(ref[0].abs().max())
        assert float((got[0] - ref[0]).abs().max()) <= 2e-5 * scale
        assert float((got[3] - ref[3]).abs().max()) <= 2e-5 * float(ref[3].abs().max())
        same = (got[2][:, :, :2] == ref[2][:, :, :2]).all(dim=2)  # same (x, y) column picked
        assert int(same.sum()) > 0
        assert float((got[1] - ref[1])[same].abs().max()) <= 2e-5 * float(ref[1].abs().max())

        net = types.SimpleNamespace(training=False)
        net.project_layer = PI(w.cfg(str(gpu_device)))
        net.project_layer.verbose = False
        net.conv_net = cnn_arch.P2PNet(J, J).eval()
        net.conv_net.load_state_dict(synthetic.seeded_state_dict(net.conv_net, 11))
        net.conv_net = net.conv_net.to(gpu_device)
        net.weight_net = cnn_arch.WeightNet(J).eval()
        net.weight_net.load_state_dict(synthetic.seeded_state_dict(net.weight_net, 15))
        net.weight_net = net.weight_net.to(gpu_device)
        net.soft_argmax_layer = jln.SoftArgmaxLayer(AttrDict.wrap({"NETWORK": {"BETA": 100}}))
        pc = torch.from_numpy(np.stack([synthetic.proposals_for_frame(w, f, 4) for f in range(2)])).to(gpu_device)
        mask = torch.ones((2, 4), dtype=torch.bool, device=gpu_device)
        with torch.no_grad():
            integration.set_options(net, cnn=False)
            rf, rp = jln.fused_jln_forward(net, meta, hm, pc.clone(), mask, cams, rt)
            integration.set_options(net, cnn=True)
            gf, gp = jln.fused_jln_forward(net, meta, hm, pc.clone(), mask, cams, rt)
        np.testing.assert_allclose(gp.cpu().numpy(), rp.cpu().numpy(), atol=0.5, rtol=0)
        np.testing.assert_allclose(gf.cpu().numpy(), rf.cpu().numpy(), atol=0.5, rtol=0)


@pytest.mark.gpu
def test_fused_hdn_forward_trains_like_reference_flow(gpu_device):
    """Training (run/train.py: backbone frozen, HDN trained): in train mode the
    fused forward keeps torch's CenterNet / C2CNet (BatchNorm batch statistics,
    autograd) and feeds them the fvp cube, xy plane and columns.  The losses'
    gradients on every CenterNet and C2CNet parameter match the reference flow's
    (torch.max / torch.gather around the same modules) within fp32 rounding."""
    import copy

    import cnn_arch

    from fvp import geometry, synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    w = WORKLOADS["c3"]
    J = w.num_joints
    cams, seq = w.cameras()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, 2)).to(gpu_device)
    meta = {"seq": [seq] * 2}
    net = types.SimpleNamespace()
    net.project_layer = ProjectLayer(w.cfg(str(gpu_device)))
    net.project_layer.verbose = False
    cn = cnn_arch.CenterNet(J, 1)
    cn.load_state_dict(synthetic.seeded_state_dict(cn, 12))
    c2c = cnn_arch.C2CNet(J, 1)
    c2c.load_state_dict(synthetic.seeded_state_dict(c2c, 14))
    net.proposal_layer = _Proposal(w)
    net.max_people = w.max_people
    grads = []
    for flow in ("fused", "reference"):
        net.center_net = copy.deepcopy(cn).to(gpu_device).train()
        net.c2c_net = copy.deepcopy(c2c).to(gpu_device).train()
        integration.set_options(net, cnn=True)  # ignored in train mode
        if flow == "fused":
            hm2d, hm1d, centers, bbox = integration.fused_hdn_forward(net, hm, meta, cams, rt)
        else:
            hm2d, hm1d, centers, bbox = _reference_flow(net, hm, meta, cams, rt)
        loss = (hm2d ** 2).mean() + (hm1d ** 2).mean() + bbox.abs().mean()
        loss.backward()
        grads.append({n: p.grad.detach().clone() for m in (net.center_net, net.c2c_net)
                      for n, p in m.named_parameters(prefix=type(m).__name__)})
    assert grads[0].keys() == grads[1].keys() and len(grads[0]) > 40
    # A conv bias followed by train-mode BatchNorm has a gradient that is zero
    # in exact arithmetic (the batch mean absorbs it); both flows leave only
    # summation noise there (~1e-7 on GPU, differing run to run), so such
    # parameters are checked to be ~0 in both flows rather than equal.
    gmax = max(float(r.abs().max()) for r in grads[1].values())
    for n in grads[0]:
        g, r = grads[0][n], grads[1][n]
        assert torch.isfinite(g).all(), n
        scale = float(r.abs().max()) + 1e-12
        if scale < 1e-4 * gmax:
            assert float(g.abs().max()) < 1e-4 * gmax, (n, float(g.abs().max()), gmax)
            continue
        assert float((g - r).abs().max()) <= 1e-4 * scale, (n, float((g - r).abs().max()), scale)
