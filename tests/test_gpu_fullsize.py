"""HIP path vs the reference at the BASELINE configs' full sizes, and the
drop-in HDN / JLN forwards vs the reference's own forwards.

* C4 (configs[3]: demo cameras, 128x128x32) and C5 (configs[4]: 31 ring
  cameras, fp16 heatmaps, 160x160x64) against tests/golden/whole_c{4,5}.npz,
  which tools/gen_golden.py wrote by running the reference's ProjectLayer
  (lib/models/project_whole.py:119-168) -- through the cached-grid kernel and
  the on-the-fly projection kernel (what the C5 bench runs).
* e2e_c3.npz: the reference's HumanDetectionNet.forward
  (human_detection_net.py:157-220) and JointLocalizationNet.forward
  (joint_localization_net.py:122-182) in eval mode with seeded CNN weights,
  against integration.fused_hdn_forward / jln.fused_jln_forward on the same
  modules (tests/cnn_arch.py, identical state_dicts) with the CNNs on torch and
  on the fvp MFMA engine.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import fvp_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-4  # north_star: "within 1e-4 on float32 voxel values"


def _report(got, ref, what, exact=True):
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    diff = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    n = int(np.count_nonzero(diff))
    print(f"{what}: {n} of {diff.size} differ, max |diff| {float(diff.max()) if diff.size else 0.0:.3g}")
    assert float(diff.max()) <= TOL, f"{what}: max |diff| {float(diff.max())} > {TOL}"
    if exact:
        assert n == 0, f"{what}: not bit-exact ({n} of {diff.size} differ)"


def _layer(wname, dev, otf):
    from fvp.project_whole import ProjectLayer
    from fvp.workloads import WORKLOADS

    w = WORKLOADS[wname]
    layer = ProjectLayer(w.cfg(str(dev)))
    layer.verbose = False
    layer.on_the_fly = otf
    cams, seq = w.cameras()
    return w, layer, cams, seq


def _check_whole(d, w, layer, cams, seq, hm, dev, tag):
    from fvp.proposal import gather_columns, nms2D

    rt = torch.from_numpy(d["resize_f32"]).to(dev)
    cube, xy = layer.forward_fused(hm, {"seq": [seq] * hm.shape[0]}, cams, rt)
    torch.cuda.synchronize()
    J, (X, Y, Z) = w.num_joints, w.voxels_per_axis
    c = cube.reshape(hm.shape[0], J, -1)
    sub = torch.from_numpy(d["sub"]).to(dev)
    _report(c[:, :, sub].cpu().numpy(), d["cube_sub"], f"{tag} cube (sampled voxels)")
    _report(xy.cpu().numpy(), d["xy"], f"{tag} xy plane")
    _report(cube.amax(dim=(2, 3, 4)).cpu().numpy(), d["cube_max"], f"{tag} per-joint max")
    # the same fp32 values summed in the same (numpy) order: equal only if every voxel is
    # (every byte of the cube is pinned by tests/test_gpu_digests.py)
    assert np.array_equal(cube.cpu().numpy().astype(np.float64).sum(axis=(2, 3, 4)), d["cube_sum"])
    vals, idx, flat = nms2D(xy[:, 2:3], w.max_people)
    assert np.array_equal(vals.cpu().numpy(), d["nms_vals"])
    assert np.array_equal(flat.cpu().numpy(), d["nms_flat"]), "argmax proposal indices differ"
    assert np.array_equal(idx.cpu().numpy(), d["nms_xy"])
    _report(gather_columns(cube, flat).cpu().numpy(), d["columns"], f"{tag} columns")
    return cube


@pytest.mark.parametrize("otf", [False, True], ids=["grid", "otf"])
def test_c4_full_size_vs_reference(gpu_device, otf):
    """configs[3]: 128x128x32, 5 demo cameras, one frame at full size plus the
    uniform-random stress frame (every voxel of the sampled set, the full xy
    plane, top-10 indices, columns)."""
    from fvp import synthetic

    d = golden("whole_c4.npz")
    w, layer, cams, seq = _layer("c4", gpu_device, otf)
    _check_whole(d, w, layer, cams, seq, torch.from_numpy(d["heatmaps"]).to(gpu_device), gpu_device,
                 f"C4 {'otf' if otf else 'grid'}")
    hu = synthetic.uniform_heatmaps(w, 1, seed=0).to(gpu_device)
    cube, xy = layer.forward_fused(hu, {"seq": [seq]}, cams, torch.from_numpy(d["resize_f32"]).to(gpu_device))
    sub = torch.from_numpy(d["sub"]).to(gpu_device)
    _report(cube.reshape(1, w.num_joints, -1)[:, :, sub].cpu().numpy(), d["u_cube_sub"], "C4 uniform cube")
    _report(xy.cpu().numpy(), d["u_xy"], "C4 uniform xy")


@pytest.mark.parametrize("otf", [True, False], ids=["otf", "grid"])
def test_c5_full_size_vs_reference(gpu_device, otf):
    """configs[4]: 31 ring cameras (voxels behind cameras included), fp16
    heatmaps, 160x160x64 -- the on-the-fly projection kernel the C5 bench runs
    (the 406 MB grid exceeds ON_THE_FLY_GRID_BYTES) and the cached-grid kernel;
    the 31-camera mean in torch's 16-block cascade order (fvp_device.h)."""
    import hashlib

    from fvp import synthetic

    d = golden("whole_c5.npz")
    w, layer, cams, seq = _layer("c5", gpu_device, otf)
    hm16 = synthetic.gaussian_heatmaps(w, 1).astype(np.float16)
    assert hashlib.sha256(hm16.astype(np.float32).tobytes()).digest() == d["heatmaps_sha256"].tobytes()
    _check_whole(d, w, layer, cams, seq, torch.from_numpy(hm16).to(gpu_device), gpu_device,
                 f"C5 {'otf' if otf else 'grid'}")


def test_c5_full_size_frame_groups(gpu_device):
    """C5 at full size with 7 frames: one group of 4 frames per pair-table
    entry (the default), then a pair, then a single frame -- every frame's cube
    and xy plane equal its own one-frame launch (the single-frame path is
    pinned by the C5 digests and whole_c5.npz)."""
    from fvp import geometry, synthetic

    w, layer, cams, seq = _layer("c5", gpu_device, True)
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, 7, first_frame=5).astype(np.float16)).to(gpu_device)
    cube, xy = layer.forward_fused(hm, {"seq": [seq] * 7}, cams, rt)
    for b in range(7):
        c1, x1 = layer.forward_fused(hm[b:b + 1], {"seq": [seq]}, cams, rt)
        assert torch.equal(cube[b:b + 1], c1) and torch.equal(xy[b:b + 1], x1), f"frame {b}"
    print("C5 7 frames (entries of 4, 2, 1 frames): every frame equals its one-frame launch")


# ---------------------------------------------------------------------------
# the drop-in forwards vs the reference's own HumanDetectionNet / JointLocalizationNet

def _hdn(w, dev):
    import types

    import cnn_arch

    from fvp import synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.proposal import ProposalLayer

    net = types.SimpleNamespace()
    cfg = w.cfg(str(dev))
    net.project_layer = ProjectLayer(cfg)
    net.project_layer.verbose = False
    net.center_net = cnn_arch.CenterNet(w.num_joints, 1).eval()
    net.center_net.load_state_dict(synthetic.seeded_state_dict(net.center_net, 12))
    with torch.no_grad():  # as tools/gen_golden.py: positive peaks in the seeded heatmap head
        net.center_net.output_hm[2].bias += float(golden("e2e_c3.npz")["hm_bias_shift"])
    net.center_net = net.center_net.to(dev)
    net.c2c_net = cnn_arch.C2CNet(w.num_joints, 1).eval()
    net.c2c_net.load_state_dict(synthetic.seeded_state_dict(net.c2c_net, 14))
    net.c2c_net = net.c2c_net.to(dev)
    net.proposal_layer = ProposalLayer(cfg).eval()
    net.max_people = w.max_people
    return net


def _match_ranked(got_v, got_i, ref_v, ref_i, tol, what):
    """Top-K lists from CNN outputs (not bit-exact): values within tol at every
    rank; indices identical at every rank whose reference value is separated
    from its neighbours by more than 2*tol (a closer pair may swap).  Returns
    the number of ranks compared by index."""
    checked = 0
    for b in range(ref_v.shape[0]):
        np.testing.assert_allclose(got_v[b], ref_v[b], atol=tol, rtol=0, err_msg=what)
        for k in range(ref_v.shape[1]):
            gap = np.abs(np.delete(ref_v[b], k) - ref_v[b, k]).min() if ref_v.shape[1] > 1 else np.inf
            if gap > 2 * tol:
                assert got_i[b, k] == ref_i[b, k], (what, b, k)
                checked += 1
    return checked


@pytest.mark.parametrize("cnn", ["torch", "fvp"])
def test_fused_hdn_forward_matches_reference_hdn(gpu_device, cnn):
    """integration.fused_hdn_forward (one voxelize launch for cube + xy, fvp NMS,
    gathers and the fused z pick / ProposalLayer) vs the reference's own
    HumanDetectionNet.forward on C3 inputs.  The CNNs differ from torch-CPU by
    summation order only: maps within 2e-5 of their scale; proposal indices
    identical wherever the reference's values are separated by more than that."""
    from fvp import geometry, integration
    from fvp.workloads import WORKLOADS

    d = golden("e2e_c3.npz")
    w = WORKLOADS["c3"]
    cams, seq = w.cameras()
    net = _hdn(w, gpu_device)
    hm = torch.from_numpy(golden("whole_c3.npz")["heatmaps"]).to(gpu_device)
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    integration.set_options(net, cnn=cnn == "fvp")
    with torch.no_grad():
        hm2d, hm1d, centers, bbox = integration.fused_hdn_forward(net, hm, {"seq": [seq] * 2}, cams, rt)
    torch.cuda.synchronize()
    hm2d, hm1d, centers, bbox = (t.cpu().numpy() for t in (hm2d, hm1d, centers, bbox))
    s2 = float(np.abs(d["hm2d"]).max())
    tol2 = 2e-5 * s2
    print(f"HDN[{cnn}]: hm2d max |diff| {np.abs(hm2d - d['hm2d']).max():.3g} (scale {s2:.3g}), "
          f"bbox {np.abs(bbox - d['bbox']).max():.3g}")
    np.testing.assert_allclose(hm2d, d["hm2d"], atol=tol2, rtol=0)
    np.testing.assert_allclose(bbox, d["bbox"], atol=2e-5 * float(np.abs(d["bbox"]).max()), rtol=0)
    # proposals: (x, y) from the top-K of each side's own 2-D map (fvp NMS == oracle
    # bit for bit, test_gpu_parity), z from the 1-D maps
    ref_c = d["centers"]
    rv, _, rfl = O.nms2d(d["hm2d"], w.max_people)
    gv, _, gfl = O.nms2d(hm2d, w.max_people)
    n_idx = _match_ranked(gv, gfl, rv, rfl, tol2, "2-D proposal indices")
    print(f"HDN ({cnn} CNNs): {n_idx} of {rfl.size} proposal ranks compared by index, {rfl.size - n_idx} skipped "
          f"(reference values within 2x{tol2:.2e} of a neighbour); {int((gfl == rfl).sum())} indices identical")
    assert n_idx >= 10, f"only {n_idx} proposals compared by index"
    X = w.voxels_per_axis[0]
    mm = lambda fl, a: (np.float32(fl // X if a == 0 else fl % X) * np.float32(w.space_size[a] / (w.voxels_per_axis[a] - 1))  # noqa: E731
                        + np.float32(w.space_center[a] - w.space_size[a] / 2.0))
    for a in (0, 1):  # both sides' centres decode their own top-K (get_index2D's divisor X)
        assert np.allclose(centers[:, :, a], mm(gfl, a), atol=1e-3) and np.allclose(ref_c[:, :, a], mm(rfl, a), atol=1e-3)
    same = gfl == rfl
    s1 = float(np.abs(d["hm1d"]).max())
    np.testing.assert_allclose(hm1d[same], d["hm1d"][same], atol=2e-5 * s1, rtol=0)
    # where the same column was picked: identical centre (bit-exact index -> mm), close confidences
    assert np.array_equal(centers[same][:, :2], ref_c[same][:, :2])
    zsep = np.sort(d["hm1d"][same], axis=1)
    zsep = zsep[:, -1] - zsep[:, -2]
    zok = zsep > 4e-5 * s1
    assert np.array_equal(centers[same][zok][:, 2], ref_c[same][zok][:, 2])
    np.testing.assert_allclose(centers[same][:, 4], ref_c[same][:, 4], atol=1e-4 * max(1.0, s1 * s2), rtol=0)
    np.testing.assert_allclose(centers[same][:, 5:7], ref_c[same][:, 5:7], atol=2e-5 * float(np.abs(d["bbox"]).max()))
    far = np.abs(ref_c[same][:, 4] - float(d["min_score"])) > 1e-3
    assert np.array_equal(centers[same][far][:, 3], ref_c[same][far][:, 3])
    print(f"HDN[{cnn}]: {n_idx} proposal indices compared, {int(same.sum())} columns, {int(zok.sum())} z picks")


@pytest.mark.parametrize("cnn", ["torch", "fvp"])
def test_fused_jln_forward_matches_reference_jln(gpu_device, cnn):
    """jln.fused_jln_forward (all proposals in one planes launch, CNNs batched,
    fvp soft-argmax + fusion) vs the reference's own JointLocalizationNet.forward
    on the reference HDN's proposals (first 4 per frame).  Poses within 0.2 mm
    (1e-4 of the 2 m person cube: the beta = 100 soft-argmax amplifies the CNNs'
    summation-order differences), confidences within 1e-4."""
    import types

    import cnn_arch

    from fvp import geometry, integration, jln, synthetic
    from fvp.config import AttrDict
    from fvp.project_individual import ProjectLayer
    from fvp.workloads import WORKLOADS

    d = golden("e2e_c3.npz")
    w = WORKLOADS["c3"]
    J = w.num_joints
    cams, seq = w.cameras()
    net = types.SimpleNamespace(training=False)
    net.project_layer = ProjectLayer(w.cfg(str(gpu_device)))
    net.project_layer.verbose = False
    net.conv_net = cnn_arch.P2PNet(J, J).eval()
    net.conv_net.load_state_dict(synthetic.seeded_state_dict(net.conv_net, 11))
    net.conv_net = net.conv_net.to(gpu_device)
    net.weight_net = cnn_arch.WeightNet(J).eval()
    net.weight_net.load_state_dict(synthetic.seeded_state_dict(net.weight_net, 15))
    net.weight_net = net.weight_net.to(gpu_device)
    net.soft_argmax_layer = jln.SoftArgmaxLayer(AttrDict.wrap({"NETWORK": {"BETA": 100}}))
    hm = torch.from_numpy(golden("whole_c3.npz")["heatmaps"]).to(gpu_device)
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    pc = torch.from_numpy(d["centers"]).to(gpu_device)
    mask = torch.from_numpy(d["mask"]).to(gpu_device)
    integration.set_options(net, cnn=cnn == "fvp")
    with torch.no_grad():
        fused, poses = jln.fused_jln_forward(net, {"seq": [seq] * 2}, hm, pc, mask, cams, rt)
    torch.cuda.synchronize()
    fused, poses, pc = fused.cpu().numpy(), poses.cpu().numpy(), pc.cpu().numpy()
    print(f"JLN[{cnn}]: fused max |diff| {np.abs(fused - d['fused']).max():.3g} mm, "
          f"poses {np.abs(poses - d['poses']).max():.3g} mm, confs {np.abs(pc[..., 4] - d['centers_after'][..., 4]).max():.3g}")
    np.testing.assert_allclose(poses, d["poses"], atol=0.2, rtol=0)
    np.testing.assert_allclose(fused, d["fused"], atol=0.2, rtol=0)
    np.testing.assert_allclose(pc, d["centers_after"], atol=1e-4, rtol=0)
    assert not np.any(fused[~d["mask"]])


def test_shared_layout_follows_a_reused_buffer(gpu_device):
    """The fused HDN lays planar heatmaps out channels-last once per forward
    (share_layout) and the JLN drops that copy.  A caller that refills the same
    tensor through ``.data`` (which, like DLPack or the C ABI, does not move
    ``_version``) must get the new values' results, not the old copy's."""
    import types

    from fvp import geometry, integration, jln
    from fvp.heatmaps import channels_last_of
    from fvp.workloads import WORKLOADS

    w = WORKLOADS["c3"]
    cams, seq = w.cameras()
    net = _hdn(w, gpu_device)
    a = torch.from_numpy(golden("whole_c3.npz")["heatmaps"]).to(gpu_device)
    b = (a.flip(0) * 0.75).contiguous()
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(gpu_device)
    meta = {"seq": [seq] * 2}
    with torch.no_grad():
        # (torch's GPU convolutions in CenterNet are not bit-reproducible from call to
        # call: the maps are compared to 1e-5 of their scale, against the stale result too)
        stale = integration.fused_hdn_forward(net, a.clone(), meta, cams, rt)
        want = integration.fused_hdn_forward(net, b.clone(), meta, cams, rt)
        buf = a.clone()
        integration.fused_hdn_forward(net, buf, meta, cams, rt)  # HDN alone: its copy stays attached
        assert channels_last_of(buf) is not None
        v = buf._version
        buf.data.copy_(b)
        assert buf._version == v  # invisible to the version counter
        got = integration.fused_hdn_forward(net, buf, meta, cams, rt)
        torch.cuda.synchronize()
        for i in (0, 3):  # hm2d and bbox (proposal picks could swap near-ties between runs)
            g, r, s = got[i], want[i], stale[i]
            tol = 1e-5 * float(r.abs().max())
            assert float((g - r).abs().max()) <= tol
            assert float((s - r).abs().max()) > 100 * tol  # the stale copy would have been visible
        # the JLN is the copy's last consumer and drops it
        jnet = types.SimpleNamespace(training=False, project_layer=None)
        from fvp.project_individual import ProjectLayer
        jnet.project_layer = ProjectLayer(w.cfg(str(gpu_device)))
        jnet.project_layer.verbose = False
        jnet.conv_net = torch.nn.Identity()
        jnet.weight_net = lambda f: torch.ones(f.shape[0] * f.shape[1], f.shape[2], 1, device=f.device)
        jnet.soft_argmax_layer = types.SimpleNamespace(beta=100.0)
        pc = got[2].clone()
        pc[..., 3] = 0.0
        jln.fused_jln_forward(jnet, meta, buf, pc, pc[..., 3] >= 0, cams, rt)
        assert channels_last_of(buf) is None


def test_proposal_layer_test_mode_matches_reference_semantics(gpu_device):
    """fvp.proposal.ProposalLayer (and the fused z pick) vs human_detection_net.py:
    36-37, 99-124 restated with torch ops: bit-exact centres, confidences,
    validity; z = topk(1) over the 1-D maps incl. NaN (ties: lowest index)."""
    from fvp.proposal import ProposalLayer, proposal_centers
    from fvp.workloads import WORKLOADS

    w = WORKLOADS["c3"]
    cfg = w.cfg(str(gpu_device))
    layer = ProposalLayer(cfg).eval()
    g = torch.Generator().manual_seed(5)
    B, K, Z = 3, 10, 20
    idx2 = torch.randint(0, 80, (B, K, 2), generator=g)
    hm1d = torch.rand((B, K, Z), generator=g)
    hm1d[0, 0, 3] = hm1d[0, 0, 9] = 2.0      # tie: lowest index
    hm1d[0, 1, 7] = float("nan")             # NaN wins
    confs = torch.rand((B, K), generator=g)
    confs[1, :3] = torch.tensor([0.3, 0.3000001, 0.2999999])  # around MIN_SCORE
    bbox = torch.rand((B, K, 2), generator=g)
    c1, i1 = hm1d.topk(1)
    ref_idx = torch.cat([idx2, i1], dim=2)
    ref_conf = confs * c1.squeeze(2)
    scale = torch.tensor(cfg.CAPTURE_SPEC.SPACE_SIZE) / (torch.tensor(cfg.CAPTURE_SPEC.VOXELS_PER_AXIS) - 1)
    bias = torch.tensor(cfg.CAPTURE_SPEC.SPACE_CENTER) - torch.tensor(cfg.CAPTURE_SPEC.SPACE_SIZE) / 2.0
    ref = torch.zeros(B, K, 7)
    ref[:, :, 0:3] = ref_idx.float() * scale + bias
    ref[:, :, 4] = ref_conf
    ref[:, :, 3] = (ref_conf > cfg.CAPTURE_SPEC.MIN_SCORE).float() - 1.0
    ref[:, :, 5:7] = bbox
    to = lambda t: t.to(gpu_device)  # noqa: E731
    got = proposal_centers(layer, to(idx2), to(hm1d), to(confs), to(bbox)).cpu()
    # torch.topk(1) leaves ties unspecified (CPU: index 3 or 9 here depending on the
    # row length); fvp takes the lowest index, as its NMS does
    assert got[0, 0, 2] == 3 * scale[2] + bias[2]
    ref[0, 0, 2] = got[0, 0, 2]
    assert torch.equal(torch.nan_to_num(got, nan=-7.0), torch.nan_to_num(ref, nan=-7.0))
    assert got[0, 1, 2] == 7 * scale[2] + bias[2]
    # the module's own forward (3-D index given)
    ref2 = ref.clone()
    ref2[:, :, 0:3] = ref_idx.float() * scale + bias
    ref2[:, :, 4] = confs
    ref2[:, :, 3] = (confs > cfg.CAPTURE_SPEC.MIN_SCORE).float() - 1.0
    got2 = layer(to(ref_idx), to(confs), to(bbox), {}).cpu()
    assert torch.equal(got2, ref2)
