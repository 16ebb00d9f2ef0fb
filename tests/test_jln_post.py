"""JLN post-processing: soft-argmax + offsets + fusion.

Golden vectors: tests/golden/jln_post.npz, produced by the reference's own
SoftArgmaxLayer and JointLocalizationNet.fuse_pose_preds (tools/gen_golden.py)
on stand-in CNN outputs rebuilt from numpy seeds (fvp/synthetic.py).

Tolerance (floating point; exp and 4096-term sums are not reproduced
bit-for-bit): poses within 0.1 mm (the scene is ~4 m, so ~2.5e-5 relative;
the fp32 reference itself differs from a float64 evaluation by 0.035 mm),
confidences within 1e-4.  The fusion arithmetic itself is elementwise and is
checked to 1e-3 mm on identical inputs.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import fvp_oracle as O

POSE_ATOL = 0.1   # mm
CONF_ATOL = 1e-4


def _inputs(d):
    from fvp import synthetic

    P, J, seed = int(d["P"]), int(d["J"]), int(d["seed"])
    return (synthetic.joint_features(P, J, 64, seed), synthetic.jln_weights(P, J, seed),
            synthetic.jln_offsets(P, seed))


def test_oracle_matches_reference_golden():
    d = golden("jln_post.npz")
    feats, weights, offsets = _inputs(d)
    coords, confs = O.soft_argmax(feats, d["center_grid"], float(d["beta"]))
    pose = O.add_offsets(coords, offsets)
    np.testing.assert_allclose(pose, d["pose"], atol=POSE_ATOL, rtol=0)
    np.testing.assert_allclose(confs, d["confs"], atol=CONF_ATOL, rtol=0)
    np.testing.assert_allclose(O.fuse_pose_preds(d["pose"], weights), d["fused"], atol=1e-3, rtol=0)


@pytest.mark.gpu
def test_soft_argmax_and_fuse_match_reference(gpu_device):
    from fvp import ops

    d = golden("jln_post.npz")
    feats, weights, offsets = _inputs(d)
    f = torch.from_numpy(feats).to(gpu_device)
    grid = torch.from_numpy(d["center_grid"]).to(gpu_device)
    pose, maxprob = ops.soft_argmax(f, grid, torch.from_numpy(offsets).to(gpu_device), float(d["beta"]))
    fused, confs = ops.fuse_poses(pose, torch.from_numpy(weights).to(gpu_device), maxprob)
    torch.cuda.synchronize()
    np.testing.assert_allclose(pose.cpu().numpy(), d["pose"], atol=POSE_ATOL, rtol=0)
    np.testing.assert_allclose(confs.cpu().numpy(), d["confs"], atol=CONF_ATOL, rtol=0)
    np.testing.assert_allclose(fused.cpu().numpy(), d["fused"], atol=POSE_ATOL, rtol=0)
    # the fusion arithmetic on the reference's own poses: elementwise, tight
    fz, _ = ops.fuse_poses(torch.from_numpy(d["pose"]).to(gpu_device), torch.from_numpy(weights).to(gpu_device),
                           maxprob)
    np.testing.assert_allclose(fz.cpu().numpy(), d["fused"], atol=1e-3, rtol=0)


@pytest.mark.gpu
def test_soft_argmax_layer_dropin(gpu_device):
    """fvp.jln.SoftArgmaxLayer(cfg).forward(x[3,B,C,H*W,1], grids) like the reference's."""
    from fvp import jln
    from fvp.config import AttrDict

    d = golden("jln_post.npz")
    feats, _, _ = _inputs(d)
    P, J = feats.shape[1], feats.shape[2]
    layer = jln.SoftArgmaxLayer(AttrDict.wrap({"NETWORK": {"BETA": 100}}))
    x = torch.from_numpy(feats).reshape(3, P, J, -1, 1).to(gpu_device)
    coords, confs = layer(x, torch.from_numpy(d["center_grid"]).to(gpu_device))
    ref, rconfs = O.soft_argmax(feats, d["center_grid"], 100.0)
    np.testing.assert_allclose(coords.cpu().numpy(), ref, atol=POSE_ATOL, rtol=0)
    np.testing.assert_allclose(confs.cpu().numpy(), rconfs, atol=CONF_ATOL, rtol=0)
    np.testing.assert_allclose(confs.cpu().numpy(), d["confs"], atol=CONF_ATOL, rtol=0)


@pytest.mark.gpu
def test_empty_batch_is_a_no_op(gpu_device):
    from fvp import ops

    f = torch.zeros((3, 0, 15, 64, 64), device=gpu_device)
    grid = torch.zeros((3, 4096, 2), device=gpu_device)
    pose, maxprob = ops.soft_argmax(f, grid, None, 100.0)
    fused, confs = ops.fuse_poses(pose, torch.zeros((0, 15, 1), device=gpu_device), maxprob)
    assert pose.shape == (3, 0, 15, 2) and fused.shape == (0, 15, 3) and confs.shape == (0,)


@pytest.mark.gpu
@pytest.mark.parametrize("rows,cols,p", [(8, 10, 0.5), (1, 1, 1.0), (3, 7, 0.0), (32, 10, 1.0), (40, 97, 0.3),
                                         (1, 3000, 0.01)])
def test_mask_nonzero_matches_torch(gpu_device, rows, cols, p):
    """fvp_mask_nonzero (the JLN's one sync): exactly torch.nonzero's (row, col) pairs, in
    its row-major order, over one and several 1,024-entry tiles, empty and full masks."""
    from fvp import ops

    g = torch.Generator().manual_seed(rows * cols)
    mask = (torch.rand((rows, cols), generator=g) < p).to(gpu_device)
    got = ops.mask_nonzero(mask)
    assert torch.equal(got, mask.nonzero())
    assert torch.equal(ops.mask_nonzero(mask.t()), mask.t().nonzero())  # a non-contiguous view


@pytest.mark.gpu
def test_scatter_poses_matches_index_put(gpu_device):
    """fvp_scatter_poses: the three boolean scatters of joint_localization_net.py:176-180
    (all_fused, all_pose, the confidence column of proposal_centers) bit for bit."""
    from fvp import ops

    B, K, J = 4, 10, 15
    g = torch.Generator().manual_seed(5)
    mask = (torch.rand((B, K), generator=g) < 0.6).to(gpu_device)
    idx = mask.nonzero()
    P = idx.shape[0]
    fused = torch.randn((P, J, 3), generator=g).to(gpu_device)
    pose = torch.randn((3, P, J, 2), generator=g).to(gpu_device)
    confs = torch.rand((P,), generator=g).to(gpu_device)
    centers = torch.randn((B, K, 7), generator=g).to(gpu_device)
    af, ap, ce = torch.zeros((B, K, J, 3), device=gpu_device), torch.zeros((3, B, K, J, 2), device=gpu_device), \
        centers.clone()
    ops.scatter_poses(idx, fused, pose, confs, af, ap, ce, 4)
    rf, rp, rc = torch.zeros_like(af), torch.zeros_like(ap), centers.clone()
    rf[mask] = fused
    rp[:, mask] = pose
    rc[mask, 4] = confs
    torch.cuda.synchronize()
    assert torch.equal(af, rf) and torch.equal(ap, rp) and torch.equal(ce, rc)


@pytest.mark.gpu
def test_mask_select_matches_torch(gpu_device):
    """fvp_mask_select: nonzero, its frame column as int32 and the selected proposal rows (a
    strided view too) exactly as torch computes them."""
    from fvp import ops

    g = torch.Generator().manual_seed(11)
    for B, K, p in ((8, 10, 0.4), (3, 5, 0.0), (2, 700, 0.5)):
        mask = (torch.rand((B, K), generator=g) < p).to(gpu_device)
        big = torch.randn((B, K, 9), generator=g).to(gpu_device)
        rows = big[:, :, 1:8]  # last dim contiguous, rows strided
        idx, frame_of, sel = ops.mask_select(mask, rows)
        ref = mask.nonzero()
        assert torch.equal(idx, ref)
        assert torch.equal(frame_of, ref[:, 0].to(torch.int32))
        assert torch.equal(sel, rows[mask])
