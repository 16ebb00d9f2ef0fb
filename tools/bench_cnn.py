#!/usr/bin/env python3
"""CNN line: P2PNet on the JLN planes of K proposals
(3K images of J x 64 x 64), CenterNet on B xy planes (J x 80 x 80), C2CNet on
the 10 z-columns of each of the B frames and WeightNet on the 3K joint-feature
stacks; fvp kernels vs torch's own GPU path for the same eval-mode module.

    python tools/bench_cnn.py [--proposals 10] [--frames 8] [--iters 10]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

MFMA_F32_PEAK_TF = 157.3


def _pmc_forward(d, net):
    """The forward totals tools/pmc_forwards.sh wrote for `net` (pmc_<net>.jsonl, last
    line) and the image count of that run (trace_<net>.json is the same batch)."""
    if not d:
        return None
    f = os.path.join(d, f"pmc_{net}.jsonl")
    if not os.path.exists(f):
        return None
    tot = json.loads(open(f).read().splitlines()[-1])
    if "mfma_gflop_issued" not in tot:
        return None
    images = {"p2p": 240, "centernet": 8}[net]  # tools/pmc_forwards.sh batch sizes
    return dict(tot, images=images, file=os.path.relpath(f, REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proposals", type=int, default=40, help="JLN proposals in the batch (4 frames x 10)")
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--pmc-dir", default=None,
                    help="tools/pmc_forwards.sh output: add the measured MFMA work issued and MFMA-busy share "
                         "of the same forwards to the P2PNet / CenterNet lines")
    args = ap.parse_args()
    import numpy as np
    import torch
    from fvp import _lib

    cnn_algo = None  # A/B: FVP_CONV_HALO=0 -> per-tap kernel only (FVP_CONV_SPLIT=0: never split)
    if os.environ.get("FVP_CONV_HALO") == "0":
        cnn_algo = 3 if os.environ.get("FVP_CONV_SPLIT") == "0" else 1

    import cnn_arch
    from fvp import cnn, synthetic

    dev = torch.device("cuda:0")
    J = 15
    p2p = cnn_arch.P2PNet(J, J).eval()
    p2p.load_state_dict(synthetic.seeded_state_dict(p2p, 11))
    cn = cnn_arch.CenterNet(J, 1).eval()
    cn.load_state_dict(synthetic.seeded_state_dict(cn, 12))
    p2p, cn = p2p.to(dev), cn.to(dev)
    g = torch.Generator().manual_seed(0)
    x_jln = torch.rand((3 * args.proposals, J, 64, 64), generator=g).to(dev)
    x_hdn = torch.rand((args.frames, J, 80, 80), generator=g).to(dev)
    f_p2p, f_cn = cnn.FvpCNN(p2p, algo=cnn_algo), cnn.FvpCNN(cn, algo=cnn_algo)
    b_p2p, b_cn = cnn.FvpCNN(p2p, torch.bfloat16), cnn.FvpCNN(cn, torch.bfloat16)

    def flops(plan_net, x, net=None):
        # count with the fvp layer descriptions: 2*M*N*K per conv (the front 7x7 layer counted
        # through its ConvLayer: net.front7, the NCHW front kernel, is off while counting)
        tot = 0
        orig = cnn.ConvLayer.__call__

        def counting(self, a, relu, res_pre=None, res_post=None, **kw):
            nonlocal tot
            tot += self.flops(a)
            return orig(self, a, relu, res_pre, res_post, **kw)
        cnn.ConvLayer.__call__ = counting
        front7 = getattr(net, "front7", None)
        if net is not None:
            net.front7 = None
        try:
            plan_net(x)
        finally:
            cnn.ConvLayer.__call__ = orig
            if net is not None:
                net.front7 = front7
        return tot

    def timeit(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(3):
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / args.iters)
        return float(np.median(ts))

    out = {}
    with torch.no_grad():
        for name, fv, bv, tv, x in (("p2pnet_jln", lambda: f_p2p(x_jln), lambda: b_p2p(x_jln),
                                     lambda: p2p(x_jln), x_jln),
                                    ("centernet_hdn", lambda: f_cn.from_xy(x_hdn), lambda: b_cn.from_xy(x_hdn),
                                     lambda: (cn.output_hm(cn.encoder_decoder(cn.front_layers(x_hdn))),), x_hdn)):
            p2p_line = name.startswith("p2p")
            fl = flops(f_p2p if p2p_line else (lambda t: f_cn.from_xy(t)), x, f_p2p if p2p_line else f_cn)
            t_f, t_t, t_b = timeit(fv), timeit(tv), timeit(bv)
            from fvp.graphs import CapturedStep
            t_g = timeit(CapturedStep(fv).replay)  # the same launches replayed from one hipGraph
            out[name] = {"images": int(x.shape[0]), "shape": list(x.shape[1:]), "gflop": round(fl / 1e9, 3),
                         "fvp_ms": round(t_f, 4), "torch_ms": round(t_t, 4),
                         "fvp_graph_ms": round(t_g, 4), "fvp_graph_tflops": round(fl / (t_g * 1e-3) / 1e12, 2),
                         "fvp_tflops": round(fl / (t_f * 1e-3) / 1e12, 2),
                         "mfma_frac_of_f32_peak": round(fl / (t_f * 1e-3) / 1e12 / MFMA_F32_PEAK_TF, 4),
                         "flops_counted": "direct convolution (Winograd layers issue fewer: mfma_issued)",
                         "speedup_vs_torch": round(t_t / t_f, 3),
                         "bf16_ms": round(t_b, 4), "bf16_tflops": round(fl / (t_b * 1e-3) / 1e12, 2),
                         "bf16_frac_of_bf16_peak": round(fl / (t_b * 1e-3) / 1e12 / 2500.0, 4)}
            pmc = _pmc_forward(args.pmc_dir, "p2p" if p2p_line else "centernet")
            if pmc:  # the measured MFMA work of the same network per image, at this line's time
                per_img = pmc["mfma_gflop_issued"] / pmc["images"]
                issued = per_img * int(x.shape[0])
                out[name]["mfma_issued"] = {
                    "gflop": round(issued, 3), "tflops": round(issued / (t_f * 1e-3) / 1e3, 2),
                    "frac_of_f32_peak": round(issued / (t_f * 1e-3) / 1e3 / MFMA_F32_PEAK_TF, 4),
                    "mfma_busy": pmc["mfma_busy"], "mfma_busy_per_sq_busy": pmc.get("mfma_busy_per_sq_busy"),
                    "source": f"{pmc['file']} (SQ_INSTS_VALU_MFMA_MOPS_F32 x 512 over {pmc['images']} images; "
                              "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE))"}
        # C2CNet on the K z-columns of every frame; WeightNet on the 3K joint-feature stacks
        c2c = cnn_arch.C2CNet(J, 1).eval()
        c2c.load_state_dict(synthetic.seeded_state_dict(c2c, 14))
        wn = cnn_arch.WeightNet(J).eval()
        wn.load_state_dict(synthetic.seeded_state_dict(wn, 15))
        c2c, wn = c2c.to(dev), wn.to(dev)
        x_col = torch.rand((args.frames * 10, J, 20), generator=g).to(dev)
        x_feat = torch.randn((3, args.proposals, J, 64, 64), generator=g).to(dev)
        f_c2c, f_wn = cnn.FvpCNN(c2c), cnn.FvpWeightNet(wn)
        fl = flops(lambda t: f_c2c(t), x_col)
        t_f, t_t = timeit(lambda: f_c2c(x_col)), timeit(lambda: c2c(x_col))
        from fvp.graphs import CapturedStep
        t_g = timeit(CapturedStep(lambda: f_c2c(x_col)).replay)
        out["c2cnet_hdn"] = {"columns": int(x_col.shape[0]), "shape": list(x_col.shape[1:]),
                             "gflop": round(fl / 1e9, 4), "fvp_ms": round(t_f, 4), "torch_ms": round(t_t, 4),
                             "fvp_graph_ms": round(t_g, 4),
                             "speedup_vs_torch": round(t_t / t_f, 3)}
        t_f, t_t = timeit(lambda: f_wn(x_feat)), timeit(lambda: wn(x_feat))
        nbytes = x_feat.numel() * 4
        out["weightnet_jln"] = {"maps": int(x_feat.shape[0] * x_feat.shape[1] * J), "shape": [64, 64],
                                "gflop_conv": round(2 * x_feat.numel() * 32 * 9 / 1e9, 3),
                                "fvp_ms": round(t_f, 4), "torch_ms": round(t_t, 4),
                                "fvp_gbs_input": round(nbytes / (t_f * 1e-3) / 1e9, 1),
                                "speedup_vs_torch": round(t_t / t_f, 3)}
    print(json.dumps({"metric": "HDN/JLN CNNs on fp32 MFMA (implicit GEMM, folded BN)", "peak_tflops_f32": MFMA_F32_PEAK_TF,
                      "note": "torch_ms = the same eval module on torch's GPU convolution (MIOpen); torch centernet "
                              "time covers the same layers (hm head only)", **out}))


if __name__ == "__main__":
    main()
