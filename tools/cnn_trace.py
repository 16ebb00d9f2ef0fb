#!/usr/bin/env python3
"""Kernel durations of one fvp CNN forward, per dispatch, from a rocprofv3
kernel trace (event-timed per-layer numbers, tools/cnn_layers.py, carry
~10 us of host/event overhead per layer and overstate small layers).

    # on the GPU box: trace --iters forwards of CenterNet at 8 images
    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cn -o run -- \
        python3 tools/cnn_trace.py run --net centernet --images 8 --algo auto
    # then: per-dispatch table of the last forward + per-forward totals
    python3 tools/cnn_trace.py parse gpurun_out/cn
    # PMC passes (tools/pmc.sh with PMC_CMD = the run leg): per-dispatch
    # counters of the last forward, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES over
    # (GRBM_GUI_ACTIVE / 8 XCDs) x 1024 SIMDs
    python3 tools/cnn_trace.py pmc gpurun_out/cn_pmc --per-forward 37

The run leg synchronises and sleeps 20 ms between forwards so the parser can
split the trace at the gaps.
"""
import argparse
import csv
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def run(args):
    import torch

    import cnn_arch
    from fvp import cnn, synthetic

    dev = torch.device("cuda:0")
    J = 15
    algo = {"auto": cnn.CONV_AUTO, "dma": cnn.CONV_DMA, "halo": cnn.CONV_HALO, "pertap": cnn.CONV_PER_TAP,
            "nosplit": cnn.CONV_PER_TAP_NOSPLIT}[args.algo]
    dt = torch.bfloat16 if args.bf16 else torch.float32
    if args.net == "backbone":  # PoseResNet-50 on --images views of the Panoptic IMAGE_SIZE (960 x 512)
        from fvp.backbone import FvpPoseResNet

        m = cnn_arch.PoseResNet(50, J).eval()
        m.load_state_dict(synthetic.seeded_state_dict(m, 21))
        f = FvpPoseResNet(m.to(dev), dt)
        x = torch.randn((args.images, 3, 512, 960), device=dev)
        fwd = lambda: f.forward_nhwc(x)  # noqa: E731
    elif args.net == "c2c":  # C2CNet on --images z-columns of 15 x --length
        m = cnn_arch.C2CNet(J, 1).eval()
        m.load_state_dict(synthetic.seeded_state_dict(m, 14))
        f = cnn.FvpCNN(m.to(dev), dt, algo=algo)
        x = torch.rand((args.images, J, args.length), device=dev)
        fwd = lambda: f(x)  # noqa: E731
    else:
        if args.net == "p2p":
            m, hw = cnn_arch.P2PNet(J, J).eval(), (64, 64)
        else:
            m, hw = cnn_arch.CenterNet(J, 1).eval(), (80, 80)
        m.load_state_dict(synthetic.seeded_state_dict(m, 11))
        f = cnn.FvpCNN(m.to(dev), dt, algo=algo)
        x = torch.rand((args.images, J) + hw, device=dev)
        fwd = (lambda: f(x)) if args.net == "p2p" else (lambda: f.from_xy(x))
    with torch.no_grad():
        for _ in range(args.iters):
            fwd()
            torch.cuda.synchronize()
            time.sleep(0.02)


def parse(args):
    files = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)
    assert files, f"no kernel_trace.csv under {args.dir}"
    rows = []
    for fn in files:
        with open(fn) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    iters, cur = [], []
    for r in rows:
        if cur and r[0] - cur[-1][1] > 5_000_000:  # a 5-ms gap: the sleep between forwards
            iters.append(cur)
            cur = []
        cur.append(r)
    if cur:
        iters.append(cur)
    iters = [it for it in iters if len(it) >= args.min_dispatches]
    last = iters[-1]
    busy = [sum(e - s for s, e, _ in it) / 1e3 for it in iters]
    span = [(it[-1][1] - it[0][0]) / 1e3 for it in iters]
    out = {"forwards": len(iters), "dispatches": len(last), "last_busy_us": round(busy[-1], 1),
           "last_span_us": round(span[-1], 1), "min_span_us": round(min(span[2:] or span), 1),
           "kernels": [[round((e - s) / 1e3, 2), n.split("(")[0][:90]] for s, e, n in last]}
    print(json.dumps(out))


def pmc(args):
    per = {}  # counter -> {dispatch id: (kernel, value)}
    for fn in glob.glob(os.path.join(args.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as fh:
            for r in csv.DictReader(fh):
                d = per.setdefault(r["Counter_Name"], {})
                k = int(r["Dispatch_Id"])
                name, v = d.get(k, (r["Kernel_Name"], 0.0))
                d[k] = (name, v + float(r["Counter_Value"]))
    rows = []
    for c, d in per.items():
        last = sorted(d)[-args.per_forward:]
        for i, k in enumerate(last):
            if len(rows) <= i:
                rows.append({"kernel": d[k][0].split("(")[0].replace("void ", "")[:80]})
            rows[i][c] = d[k][1]
    for r in rows:
        if "SQ_VALU_MFMA_BUSY_CYCLES" in r and r.get("GRBM_GUI_ACTIVE"):
            r["mfma_busy"] = round(r["SQ_VALU_MFMA_BUSY_CYCLES"] / (r["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
        if "SQ_WAVE_CYCLES" in r and r["SQ_WAVE_CYCLES"]:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in r:
                    r[c.lower()[3:] + "_frac"] = round(r[c] / r["SQ_WAVE_CYCLES"], 3)
        if r.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_conflict_frac"] = round(r.get("SQ_LDS_BANK_CONFLICT", 0) / r["SQ_LDS_IDX_ACTIVE"], 3)
    for r in rows:
        print(json.dumps(r))
    # the whole forward: MFMA busy over the GPU-active time of its dispatches (each
    # dispatch's GRBM_GUI_ACTIVE counts that dispatch), the ratio of MFMA-busy to
    # SQ-busy cycles as rocprofv3 sums them, and the MFMA work actually issued
    # (SQ_INSTS_VALU_MFMA_MOPS_F32 in units of 512 FLOPs) against the direct-conv
    # FLOPs that the TF/s figures of tools/bench_cnn.py count
    tot = {c: sum(r.get(c, 0.0) for r in rows) for c in
           ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_F32")}
    out = {"forward": True, "dispatches": len(rows), **{k: v for k, v in tot.items() if v}}
    if tot["GRBM_GUI_ACTIVE"]:
        out["mfma_busy"] = round(tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (tot["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
    if tot["SQ_BUSY_CYCLES"]:
        # SQ_BUSY_CYCLES counts per shader engine (32 on MI355X: 8 XCDs x 4), SQ_VALU_MFMA_BUSY_CYCLES
        # per SIMD (rocprofv3 --list-avail): the MFMA-busy share of the SIMD cycles in which the
        # engines had waves is the ratio over the 32 SIMDs of an engine
        out["mfma_busy_per_sq_busy"] = round(tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (tot["SQ_BUSY_CYCLES"] * 32), 4)
    if tot["SQ_INSTS_VALU_MFMA_MOPS_F32"]:
        out["mfma_gflop_issued"] = round(tot["SQ_INSTS_VALU_MFMA_MOPS_F32"] * 512 / 1e9, 3)
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--net", choices=["p2p", "centernet", "c2c", "backbone"], default="centernet")
    r.add_argument("--length", type=int, default=20, help="c2c: column length Z")
    r.add_argument("--images", type=int, default=8)
    r.add_argument("--bf16", action="store_true")
    r.add_argument("--algo", choices=["auto", "dma", "halo", "pertap", "nosplit"], default="auto")
    r.add_argument("--iters", type=int, default=8)
    p = sub.add_parser("parse")
    p.add_argument("dir")
    p.add_argument("--min-dispatches", type=int, default=3,
                   help="groups with fewer dispatches are setup work, not forwards (1 for the one-launch C2CNet)")
    m = sub.add_parser("pmc")
    m.add_argument("dir")
    m.add_argument("--per-forward", type=int, default=37)
    args = ap.parse_args()
    {"run": run, "parse": parse, "pmc": pmc}[args.cmd](args)


if __name__ == "__main__":
    main()
