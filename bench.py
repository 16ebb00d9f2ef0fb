#!/usr/bin/env python3
"""Voxelize+project throughput benchmark (BASELINE.json metric).

One step = the hot path over one batch of B synthetic frames per GPU, inputs
resident in HBM:
  fvp_voxelize (cube [B,J,X,Y,Z] + xy max-plane, one launch)
  -> fvp_nms_topk_columns: NMS top-K on the root-joint xy plane (stand-in for
     CenterNet's map) and the winners' z-columns [B,K,J,Z] in one launch
  -> (N > 1) one RCCL all_gather of the compact proposals (the NMS writes them
     into one buffer, sent as it is; at N = 1 there is nothing to exchange).
Frames are sharded across ranks (weak scaling).  Default workload: C2 =
BASELINE configs[1] (Shelf calibration, 5 cams, J=15, 128x240 -> 80x80x20).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    torchrun --nproc-per-node N bench.py --gpus N ...

Without a launcher, `--gpus N > 1` starts `python -m torch.distributed.run
--nproc-per-node N` on this same command line as a child process (this process
never touches the GPU), relays rank 0's JSON line and exits with the child's
status.  Under a launcher `--gpus` must equal WORLD_SIZE.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "faster-voxelpose_amd"))

METRIC = "voxelize+project FPS (5 cams, 80×80×20 grid) @1/2/4/8 GPU; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# the fvp_voxelize op: layout pass (fp32 channels-last, fp16 pair table per 8 entries, per row or per
# entry) + gather
LAYOUT_KERNELS = ("heatmaps_to_cl_kernel", "pairs_vec8_kernel", "heatmaps_to_pairs_kernel", "pairs_rows_kernel")
GATHER_KERNELS = ("voxelize_kernel", "voxelize_cams_kernel")
VOX_KERNELS = LAYOUT_KERNELS + GATHER_KERNELS
# The gather's tap-instruction floor: one wave-load (64 lanes x 16 B = 1 KiB) costs
# 16.5 cycles of a CU's vector-memory path whether its lanes hit L1, miss, or are
# off-image (tools/gather_probe.hip replay of the C2 gather: TAPS_ALL_OOB = 34.5 us
# per 8 frames = 1.28 M wave-loads over 256 CUs at 2.4 GHz;
# profiles/round3/gather_probe_c2_modes.jsonl, DESIGN.md §5 "The C2 ceiling").
TAP_CYCLES_PER_WAVELOAD = 16.5
TAP_PROBE = "profiles/round3/gather_probe_c2_modes.jsonl (TAPS_ALL_OOB)"
CUS, CLOCK_HZ = 256, 2.4e9
JOINT_SLICE = 32  # fvp_voxelize's joints per slice (kJointSlice)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None, help="frames per GPU per step (default per workload)")
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--traffic", choices=["auto", "off"], default="auto",
                    help="collect FETCH_SIZE/WRITE_SIZE with rocprofv3 child runs (N=1, rank 0)")
    ap.add_argument("--cpu-baseline", choices=["on", "off"], default="on")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="the CPU baseline's pool-share line (default: OMP_NUM_THREADS)")
    ap.add_argument("--graph", choices=["on", "off"], default="off",
                    help="replay the GPU-local part of the step from captured hipGraphs (the collective stays eager)")
    ap.add_argument("--slabs", action="store_true",
                    help="large-frame mode (SURVEY.md §8(e)): every rank holds the same frames and voxelises one "
                         "x-slab of each; strong scaling")
    ap.add_argument("--strong", action="store_true",
                    help="--batch is the whole job's frames, split over the ranks (strong scaling)")
    ap.add_argument("--heatmap-layout", choices=["planar", "channels-last"], default="planar",
                    help="planar: the reference's [B,V,J,H,W] heatmaps (the headline); channels-last: "
                         "[B,V,H,W,Cp] as the fvp backbone writes them (no layout pass)")
    ap.add_argument("--on-the-fly", choices=["auto", "on", "off"], default="auto",
                    help="sampling coordinates from the cached grid (off) or projected in-kernel (on)")
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# `--gpus N` without a launcher: spawn one.  Nothing here may initialise the
# GPU (a process that has initialised it must not be replaced, and its ranks
# need the devices): no torch import, the device count comes from a child.
def visible_gpus():
    """GPUs a rank could use, counted in a child process (torch.cuda.device_count
    there; this process stays GPU-free).  FVP_BENCH_VISIBLE_GPUS overrides (tests)."""
    if os.environ.get("FVP_BENCH_VISIBLE_GPUS", "").isdigit():
        return int(os.environ["FVP_BENCH_VISIBLE_GPUS"])
    out = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                         capture_output=True, text=True, timeout=300)
    try:
        return int(out.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        raise SystemExit(f"bench: could not count the visible GPUs: {out.stderr.strip()[-300:]}")


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(argv, n, port):
    """(argv, env) of the torch.distributed.run child that runs this benchmark as
    n ranks on this node (rendezvous on 127.0.0.1; dmabuf IPC for RCCL)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return cmd, env


def check_world(args, env=None):
    """Under a launcher (WORLD_SIZE set) --gpus must equal WORLD_SIZE."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" in env and not args.child and args.gpus != int(env["WORLD_SIZE"]):
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={env['WORLD_SIZE']} ranks")


def maybe_launch(argv, json_out, popen=subprocess.Popen):
    """If this is a bare `bench.py --gpus N` (N > 1, no WORLD_SIZE), run the
    benchmark as N ranks in a torch.distributed.run child, relay rank 0's JSON
    line to `json_out` and return the child's exit status; else return None."""
    args = parse(argv)
    if "WORLD_SIZE" in os.environ or args.child or args.gpus <= 1:
        return None
    gloo = os.environ.get("FVP_BENCH_BACKEND", "nccl") == "gloo"
    if not gloo:
        ndev = visible_gpus()
        if args.gpus > ndev:
            raise SystemExit(f"bench: --gpus {args.gpus} but {ndev} visible GPU(s); one rank per GPU "
                             f"(FVP_BENCH_BACKEND=gloo for a shared-device rehearsal)")
    cmd, env = launcher_command(argv, args.gpus, free_port())
    note(f"launching {args.gpus} ranks: {' '.join(cmd[1:])}")
    proc = popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    import signal

    def forward(signum, _frame):
        proc.send_signal(signum)

    old = {s: signal.signal(s, forward) for s in (signal.SIGTERM, signal.SIGINT)}
    lines = 0
    try:
        for ln in proc.stdout:
            s = ln.strip()
            if s.startswith("{") and s.endswith("}"):
                print(s, file=json_out, flush=True)  # rank 0's result line (only rank 0 prints one)
                lines += 1
            elif s:
                print(ln.rstrip("\n"), file=sys.stderr, flush=True)
        rc = proc.wait()
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    if rc == 0 and lines != 1:
        note(f"expected one JSON line from rank 0, got {lines}")
        return 1
    return rc


# ---------------------------------------------------------------------------
CHILD_OPS = 4  # warmup + steps of a profiled child run
WORKLOAD_DESC = {"c1": "BASELINE configs[0] (1 demo camera)", "c2": "BASELINE configs[1] Shelf jln64 geometry",
                 "c3": "BASELINE configs[2] Panoptic demo cameras", "c4": "BASELINE configs[3] Panoptic 128x128x32",
                 "c5": "BASELINE configs[4] stress: 31 ring cameras, fp16 heatmaps",
                 "shelf_native": "Shelf native J=17 152x200"}
DEFAULT_BATCH = {"c1": 256, "c2": 256, "c3": 256, "c4": 64, "c5": 8, "shelf_native": 256}


def traffic_from_csvs(fetch_csvs, write_csvs, ops):
    """Per-op HBM bytes of the fvp_voxelize op from rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE counter CSVs (KB per dispatch), split into the layout pass and the
    gather.  Which FETCH correction each gets (MI355X_MICROARCH.md §HBM):
    * the layout pass is a wide coalesced stream (16 B per lane, whole lines): the
      guide's calibrated case, where FETCH_SIZE reads exactly half the bytes -> x2;
    * the gather's loads are scattered 16-B lanes (4 lanes of a voxel share one
      64-B pixel): the guide leaves other access widths uncalibrated, so its fetch
      is reported raw (x1, `traffic`) and doubled (`traffic_upper`) -- the true
      value lies between.
    Returns None if a counter has no rows for these kernels."""
    out = {}
    for counter, files in (("FETCH_SIZE", fetch_csvs), ("WRITE_SIZE", write_csvs)):
        tot = {"layout": 0.0, "gather": 0.0}
        rows = 0
        for f in files:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if row.get("Counter_Name") != counter:
                        continue
                    name = row.get("Kernel_Name", "")
                    kind = ("layout" if any(k in name for k in LAYOUT_KERNELS) else
                            "gather" if any(k in name for k in GATHER_KERNELS) else None)
                    if kind:
                        tot[kind] += float(row["Counter_Value"]) * 1024.0 / ops  # KB per dispatch -> B per op
                        rows += 1
        if not rows:
            return None
        out[counter] = tot
    f, w = out["FETCH_SIZE"], out["WRITE_SIZE"]
    layout = 2.0 * f["layout"] + w["layout"]
    return {"layout_fetch_raw": f["layout"], "layout_write": w["layout"], "layout": layout,
            "layout_fetch_correction": 2.0,
            "gather_fetch_raw": f["gather"], "gather_write": w["gather"],
            "gather": f["gather"] + w["gather"], "gather_fetch_correction": "1 (raw; uncalibrated width) .. 2",
            "traffic": layout + f["gather"] + w["gather"],
            "traffic_upper": layout + 2.0 * f["gather"] + w["gather"]}


def collect_traffic(args):
    """Run this benchmark twice under rocprofv3 (one counter pass each, as
    MI355X_MICROARCH.md prescribes) BEFORE this process touches the GPU, and
    return per-op HBM bytes of the voxelize op's layout pass and gather."""
    out_root = os.path.join(REPO, "gpurun_out", "bench_pmc")
    os.makedirs(out_root, exist_ok=True)
    files = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix=f"pmc_{counter}_", dir=out_root)
        cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run", "--",
               sys.executable, os.path.abspath(__file__), "--child", "--steps", str(CHILD_OPS - 1), "--warmup", "1",
               "--workload", args.workload, "--traffic", "off", "--cpu-baseline", "off",
               "--heatmap-layout", args.heatmap_layout, "--on-the-fly", args.on_the_fly]
        if args.batch:
            cmd += ["--batch", str(args.batch)]
        if args.slabs:
            cmd += ["--slabs"]
        try:
            subprocess.run(cmd, check=True, timeout=240, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           cwd=REPO)
        except Exception as e:  # profiler unavailable or failed: report null, never fake
            return None, f"rocprofv3 {counter} failed: {e}"
        files[counter] = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    t = traffic_from_csvs(files["FETCH_SIZE"], files["WRITE_SIZE"], CHILD_OPS)
    if t is None:
        return None, f"no FETCH_SIZE / WRITE_SIZE rows for {VOX_KERNELS}"
    t["csv_dirs"] = [os.path.relpath(os.path.dirname(v[0]), REPO) for v in files.values() if v]
    return t, None


def lanes_per_voxel(J):
    """fvp_layout.h lanes_per_voxel: 16-B lanes per voxel of a joint slice."""
    return 1 if J <= 4 else 2 if J <= 8 else 4 if J <= 16 else 8


def tap_floor_ceiling(n_vox, V, J, H, W, elem, layout_pass, copy_gbs, alg_per_frame):
    """The design ceiling the roofline fraction is measured against:
    the gather's tap-instruction floor -- wave-loads x 16.5 cycles over 256 CUs,
    TAP_PROBE -- plus, for planar input, the layout pass at the measured copy
    rate (it reads the planar heatmaps and writes the channels-last / pixel-pair
    table).  Cube stores, L1/L2 misses and setup are taken as free, so this
    bounds the achievable HBM fraction from above.  Per frame."""
    wave_loads = 0.0
    layout_bytes = 0.0
    for j0 in range(0, J, JOINT_SLICE):
        js = min(JOINT_SLICE, J - j0)
        lpv = lanes_per_voxel(js)
        pairs = elem == 2 and js <= 16
        # per voxel-camera: 4 taps (fp32: one 16-B load per lane per tap) or 2 rows
        # (fp16 pixel pairs: both x taps of a row in one 16-B lane load)
        wave_loads += n_vox * V * (2 if pairs else 4) * lpv * 16 / 1024.0
        if layout_pass:
            table = V * H * (W + 1) * 64 if pairs else V * H * W * 4 * lpv * 4
            layout_bytes += V * js * H * W * elem + table
    t_taps = wave_loads * TAP_CYCLES_PER_WAVELOAD / (CUS * CLOCK_HZ)
    t_layout = layout_bytes / (copy_gbs * 1e9) if (layout_pass and copy_gbs) else 0.0
    # (the HBM roof itself bounds the op where the taps are few: C1's one camera)
    t = max(t_taps + t_layout, alg_per_frame / (HBM_PEAK_GBS * 1e9))
    frac = alg_per_frame / t / (HBM_PEAK_GBS * 1e9)
    return {"frac": round(frac, 4),
            "us_per_frame": round(t * 1e6, 3), "tap_floor_us_per_frame": round(t_taps * 1e6, 3),
            "layout_us_per_frame": round(t_layout * 1e6, 3), "wave_loads_per_frame": round(wave_loads),
            "layout_bytes_per_frame": round(layout_bytes),
            "what": ("tap-instruction floor (16.5 cycles per 1-KiB wave-load, " + TAP_PROBE + ")"
                     + (" + layout pass at the measured copy rate" if layout_pass else "")
                     + "; stores and L1/L2 misses free: an upper bound on frac"
                     + (" (the north star's >= 0.60 lies above it)" if frac < 0.6 else ""))}


def rank_stats(values, device):
    """Every rank's `values` (a list of floats) -> [world][len(values)] on every
    rank (one all-reduce of a zero-padded row per rank; gloo and RCCL alike)."""
    import torch
    import torch.distributed as dist

    world, rank = dist.get_world_size(), dist.get_rank()
    t = torch.zeros((world, len(values)), dtype=torch.float64, device=device)
    t[rank] = torch.tensor(values, dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return t.cpu().tolist()


def host_cores():
    """(physical cores of the host per lscpu, logical CPUs this process may run on)."""
    phys = None
    try:
        out = subprocess.run(["lscpu", "-p=CORE,SOCKET"], capture_output=True, text=True, timeout=10).stdout
        phys = len({ln for ln in out.splitlines() if ln and not ln.startswith("#")}) or None
    except Exception:
        pass
    return phys, len(os.sched_getaffinity(0))


def cgroup_cpu_limit():
    """The cgroup v2 CPU quota of this process ("max" or "<quota> <period>"), or None."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                return f.read().strip()
        except OSError:
            pass
    return None


def cpu_quota_cpus(limit):
    """CPUs' worth of time the quota allows (None when unlimited / unknown)."""
    if not limit or limit.startswith("max"):
        return None
    try:
        q, per = limit.split()[:2]
        return int(q) / int(per)
    except ValueError:
        return None


def cpu_baseline_run(w, sample_grid_cpu, threads, runs=10, warmup=2, budget_s=30.0):
    """Reference op sequence on the host cores (oracle/torch_cpu.py): `warmup`
    untimed calls, then the median of `runs` timed calls of 4 frames each
    (SURVEY.md §8(d)); fewer runs only if one call would blow `budget_s`."""
    import numpy as np
    import torch
    from fvp import synthetic
    from oracle import torch_cpu

    torch.set_num_threads(threads)
    frames = 4
    hm = torch.from_numpy(synthetic.gaussian_heatmaps(w, frames, first_frame=10_000))
    for _ in range(warmup):
        t0 = time.perf_counter()
        torch_cpu.hot_path(hm, sample_grid_cpu, w.voxels_per_axis, w.max_people)
        one = time.perf_counter() - t0
    runs = max(3, min(runs, int(budget_s / max(one, 1e-6))))
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        torch_cpu.hot_path(hm, sample_grid_cpu, w.voxels_per_axis, w.max_people)
        ts.append(time.perf_counter() - t0)
    return frames / float(np.median(ts)), frames, runs


def cpu_baseline(w, sample_grid_cpu, threads_req):
    """the reference's CPU op order timed on the box's host
    cores -- at every physical core, at 8 threads (the survey container's
    count), and at the pool's per-GPU share (OMP_NUM_THREADS).  A cgroup CPU
    quota is recorded as found; where it caps the process below the physical
    core count, the all-core line runs at the quota's CPUs instead (more
    threads than the quota only queue)."""
    phys, avail = host_cores()
    limit = cgroup_cpu_limit()
    quota = cpu_quota_cpus(limit)
    share = threads_req or (int(os.environ["OMP_NUM_THREADS"]) if os.environ.get("OMP_NUM_THREADS", "").isdigit()
                            else avail)
    all_cores = min(x for x in (phys or avail, avail, int(quota) if quota else 10 ** 9) if x)
    lines = {}
    for tag, th in (("all_cores", all_cores), ("8_threads", 8), ("pool_share", share)):
        if th in [v["threads"] for v in lines.values()]:
            lines[tag] = dict(next(v for v in lines.values() if v["threads"] == th))
            continue
        fps, frames, runs = cpu_baseline_run(w, sample_grid_cpu, th)
        lines[tag] = {"threads": th, "frames_per_s": round(fps, 2), "runs": runs}
    # the reported value is the fastest measured thread count (the baseline most
    # favourable to the CPU); on the pool the cgroup quota (cgroup_cpu_max) caps
    # the process at 16 CPUs, where 16 threads ran slower than 8
    main_line = max(lines.values(), key=lambda v: v["frames_per_s"])
    return {"value": main_line["frames_per_s"], "unit": "frames/s", "cores": main_line["threads"], "kind": "port",
            "value_all_cores": lines["all_cores"]["frames_per_s"], "all_cores_threads": lines["all_cores"]["threads"],
            "host_physical_cores": phys, "host_logical_cpus_available": avail, "cgroup_cpu_max": limit,
            "value_8_threads": lines["8_threads"]["frames_per_s"],
            "value_pool_share": lines["pool_share"]["frames_per_s"], "pool_share_threads": share,
            "sample": f"{w.name}, 4 frames per call, 2 warm-up calls then the median of {main_line['runs']} timed calls "
                      f"per thread count: torch-CPU restatement of project_whole.forward (per-frame F.grid_sample, "
                      f"mean, clamp) + max(dim=4) + nms2D + column gather (oracle/torch_cpu.py), sample grid prebuilt"}


def roofline_fields(kernel, alg_bytes, kernel_ms_per_rank, kernel_ms_steps, traffic, copy_gbs, taps, tap_bytes,
                    ceiling):
    """The line's `roofline` object.  kernel_ms is the SLOWEST rank's mean op time
    (every rank processes the same per-rank algorithmic bytes), so achieved / frac
    describe the slowest GPU; rank 0's and every rank's times are listed."""
    ms = max(kernel_ms_per_rank)
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    tap_peak = CUS * CLOCK_HZ * 64 / tap_bytes / 1e12
    tap_rate = taps / (ms * 1e-3) / 1e12
    r = {
        "bound": "hbm",
        "kernel": kernel,
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": None if traffic is None else round(traffic["traffic"]),
        "algorithmic_bytes_per_launch": alg_bytes,
        "kernel_ms": round(ms, 4),
        "kernel_ms_rank0": round(kernel_ms_per_rank[0], 4),
        "kernel_ms_per_rank": [round(v, 4) for v in kernel_ms_per_rank],
        "slowest_rank": int(max(range(len(kernel_ms_per_rank)), key=lambda i: kernel_ms_per_rank[i])),
        "kernel_ms_steps": kernel_ms_steps,  # timed steps that carried the event pair (every steps // 50-th)
        "measured_copy_gbs": round(copy_gbs or 0.0, 1),
        "frac_of_measured_copy": round(achieved / copy_gbs, 4) if copy_gbs else None,
        "tap_rate": {"bound": "vector-memory 64 B/clk/CU", "achieved": round(tap_rate, 3),
                     "peak": round(tap_peak, 3), "unit": "T joint-taps/s",
                     "frac": round(tap_rate / tap_peak, 4), "joint_taps_per_launch": taps},
    }
    if ceiling is not None:
        r["ceiling"] = dict(ceiling)
        r["frac_of_ceiling"] = round(r["frac"] / ceiling["frac"], 4)
    if traffic is not None:
        r["traffic_detail"] = {k: (round(v, 1) if isinstance(v, float) else v) for k, v in traffic.items()}
        r["traffic_upper"] = round(traffic["traffic_upper"])
    return r


def note(msg):
    """Progress on stderr (long runs must keep writing; stdout holds only the JSON line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------
# The step's sharding and its GPU-local / collective parts, importable so that
# tests/test_bench_step_gloo.py runs this exact code at world 2 and 3 over gloo
# with the CPU oracle as the compute (the driver's SCALE run executes it over
# RCCL with the HIP ops).
def shard_plan(world, rank, batch, X, slabs=False, strong=False):
    """(frames per rank, the rank's first frame of the job, x0, x1) of one step.

    weak (default): every rank takes `batch` frames, rank r frames
    [r*batch, (r+1)*batch) of the job; --strong: `batch` is the job's frames,
    split evenly; --slabs: every rank holds the same `batch` frames and
    voxelises x-rows [x0, x1) of each (SURVEY.md §8(e) large-frame mode)."""
    from fvp import parallel

    B = batch
    if strong and not slabs:  # fixed total frames: each rank takes its shard
        if B % world:
            raise ValueError(f"--strong: {B} frames do not split evenly over {world} ranks")
        B //= world
    first = 0 if slabs else parallel.shard_frames(world * B, world, rank)[0]
    x0, x1 = parallel.shard_slab(X, world, rank) if slabs else (0, X)
    return B, first, x0, x1


class HipCompute:
    """The step's compute on the HIP ops (fvp.project_whole / fvp.proposal)."""

    def __init__(self, layer, cams, rt):
        self.layer, self.cams, self.rt = layer, cams, rt

    def voxelize(self, hm, meta, x0=None, x1=None):
        if x0 is None:
            return self.layer.forward_fused(hm, meta, self.cams, self.rt, want_cube=True, want_xy=True)
        return self.layer.forward_slab(hm, meta, self.cams, self.rt, x0, x1, want_cube=True, want_xy=True)

    @staticmethod
    def nms2D(prob, K):
        from fvp.proposal import nms2D
        return nms2D(prob, K)

    @staticmethod
    def nms2D_columns(prob, K, cube):
        from fvp.proposal import nms2D_columns
        return nms2D_columns(prob, K, cube)

    @staticmethod
    def gather_columns(cube, flat):
        from fvp.proposal import gather_columns
        return gather_columns(cube, flat)


def step_functions(compute, hm, meta, x0, x1, X, world, grouped, slabs, root, K):
    """vox() -> (cube, xy); post(cube, xy) -> (vals, flat, cols); collect(vals, flat)
    -> every rank's proposals or None.  One step = vox, post, collect."""
    from fvp import parallel

    def vox():
        return compute.voxelize(hm, meta, x0, x1) if slabs else compute.voxelize(hm, meta)

    def post(cube, xy):
        if slabs and world > 1:  # xy slabs -> full planes; owned columns -> one all-reduce
            xy = parallel.gather_xy_slabs(xy, X)
            vals, idx, flat = compute.nms2D(xy[:, root:root + 1], K)
            return vals, flat, parallel.columns_from_slab(cube, flat, x0, gather=compute.gather_columns)
        vals, idx, flat, cols = compute.nms2D_columns(xy[:, root:root + 1], K, cube)  # one launch
        return vals, flat, cols

    def collect(vals, flat):
        if grouped and not slabs:  # the one collective: compact proposals of every rank's frames (RCCL over xGMI)
            return parallel.gather_proposals(vals, flat)
        return None

    return vox, post, collect


def run_step(run_vox, run_post, collect, after_vox=None):
    cube, xy = run_vox()
    if after_vox is not None:
        after_vox()
    vals, flat, cols = run_post(cube, xy)
    return vals, flat, cols, collect(vals, flat)


def main():
    # stdout carries only the JSON line: native libraries (RCCL prints a version
    # banner when a communicator comes up) write to fd 1 directly, so fd 1 points
    # at stderr until the result is printed
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    rc = maybe_launch(sys.argv[1:], json_out)
    if rc is not None:
        json_out.close()
        raise SystemExit(rc)
    args = parse()
    check_world(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    traffic, traffic_note = None, None
    if args.traffic == "auto" and world == 1 and not args.child:
        note("traffic counters (two rocprofv3 child runs)")
        traffic, traffic_note = collect_traffic(args)  # before any GPU use in this process

    import numpy as np
    import torch
    import torch.distributed as dist

    from fvp import geometry, synthetic
    from fvp.project_whole import ProjectLayer
    from fvp.proposal import nms2D_columns
    from fvp.workloads import WORKLOADS

    # FVP_BENCH_BACKEND=gloo: plumbing rehearsal of N ranks that may share a
    # device (not a measurement; labelled as such).  Otherwise one rank per GPU
    # over RCCL, and more ranks than GPUs is an error, never a silent wrap.
    # One process group at every N (a one-rank RCCL group when launched without
    # torchrun), so the timed step runs the same all-gather code at N = 1.
    backend = os.environ.get("FVP_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend != "gloo" and (world > ndev or local_rank >= ndev):
        raise SystemExit(f"bench: {world} ranks (local rank {local_rank}) but {ndev} visible GPU(s); "
                         f"one rank per GPU (FVP_BENCH_BACKEND=gloo for a shared-device rehearsal)")
    local_rank %= max(1, ndev)  # (gloo rehearsal only: ranks share devices)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    pg_kw = {"device_id": dev} if backend == "nccl" else {}
    if world > 1 or "MASTER_ADDR" in os.environ:
        dist.init_process_group(backend, **pg_kw)
    elif not args.child:
        fd, store_path = tempfile.mkstemp(prefix="fvp_bench_pg_")
        os.close(fd)
        # (the FileStore removes its file when the group is destroyed; unlinking it
        # earlier makes the store's cleanup at exit wait forever)
        dist.init_process_group(backend, store=dist.FileStore(store_path, 1), rank=0, world_size=1, **pg_kw)
    grouped = dist.is_initialized()
    pg_backend = dist.get_backend() if grouped else None
    collective = {"nccl": "RCCL", "gloo": "gloo"}.get(pg_backend, str(pg_backend))
    rehearsal = pg_backend == "gloo"
    n_devices = min(world, ndev) if rehearsal else world  # distinct GPUs doing the work

    w = WORKLOADS[args.workload]
    try:
        B, first, x0, x1 = shard_plan(world, rank, args.batch or DEFAULT_BATCH.get(args.workload, 64),
                                      w.voxels_per_axis[0], args.slabs, args.strong)
    except ValueError as e:
        raise SystemExit(str(e))
    cams, seq = w.cameras()
    V = len(cams[seq])
    J = w.num_joints
    X, Y, Z = w.voxels_per_axis
    Wd, Hd = w.heatmap_size
    K = w.max_people
    root = 2 if J > 2 else 0

    layer = ProjectLayer(w.cfg(str(dev)))
    layer.verbose = False
    layer.on_the_fly = {"auto": None, "on": True, "off": False}[args.on_the_fly]
    rt = torch.as_tensor(geometry.resize_transform(w.ori_image_size, w.image_size), dtype=torch.float).to(dev)
    # large-frame mode: all ranks hold the same frames (x-slabs); otherwise own frames
    hm_host = synthetic.gaussian_heatmaps(w, B, first_frame=first)
    hm = torch.from_numpy(hm_host).to(dev)
    if w.dtype == "float16":  # C5: fp16 heatmaps (computed in fp32 by the kernels)
        hm = hm.half()
    del hm_host
    meta = {"seq": [seq] * B}

    def channels_last(planar):
        """[B,V,J,H,W] -> ChannelsLastHeatmaps [B,V,H,W,Cp] (the fvp backbone's output layout)."""
        from fvp.heatmaps import ChannelsLastHeatmaps

        cp = 16 * ((J + 15) // 16)
        t = torch.zeros(planar.shape[:2] + planar.shape[3:] + (cp,), dtype=torch.float32, device=dev)
        t[..., :J] = planar.permute(0, 1, 3, 4, 2)
        return ChannelsLastHeatmaps(t, J)

    hm_planar = hm
    if args.heatmap_layout == "channels-last":
        if hm.dtype != torch.float32:
            raise SystemExit("--heatmap-layout channels-last: fp32 heatmaps only")
        hm = channels_last(hm)

    # once-per-sequence cache build, timed separately (excluded from the step):
    # the first call also pays the library / code-object load; a second
    # sequence (same cameras, new key) times the grid build alone
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    layer.prepare(hm, meta, cams, rt)
    torch.cuda.synchronize()
    first_ms = (time.perf_counter() - t0) * 1e3
    seq_b = seq + "#second"
    cams_b = {seq_b: cams[seq]}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    layer.prepare(hm_planar[:1], {"seq": [seq_b]}, cams_b, rt)
    e1.record()
    torch.cuda.synchronize()
    cache_ms = {"first_call_ms": round(first_ms, 2), "sequence_build_ms": round((time.perf_counter() - t0) * 1e3, 3),
                "sequence_build_gpu_ms": round(e0.elapsed_time(e1), 3),
                "what": "grid" if not layer._project_on_the_fly(V) else "camera records (on-the-fly projection)"}

    stream = torch.cuda.current_stream(dev)
    ev = []

    vox, post, collect = step_functions(HipCompute(layer, cams, rt), hm, meta, x0, x1, X, world, grouped,
                                        args.slabs, root, K)

    if args.graph == "on" and args.slabs and world > 1:
        raise SystemExit("--graph on captures GPU-local work only; the slab collectives sit inside post()")
    if args.graph == "on":  # two hipGraphs: the voxelize op (timed on its own) and NMS + columns
        from fvp.graphs import CapturedStep

        cap_vox = CapturedStep(vox)
        cap_post = CapturedStep(lambda: post(*cap_vox.outputs))
        run_vox, run_post = cap_vox.replay, lambda cube, xy: cap_post.replay()
    else:
        run_vox, run_post = vox, post

    pool = []  # timing events, created before the timed region (creation is a HIP call per event)

    def step(record):
        if record:
            e0, e1 = pool.pop() if pool else (torch.cuda.Event(enable_timing=True),
                                              torch.cuda.Event(enable_timing=True))
            e0.record(stream)
            ev.append((e0, e1))
        return run_step(run_vox, run_post, collect, after_vox=(lambda: e1.record(stream)) if record else None)[2]

    note(f"warmup {args.warmup} + {args.steps} timed steps of {B} frames")
    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if grouped:
        dist.barrier()
    # the op's HIP-event pair (roofline kernel_ms) on at most ~50 of the timed steps: each record is a
    # marker in the stream, ~5 % of a C3 B=8 step (profiles/round5/c3_b8/event_sampling.txt)
    rec_every = max(1, args.steps // 50)
    pool.extend((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(args.steps))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i % rec_every == 0)
    torch.cuda.synchronize()
    if grouped:
        dist.barrier()
    el = time.perf_counter() - t0
    vox_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    # every rank's wall time and op time: the job's time is the slowest rank's,
    # and so is the roofline's kernel time (the line describes the slowest GPU)
    per_rank = [[el, vox_ms]]
    if grouped and world > 1:
        per_rank = rank_stats([el, vox_ms], "cpu" if pg_backend == "gloo" else dev)
    el = max(r[0] for r in per_rank)
    if args.child:
        if grouped:
            dist.destroy_process_group()
        return

    frames = (1 if args.slabs else world) * B * args.steps
    fps = frames / el
    Xs = x1 - x0  # this rank's x-rows (X unless --slabs)
    # (channels-last input: the J joints' bytes are counted, not the zero padding)
    per_frame = V * J * Hd * Wd * hm_planar.element_size() + J * Xs * Y * Z * 4 + J * Xs * Y * 4
    alg_bytes = B * per_frame
    # secondary bound: the bilinear tap rate, N*V*J*4 joint-taps
    # per frame, against the per-CU vector-memory (texture addresser / L1) rate of
    # 64 B/clk: 16 fp32 joint-taps/clk/CU, 32 with the fp16 pixel-pair table.
    taps = B * Xs * Y * Z * V * J * 4
    tap_bytes = 2 if (hm_planar.element_size() == 2 and J <= 16) else 4

    extra = {}
    if rank == 0:
        # measured copy bandwidth: fvp_copy_f4 (float4 streaming copy, 1 GiB each
        # way, csrc/fvp_copy.hip) on this stream; and the one-frame latency of
        # the step; both outside the timed region
        from fvp import _lib

        nbytes = 1 << 30
        src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).fill_(1.0)
        dst = torch.empty_like(src)
        cs = torch.cuda.current_stream(dev).cuda_stream
        _lib.call("fvp_copy_f4", src.data_ptr(), dst.data_ptr(), nbytes, cs)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            _lib.call("fvp_copy_f4", src.data_ptr(), dst.data_ptr(), nbytes, cs)
        e1.record()
        torch.cuda.synchronize()
        extra["copy_gbs"] = 2 * nbytes * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9
        del src, dst
        # the same voxelize op on channels-last heatmaps (as the fvp backbone
        # writes them: the gather alone, no layout pass), same frames and events
        if args.heatmap_layout == "planar" and hm_planar.dtype == torch.float32 and not args.slabs:
            hcl = channels_last(hm_planar)
            for _ in range(2):
                layer.forward_fused(hcl, meta, cams, rt)
            evs = []
            for _ in range(args.steps):
                a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                layer.forward_fused(hcl, meta, cams, rt)
                b_.record(stream)
                evs.append((a, b_))
            torch.cuda.synchronize()
            cl_ms = float(np.mean([a.elapsed_time(b_) for a, b_ in evs]))
            cl_frac = alg_bytes / (cl_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
            cl_ceiling = tap_floor_ceiling(Xs * Y * Z, V, J, Hd, Wd, 4, False, None, per_frame)
            extra["channels_last"] = {"kernel_ms": round(cl_ms, 4),
                                      "achieved": round(alg_bytes / (cl_ms * 1e-3) / 1e9, 1),
                                      "frac": round(cl_frac, 4),
                                      "ceiling_frac": cl_ceiling["frac"],
                                      "frac_of_ceiling": round(cl_frac / cl_ceiling["frac"], 4),
                                      "frames_per_s_op_only": round(B / (cl_ms * 1e-3), 1),
                                      "what": "the same op on [B,V,H,W,16] heatmaps as fvp.backbone writes them "
                                              "(fvp_voxelize_cl: no layout pass); bit-identical outputs"}
            del hcl
        hm1, meta1 = (hm_planar[:1] if args.heatmap_layout == "planar" else channels_last(hm_planar[:1])), \
            {"seq": [seq]}

        def step1():
            cube, xy = layer.forward_fused(hm1, meta1, cams, rt, want_cube=True, want_xy=True)
            return nms2D_columns(xy[:, root:root + 1], K, cube)[3]

        for _ in range(3):
            step1()
        torch.cuda.synchronize()
        lat = []
        for _ in range(20):
            t1 = time.perf_counter()
            step1()
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - t1) * 1e3)
        extra["latency_b1_ms"] = float(np.median(lat))
        # the same one-frame step replayed from a captured hipGraph (fvp/graphs.py)
        from fvp.graphs import CapturedStep

        cap = CapturedStep(step1)
        cap.replay()
        torch.cuda.synchronize()
        lat = []
        for _ in range(20):
            t1 = time.perf_counter()
            cap.replay()
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - t1) * 1e3)
        extra["latency_b1_graph_ms"] = float(np.median(lat))
        # the same step at the C ABI (include/fvp.h) as a C / C++ host binds it:
        # fvp_voxelize (layout + gather) and fvp_nms_topk_columns on preallocated
        # buffers, then a stream sync -- no op wrappers, no allocation per call
        if isinstance(hm1, torch.Tensor) and hm1.dim() == 5 and not layer._project_on_the_fly(V):
            from fvp import _lib
            grids1, _ = layer._grids_for_batch(hm1, meta1, cams, rt)
            L = _lib.load()
            half = hm1.dtype == torch.float16
            nws = (L.fvp_voxelize_f16_workspace_bytes if half else L.fvp_voxelize_workspace_bytes)(1, V, J, Hd, Wd)
            ws1 = torch.empty((nws + 3) // 4, device=dev)
            cube1 = torch.empty((1, J, X, Y, Z), device=dev)
            xy1 = torch.empty((1, J, X, Y), device=dev)
            vals1 = torch.empty((1, K), device=dev)
            flat1 = torch.empty((1, K), dtype=torch.int64, device=dev)
            kxy1 = torch.empty((1, K, 2), dtype=torch.int64, device=dev)
            cols1 = torch.empty((1, K, J, Z), device=dev)
            st1 = torch.cuda.current_stream(dev)
            f_vox = L.fvp_voxelize_f16 if half else L.fvp_voxelize
            a_vox = (hm1.data_ptr(), 1, V, J, Hd, Wd, grids1.data_ptr(), None, X, Y, Z, cube1.data_ptr(),
                     xy1.data_ptr(), ws1.data_ptr(), nws, st1.cuda_stream)
            a_nms = (xy1.data_ptr() + root * X * Y * 4, 1, X, Y, J * X * Y, K, vals1.data_ptr(), flat1.data_ptr(),
                     kxy1.data_ptr(), cube1.data_ptr(), J, Z, cols1.data_ptr(), st1.cuda_stream)

            def step_abi():
                _lib.check(f_vox(*a_vox), "fvp_voxelize")
                _lib.check(L.fvp_nms_topk_columns(*a_nms), "fvp_nms_topk_columns")

            for _ in range(3):
                step_abi()
            torch.cuda.synchronize()
            if not torch.equal(cols1, step1()):
                raise SystemExit("bench: the C-ABI one-frame step differs from the op path")
            torch.cuda.synchronize()
            lat = []
            for _ in range(20):
                t1 = time.perf_counter()
                step_abi()
                st1.synchronize()
                lat.append((time.perf_counter() - t1) * 1e3)
            extra["latency_b1_abi_ms"] = float(np.median(lat))

    ceiling = None
    if rank == 0:
        ceiling = tap_floor_ceiling(Xs * Y * Z, V, J, Hd, Wd, hm_planar.element_size(),
                                    args.heatmap_layout == "planar", extra.get("copy_gbs"), per_frame)
        if world > 1:
            ceiling["copy_rate"] = "rank 0's"

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline == "on":
        note("cpu baseline")
        sg_cpu = layer.build_sample_grid(cams, seq, rt, dev).cpu().contiguous()
        cpu = cpu_baseline(w, sg_cpu, args.cpu_threads)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(fps, 1),
            "unit": "frames/s",
            "n_gpus": n_devices,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if (args.slabs or args.strong) else "weak",
            "vs_baseline": None,
            "dtype": "f32" if w.dtype == "float32" else "f16-in/f32",
            "data": "synthetic",
            "config": {
                "workload": f"{w.name}: {WORKLOAD_DESC.get(w.name, '')}, {V} cams, J={J}, "
                            f"{Hd}x{Wd} heatmaps -> {X}x{Y}x{Z} voxels, K={K} proposals",
                "frames_per_gpu_step": B,
                "global_batch": B if args.slabs else world * B,
                "parallelism": ((f"x-slab x{world}" + (f" + {collective} all_gather of xy slabs, all_reduce of columns"
                                                       if world > 1 else "") if args.slabs else
                                 f"frame-sharded x{world}" + (f" + {collective} all_gather of proposals" if grouped and world > 1
                                                              else " (one rank: no collective)"))
                                + (f" -- rehearsal (gloo, {world} ranks on {n_devices} shared device(s)), not a measurement"
                                   if rehearsal else "")),
            },
            "roofline": roofline_fields(
                ("fvp_voxelize op = layout pass (heatmaps_to_cl / pairs_vec8) + voxelize_kernel per "
                 "frame chunk" if args.heatmap_layout == "planar" else
                 "fvp_voxelize_cl op = voxelize_kernel on channels-last heatmaps (no layout pass)"),
                alg_bytes, [r[1] for r in per_rank], len(ev), traffic, extra.get("copy_gbs"), taps, tap_bytes,
                ceiling),
            "latency_b1_ms": round(extra["latency_b1_ms"], 3) if "latency_b1_ms" in extra else None,
            "latency_b1_graph_ms": round(extra["latency_b1_graph_ms"], 3) if "latency_b1_graph_ms" in extra else None,
            "latency_b1_abi_ms": round(extra["latency_b1_abi_ms"], 4) if "latency_b1_abi_ms" in extra else None,
            "cpu_baseline": cpu,
            "execution": "hipGraph replay of the GPU-local step" if args.graph == "on" else "eager",
            "cache_build": cache_ms,
        }
        if "channels_last" in extra:
            line["roofline"]["channels_last_input"] = extra["channels_last"]
        if args.heatmap_layout != "planar":
            line["config"]["heatmap_layout"] = "channels-last [B,V,H,W,16] (fvp backbone output)"
        if traffic_note:
            line["roofline"]["traffic_note"] = traffic_note
        elif traffic is None and world > 1:
            line["roofline"]["traffic_note"] = ("not collected under the launcher (rocprofv3 child runs at N = 1 "
                                                "only); per-rank work equals the N = 1 line's at the same --batch")
        sys.stdout.flush()
        print(json.dumps(line), file=json_out, flush=True)
    if grouped:
        note("final barrier")
        dist.barrier()  # rank 0's extra measurements done: every rank leaves together
        note("destroy process group")
        dist.destroy_process_group()
    note("done")


if __name__ == "__main__":
    main()
