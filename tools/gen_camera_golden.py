#!/usr/bin/env python3
"""Golden vectors for fvp.cameras (the reference datasets' camera loaders).

Writes synthetic raw calibration files in the three dataset formats to
tests/golden/ (Panoptic-style ``{"cameras": [{panel, node, K, distCoef, R,
t}]}``, the custom dataset's ``{name: {k, d, p}}``; Shelf uses the committed
calibration_shelf.json), runs the reference's own ``_get_cam`` on them
(panoptic.py:171-205, custom.py:111-144, shelf.py:138-153) from /root/reference,
and stores the converted camera dicts in tests/golden/cams_ref.npz.  Skips
when /root/reference is absent.  Run with ``python3 -B`` (no __pycache__ in
the reference tree).
"""
import json
import os
import shutil
import sys
import tempfile
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
REF = "/root/reference/lib"


def rotation(rng):
    q, r = np.linalg.qr(rng.normal(size=(3, 3)))
    return q * np.sign(np.diag(r))


def synthetic(rng):
    pan = {"cameras": []}
    for panel, node in [(0, 0), (1, 3), (0, 2), (0, 5), (2, 1)]:
        K = [[rng.uniform(1300, 1500), 0.0, rng.uniform(900, 1000)],
             [0.0, rng.uniform(1300, 1500), rng.uniform(520, 560)], [0.0, 0.0, 1.0]]
        pan["cameras"].append({"name": f"{panel:02d}_{node:02d}", "panel": panel, "node": node, "K": K,
                               "distCoef": list(rng.uniform(-0.3, 0.3, 5)), "R": rotation(rng).tolist(),
                               "t": list(rng.uniform(-300, 300, 3))})
    cust = {}
    for name in ["cam_a", "cam_b", "cam_c"]:
        fx, fy, cx, cy = rng.uniform(900, 1100), rng.uniform(900, 1100), rng.uniform(600, 700), rng.uniform(330, 390)
        K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]])
        Rt = np.concatenate([rotation(rng), rng.uniform(-3000, 3000, (3, 1))], axis=1)
        cust[name] = {"k": [fx, fy, cx, cy], "d": list(rng.uniform(-0.2, 0.2, 5)), "p": (K @ Rt).reshape(-1).tolist()}
    return pan, cust


def main():
    if not os.path.isdir(REF):
        print("reference absent: skipped")
        return
    rng = np.random.default_rng(2024)
    pan, cust = synthetic(rng)
    with open(os.path.join(GOLDEN, "cams_raw_panoptic.json"), "w") as f:
        json.dump(pan, f)
    with open(os.path.join(GOLDEN, "cams_raw_custom.json"), "w") as f:
        json.dump(cust, f)

    sys.modules.setdefault("cv2", types.ModuleType("cv2"))  # only get_affine_transform uses it
    # json_tricks (absent here) reads plain JSON like the standard module
    jt = types.ModuleType("json_tricks")
    jt.load, jt.loads, jt.dump, jt.dumps = json.load, json.loads, json.dump, json.dumps
    sys.modules.setdefault("json_tricks", jt)
    sys.path.insert(0, REF)
    import dataset  # noqa: F401  (dataset/__init__.py imports the dataset modules)
    P, C, S = (sys.modules[f"dataset.{m}"] for m in ("panoptic", "custom", "shelf"))

    tmp = tempfile.mkdtemp(prefix="fvp_cams_")
    try:
        os.makedirs(os.path.join(tmp, "pan", "seqA"))
        shutil.copy(os.path.join(GOLDEN, "cams_raw_panoptic.json"), os.path.join(tmp, "pan", "seqA",
                                                                                  "calibration_seqA.json"))
        os.makedirs(os.path.join(tmp, "cust", "seqB"))
        shutil.copy(os.path.join(GOLDEN, "cams_raw_custom.json"), os.path.join(tmp, "cust", "seqB", "calibration.json"))
        os.makedirs(os.path.join(tmp, "shelf"))
        shutil.copy(os.path.join(GOLDEN, "calibration_shelf.json"), os.path.join(tmp, "shelf", "calibration_shelf.json"))
        cam_list = [(0, 0), (0, 2), (2, 1), (1, 3)]
        pan_ref = P.Panoptic._get_cam(types.SimpleNamespace(dataset_dir=os.path.join(tmp, "pan"),
                                                             sequence_list=["seqA"], cam_list=cam_list))
        cust_ref = C.Custom._get_cam(types.SimpleNamespace(dataset_dir=os.path.join(tmp, "cust"),
                                                            sequence_list=["seqB"]))
        shelf_ref = S.Shelf._get_cam(types.SimpleNamespace(dataset_dir=os.path.join(tmp, "shelf")))
    finally:
        shutil.rmtree(tmp)

    out = {"pan_cam_list": np.array(cam_list)}
    for tag, cams in (("pan", pan_ref["seqA"]), ("cust", cust_ref["seqB"])):
        out[f"{tag}_n"] = np.array(len(cams))
        for i, c in enumerate(cams):
            for k, v in c.items():
                out[f"{tag}_{i}_{k}"] = np.asarray(v, dtype=np.float64)
    out["shelf_ids"] = np.array(sorted(shelf_ref["shelf"].keys()))
    for i, c in shelf_ref["shelf"].items():
        for k, v in c.items():
            out[f"shelf_{i}_{k}"] = np.asarray(v, dtype=np.float64)
    np.savez(os.path.join(GOLDEN, "cams_ref.npz"), **out)
    print("wrote cams_ref.npz:", len(out), "arrays")


if __name__ == "__main__":
    main()
