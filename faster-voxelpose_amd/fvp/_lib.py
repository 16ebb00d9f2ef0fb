"""ctypes binding of libfvp.so (include/fvp.h).

The library is loaded AFTER ``import torch`` so that it binds to the HIP
runtime torch already loaded (one runtime per process; see csrc/Makefile).
There is no fallback: if the library is missing or fails to load, every fvp
op raises.  ``load()`` is cheap after the first call.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen below)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FVP_LIB", os.path.join(HERE, "libfvp.so"))

c_int, c_float, c_void_p, c_char_p = ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_char_p


class GridSpec(ctypes.Structure):
    _fields_ = [("start", c_float * 3), ("end", c_float * 3), ("center", c_float * 3), ("bins", ctypes.c_int32 * 3)]


class ImageSpec(ctypes.Structure):
    _fields_ = [("ori_max", c_float), ("img_w", c_float), ("img_h", c_float),
                ("hm_w", ctypes.c_int32), ("hm_h", ctypes.c_int32)]


class PersonSpec(ctypes.Structure):
    _fields_ = [("fine", ctypes.c_int32 * 3), ("scale", c_float * 3), ("bias", c_float * 3),
                ("whole_size", c_float * 3), ("ind_size", c_float * 3), ("bins", ctypes.c_int32 * 3)]


# name -> argtypes (restype is int status for all but the two info calls)
SIGNATURES = {
    "fvp_abi_version": [],
    "fvp_status_string": [c_int],
    "fvp_project_grid": [c_void_p, c_int, c_void_p, ctypes.POINTER(GridSpec), ctypes.POINTER(ImageSpec), c_void_p,
                         c_void_p],
    "fvp_pack_grid": [c_void_p, c_int, ctypes.c_longlong, c_void_p, c_void_p],
    "fvp_voxelize_workspace_bytes": [c_int, c_int, c_int, c_int, c_int],
    "fvp_voxelize_f16_workspace_bytes": [c_int, c_int, c_int, c_int, c_int],
    "fvp_voxelize": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                     c_void_p, c_void_p, ctypes.c_size_t, c_void_p],
    "fvp_voxelize_f16": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                         c_void_p, c_void_p, c_void_p, ctypes.c_size_t, c_void_p],
    "fvp_voxelize_cams": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                          ctypes.POINTER(GridSpec), ctypes.POINTER(ImageSpec), c_void_p, c_void_p, c_void_p,
                          ctypes.c_size_t, c_void_p],
    "fvp_voxelize_cams_slab": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                               ctypes.POINTER(GridSpec), ctypes.POINTER(ImageSpec), c_int, c_int, c_void_p, c_void_p,
                               c_void_p, ctypes.c_size_t, c_void_p],
    "fvp_voxelize_cl": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                        c_void_p, c_void_p, c_void_p],
    "fvp_voxelize_cl_cams": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                             ctypes.POINTER(GridSpec), ctypes.POINTER(ImageSpec), c_void_p, c_void_p, c_void_p],
    "fvp_voxelize_cl_cams_slab": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                  ctypes.POINTER(GridSpec), ctypes.POINTER(ImageSpec), c_int, c_int, c_void_p,
                                  c_void_p, c_void_p],
    "fvp_nms_topk": [c_void_p, c_int, c_int, c_int, ctypes.c_longlong, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "fvp_nms_topk_columns": [c_void_p, c_int, c_int, c_int, ctypes.c_longlong, c_int, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_int, c_int, c_void_p, c_void_p],
    "fvp_gather_columns": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p],
    "fvp_voxel_columns": [c_void_p, c_int, ctypes.c_longlong, ctypes.c_longlong, c_int, c_int, c_int, c_int, c_int,
                          c_int, c_void_p, c_void_p, c_void_p, ctypes.POINTER(GridSpec), ctypes.POINTER(ImageSpec),
                          c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p],
    "fvp_gather_bbox": [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p],
    "fvp_proposal_centers": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                             c_float, c_void_p, c_void_p],
    "fvp_person_workspace_bytes": [c_int, c_int, c_int, c_int, c_int],
    "fvp_conv2d_workspace_bytes": [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int],
    "fvp_person_planes": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, ctypes.POINTER(PersonSpec), c_void_p,
                          c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_size_t, c_void_p],
    "fvp_person_planes_cams": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                               ctypes.POINTER(GridSpec), ctypes.POINTER(ImageSpec), ctypes.POINTER(PersonSpec),
                               c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_size_t,
                               c_void_p],
    "fvp_person_planes_cl": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, ctypes.POINTER(PersonSpec),
                             c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "fvp_max_planes": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p],
    "fvp_soft_argmax": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p],
    "fvp_fuse_poses": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "fvp_conv2d_nhwc": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                        c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p],
    "fvp_conv2d_nhwc_ws": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                           c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, ctypes.c_size_t,
                           c_void_p],
    "fvp_conv2d_nhwc_bf16": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                             c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p],
    "fvp_conv2d_nhwc_ex": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                           c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                           c_void_p, c_void_p, ctypes.c_size_t, c_void_p],
    "fvp_conv2d_ex_workspace_bytes": [c_int] * 13,
    "fvp_conv2d_geom": [c_int] * 10 + [ctypes.POINTER(c_int)],
    "fvp_maxpool_pad_nhwc": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "fvp_conv1d_net_lds_bytes": [c_int, c_int, c_int, c_int],
    "fvp_conv1d_net": [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int,
                       c_int, c_int, c_void_p, c_void_p],
    "fvp_conv_front7_f32": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "fvp_conv_front7_bf16": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "fvp_conv_stem7_bf16": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "fvp_conv_stem7_f32": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "fvp_maxpool_pad_nhwc_bf16": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "fvp_maxpool2_nhwc": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "fvp_maxpool_nhwc": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "fvp_maxpool_nhwc_bf16": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "fvp_weight_net": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                       c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "fvp_copy_f4": [c_void_p, c_void_p, ctypes.c_size_t, c_void_p],
    "fvp_nchw_to_nhwc": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "fvp_conv3x3_wino_plan": [c_int, c_int, c_int, c_int, c_void_p],
    "fvp_deconv4s2_wino_nhwc": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_int, c_void_p, c_void_p],
    "fvp_conv3x3_wino_nhwc": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_int, c_void_p, c_void_p, c_void_p],
    "fvp_nhwc_to_nchw": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "fvp_conv1x1_nchw": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
                         c_int, c_void_p, c_void_p],
    "fvp_mask_nonzero": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "fvp_mask_select": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_longlong,
                        ctypes.c_longlong, c_int, c_void_p, c_void_p],
    "fvp_scatter_poses": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_void_p, ctypes.c_longlong, ctypes.c_longlong, c_int, c_void_p],
    "fvp_up2_head_nchw": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                          c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p],
}

ABI_VERSION = 22
_LIB = None


class FvpError(RuntimeError):
    pass


def load():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise FvpError(f"fvp: HIP library not built: {LIB_PATH} (run __graft_entry__.build() or make -C "
                       f"faster-voxelpose_amd/csrc)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = {"fvp_status_string": c_char_p, "fvp_voxelize_workspace_bytes": ctypes.c_size_t,
                      "fvp_voxelize_f16_workspace_bytes": ctypes.c_size_t,
                      "fvp_person_workspace_bytes": ctypes.c_size_t,
                      "fvp_conv2d_workspace_bytes": ctypes.c_size_t,
                      "fvp_conv2d_ex_workspace_bytes": ctypes.c_size_t,
                      "fvp_conv1d_net_lds_bytes": ctypes.c_size_t}.get(name, c_int)
    if lib.fvp_abi_version() != ABI_VERSION:
        raise FvpError(f"fvp: ABI version mismatch ({lib.fvp_abi_version()} != {ABI_VERSION})")
    _LIB = lib
    return lib


def check(status: int, what: str) -> None:
    if status != 0:
        msg = load().fvp_status_string(status).decode()
        raise FvpError(f"{what} failed: {msg} (status {status})")


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args), name)
