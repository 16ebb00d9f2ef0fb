"""Minimal config object with the reference's key layout.

The reference keeps a module-global EasyDict merged from YAML
(lib/core/config.py:15-188).  After YAML loading every size key is a plain
Python list (config.py:167-169), which is the form the layers are written
against.  ``make_cfg`` builds the same structure for a :class:`Workload`, and
``load_yaml`` reads one of the reference's own YAML files (keys only; unknown
keys are kept, not rejected, since only the hot-path keys are read here).
"""
from __future__ import annotations


class AttrDict(dict):
    """dict with attribute access (the subset of EasyDict the layers use)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    @classmethod
    def wrap(cls, obj):
        if isinstance(obj, dict):
            return cls({k: cls.wrap(v) for k, v in obj.items()})
        return obj


def make_cfg(w, device: str = "cuda:0") -> AttrDict:
    cams, _ = w.cameras()
    n_views = len(next(iter(cams.values())))
    return AttrDict.wrap({
        "DEVICE": device,
        "DATASET": {
            "ORI_IMAGE_SIZE": list(w.ori_image_size),
            "IMAGE_SIZE": list(w.image_size),
            "HEATMAP_SIZE": list(w.heatmap_size),
            "CAMERA_NUM": n_views,
            "NUM_JOINTS": w.num_joints,
        },
        "CAPTURE_SPEC": {
            "SPACE_SIZE": list(map(float, w.space_size)),
            "SPACE_CENTER": list(map(float, w.space_center)),
            "VOXELS_PER_AXIS": list(map(int, w.voxels_per_axis)),
            "MAX_PEOPLE": w.max_people,
            "MIN_SCORE": w.min_score,
        },
        "INDIVIDUAL_SPEC": {
            "SPACE_SIZE": list(map(float, w.ind_space_size)),
            "VOXELS_PER_AXIS": list(map(int, w.ind_voxels_per_axis)),
        },
        "NETWORK": {"BETA": 100},  # configs/*/jln64.yaml NETWORK.BETA
    })


def resnet_cfg(num_layers: int = 50, num_joints: int = 15, deconv_filters=(256, 256, 256),
               deconv_kernels=(4, 4, 4), final_kernel: int = 1, deconv_with_bias: bool = False) -> AttrDict:
    """The RESNET / DATASET keys resnet.get(cfg) reads (lib/core/config.py:101-107
    defaults: ResNet-50, three 256-filter kernel-4 deconvolutions, a 1x1 final conv)."""
    return AttrDict.wrap({
        "RESNET": {"NUM_LAYERS": num_layers, "DECONV_WITH_BIAS": deconv_with_bias,
                   "NUM_DECONV_LAYERS": len(deconv_filters), "NUM_DECONV_FILTERS": list(deconv_filters),
                   "NUM_DECONV_KERNELS": list(deconv_kernels), "FINAL_CONV_KERNEL": final_kernel},
        "DATASET": {"NUM_JOINTS": num_joints},
    })


def load_yaml(path: str, device: str | None = None) -> AttrDict:
    import yaml

    with open(path) as f:
        raw = yaml.load(f, Loader=yaml.SafeLoader)
    cfg = AttrDict.wrap(raw)
    if device is not None:
        cfg["DEVICE"] = device
    return cfg
