import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "faster-voxelpose_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def golden(name):
    import numpy as np

    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="session")
def gpu_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.fixture(params=["halo", "pertap", "pertap-nosplit", "dma", "wino"])
def conv_kernel(request):
    """The fp32 kernel choice a test builds its layers with (``algo`` of
    fvp.cnn.ConvLayer / FvpCNN): the halo-tiled KxK kernel on every eligible
    layer (so small test shapes take it too), the per-tap kernel only (split-K
    where a launch is under-filled), neither halo nor split-K
    (FVP_CONV_HALO / _PER_TAP / _PER_TAP_NOSPLIT of fvp_conv2d_nhwc_ws), and the
    LDS-DMA kernel on every layer it takes (FVP_CONV_F32_KC), and Winograd
    F(2x2, 3x3) on every 3x3 stride-1 "same" layer (fvp_conv3x3_wino_nhwc; the
    other layers as AUTO)."""
    from fvp import cnn

    return {"halo": cnn.CONV_HALO, "pertap": cnn.CONV_PER_TAP, "pertap-nosplit": cnn.CONV_PER_TAP_NOSPLIT,
            "dma": cnn.CONV_DMA, "wino": cnn.CONV_WINO}[request.param]
