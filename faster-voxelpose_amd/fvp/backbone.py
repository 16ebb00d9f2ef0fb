"""The PoseResNet heatmap backbone on the fvp MFMA convolutions (SURVEY.md
§8(f) rank 4: lib/models/resnet.py:98-201, called per view at
faster_voxelpose.py:73-75).

:class:`FvpPoseResNet` compiles an eval-mode reference ``ResNet`` (Bottleneck or
BasicBlock stages, the deconvolution head, the final conv) into
``fvp_conv2d_nhwc_ex`` launches:

* conv1 7x7/s2/p3 + BN + ReLU on the RGB input padded to 4 channels (a K chunk
  of the implicit GEMM spans 4 taps, so no MFMA work goes to padding channels);
  with bf16 operands a dedicated kernel reads the NCHW images directly
  (``fvp_conv_stem7_bf16``: halo tile in LDS, no NHWC conversion pass);
* MaxPool2d(3, 2, 1) (``fvp_maxpool_pad_nhwc``);
* each Bottleneck (resnet.py:57-95) as three launches -- 1x1 + BN + ReLU, 3x3
  (stride) + BN + ReLU, 1x1 + BN with the residual add and the ReLU fused into
  the epilogue -- plus the downsample 1x1/stride + BN (:132-137) when present;
  BasicBlock (:25-54) as two;
* each ConvTranspose2d(4, 2, 1) + BN + ReLU of the head (:160-185) as four
  parity GEMMs in one launch, the final 1x1 conv (:122-128) with its bias.

The output stays NHWC: ``[N, h, w, Cp]`` with the J joints in channels 0..J-1
and zeros after them, i.e. exactly the channels-last heatmap layout the
voxelize gather reads (``fvp_voxelize_cl``), so the views path needs no
transpose pass (:meth:`FvpPoseResNet.heatmaps_cl`).  ``__call__`` returns the
reference's NCHW heatmaps.  Eval mode only (BatchNorm with running statistics).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from .cnn import CONV_AUTO, Act, ConvLayer, maxpool_pad, to_nchw, to_nhwc
from .ops import _ptr, _stream
from .heatmaps import ChannelsLastHeatmaps

RGB_PITCH = 4  # input channel pitch of conv1 (3 colour channels + one zero)


class _Block:
    """Bottleneck (3 convs) or BasicBlock (2 convs) with an optional downsample."""

    def __init__(self, blk: nn.Module, dtype, algo=None):
        if hasattr(blk, "conv3"):
            self.convs = [ConvLayer(blk.conv1, blk.bn1, dtype, algo=algo), ConvLayer(blk.conv2, blk.bn2, dtype, algo=algo),
                          ConvLayer(blk.conv3, blk.bn3, dtype, algo=algo)]
        elif hasattr(blk, "conv2"):
            self.convs = [ConvLayer(blk.conv1, blk.bn1, dtype, algo=algo), ConvLayer(blk.conv2, blk.bn2, dtype, algo=algo)]
        else:
            raise _lib.FvpError(f"FvpPoseResNet: unsupported block {type(blk).__name__}")
        self.down = None
        if blk.downsample is not None:
            ds = list(blk.downsample.children())
            if not (len(ds) == 2 and isinstance(ds[0], nn.Conv2d) and isinstance(ds[1], nn.BatchNorm2d)):
                raise _lib.FvpError("FvpPoseResNet: downsample must be Sequential(Conv2d, BatchNorm2d)")
            self.down = ConvLayer(ds[0], ds[1], dtype, algo=algo)

    def __call__(self, x: Act) -> Act:
        residual = x if self.down is None else self.down(x, relu=False)
        last = self.convs[-1]
        want = torch.bfloat16 if (last.bf16 and last.act_bf16) else torch.float32
        if residual.t.dtype != want:  # an identity residual whose dtype differs from the block's output
            residual = Act(residual.t.to(want), residual.C)
        y = x
        for c in self.convs[:-1]:
            y = c(y, relu=True)
        return self.convs[-1](y, relu=True, res_pre=residual)  # out += residual; relu (resnet.py:89-93)

    def layers(self):
        return self.convs + ([self.down] if self.down is not None else [])


class FvpPoseResNet:
    """Eval-mode PoseResNet: ``FvpPoseResNet(resnet)(images[N,3,H,W]) -> heatmaps[N,J,H/4,W/4]``.

    dtype torch.bfloat16: bf16 operands with fp32 accumulation on every layer,
    bf16 activations between the layers (opt-in precision).  Weights are read once at construction;
    rebuild after loading a new state_dict."""

    def __init__(self, module: nn.Module, dtype=torch.float32, algo: int | None = None):
        if dtype not in (torch.float32, torch.bfloat16):
            raise _lib.FvpError(f"FvpPoseResNet: dtype {dtype} (float32 or bfloat16)")
        if module.training:
            raise _lib.FvpError("FvpPoseResNet: eval mode only (BatchNorm folded with running statistics)")
        self.module, self.dtype = module, dtype
        if module.conv1.in_channels > RGB_PITCH:
            raise _lib.FvpError(f"FvpPoseResNet: {module.conv1.in_channels} input channels (RGB expected)")
        self.stem = ConvLayer(module.conv1, module.bn1, dtype, cpi=RGB_PITCH, algo=algo)
        # bf16: the 7x7/s2/p3 -> 64 stem runs its own kernel straight from the
        # NCHW images (fvp_conv_stem7_bf16), weights packed [64][7][8][4]
        c1 = module.conv1
        self.stem7 = self.stem7_f32 = None
        stem7 = (tuple(c1.kernel_size) == (7, 7) and tuple(c1.stride) == (2, 2) and tuple(c1.padding) == (3, 3)
                 and c1.out_channels == 64 and c1.groups == 1 and tuple(c1.dilation) == (1, 1))
        if stem7 and dtype == torch.bfloat16:
            w = torch.zeros((64, 7, 8, 4), dtype=torch.float32, device=c1.weight.device)
            w[:, :, :7, :c1.in_channels] = c1.weight.detach().float().permute(0, 2, 3, 1)
            self.stem7 = w.reshape(64, 224).to(torch.bfloat16).contiguous()
        elif stem7 and c1.in_channels <= 3 and (algo is None or algo == CONV_AUTO):
            # fp32 (fvp_conv_stem7_f32): row kk = 21 ky + 3 kx + c of [148][80], column co
            w = torch.zeros((7, 7, 3, 80), dtype=torch.float32, device=c1.weight.device)
            w[:, :, :c1.in_channels, :64] = c1.weight.detach().float().permute(2, 3, 1, 0)
            self.stem7_f32 = torch.cat([w.reshape(147, 80), w.new_zeros((1, 80))]).contiguous()
        mp = module.maxpool
        k, s, p = (mp.kernel_size, mp.stride, mp.padding)
        k, s, p = (v if isinstance(v, int) else v[0] for v in (k, s, p))
        if mp.ceil_mode or (mp.dilation not in (1, (1, 1))):
            raise _lib.FvpError("FvpPoseResNet: max pool must be floor mode without dilation")
        self.pool = (k, s, p)
        self.blocks = [_Block(b, dtype, algo) for name in ("layer1", "layer2", "layer3", "layer4")
                       for b in getattr(module, name).children()]
        mods = list(module.deconv_layers.children())
        self.deconvs = []
        i = 0
        while i < len(mods):  # (ConvTranspose2d, BatchNorm2d, ReLU) * NUM_DECONV_LAYERS (resnet.py:171-183)
            conv, bn, act = mods[i], mods[i + 1], mods[i + 2]
            if not (isinstance(conv, nn.ConvTranspose2d) and isinstance(bn, nn.BatchNorm2d)
                    and isinstance(act, nn.ReLU)):
                raise _lib.FvpError("FvpPoseResNet: deconv head must be (ConvTranspose2d, BatchNorm2d, ReLU)*")
            self.deconvs.append(ConvLayer(conv, bn, dtype, algo=algo))
            i += 3
        self.final = ConvLayer(module.final_layer, None, dtype, algo=algo)
        self.num_joints = module.final_layer.out_channels
        # bf16: activations between the layers stay bf16 in HBM (half the bytes,
        # no per-chunk conversion), the stem's output and its max pool included;
        # the RGB input and the heatmaps are fp32
        for c in self.layers()[:-1]:
            c.act_bf16 = c.bf16

    def layers(self):
        out = [self.stem]
        for b in self.blocks:
            out += b.layers()
        return out + self.deconvs + [self.final]

    @torch.no_grad()
    def forward_nhwc(self, images: torch.Tensor, out: torch.Tensor | None = None) -> Act:
        """images [N,3,H,W] -> NHWC heatmaps Act [N,h,w,Cp] (J channels, zeros after).
        out: optional [N,h,w,Cp] destination of the final layer."""
        if images.device.type != "cuda":
            raise _lib.FvpError(f"fvp: images must be on a HIP device, got {images.device}")
        if self.stem7 is not None:
            x = self._stem7(images)
        elif self.stem7_f32 is not None:
            x = self._stem7_f32(images)
        else:
            x = self.stem(to_nhwc(images, RGB_PITCH), relu=True)
        x = maxpool_pad(x, *self.pool)
        for b in self.blocks:
            x = b(x)
        for d in self.deconvs:
            x = d(x, relu=True)
        return self.final(x, relu=False, out=out)

    def _stem7(self, images: torch.Tensor) -> Act:
        x = images.float().contiguous()
        N, C, H, W = x.shape
        out = torch.empty((N, (H - 1) // 2 + 1, (W - 1) // 2 + 1, 64), dtype=torch.bfloat16, device=x.device)
        _lib.call("fvp_conv_stem7_bf16", _ptr(x), N, C, H, W, _ptr(self.stem7), _ptr(self.stem.scale),
                  _ptr(self.stem.shift), _ptr(out), _stream(out))
        return Act(out, 64)

    def _stem7_f32(self, images: torch.Tensor) -> Act:
        x = images.float().contiguous()
        N, C, H, W = x.shape
        out = torch.empty((N, (H - 1) // 2 + 1, (W - 1) // 2 + 1, 64), device=x.device)
        _lib.call("fvp_conv_stem7_f32", _ptr(x), N, C, H, W, _ptr(self.stem7_f32), _ptr(self.stem.scale),
                  _ptr(self.stem.shift), _ptr(out), _stream(out))
        return Act(out, 64)

    def __call__(self, images: torch.Tensor) -> torch.Tensor:
        """ResNet.forward (resnet.py:187-201): [N,3,H,W] -> [N,J,h,w] fp32."""
        return to_nchw(self.forward_nhwc(images))

    @torch.no_grad()
    def heatmaps_cl(self, views: torch.Tensor) -> ChannelsLastHeatmaps:
        """All views of a batch in one pass: views [B,V,3,H,W] -> channels-last
        heatmaps [B,V,h,w,Cp] (the stack of faster_voxelpose.py:75 without the
        per-view loop, the stack copy, or a transpose before the voxelize)."""
        B, V = views.shape[:2]
        act = self.forward_nhwc(views.reshape((B * V,) + tuple(views.shape[2:])))
        return ChannelsLastHeatmaps(act.t.view(B, V, act.H, act.W, act.Cp), self.num_joints)

    def flops(self, N: int, H: int, W: int) -> int:
        """Multiply-add FLOPs of one forward on N images of H x W (MFMA work, padding excluded)."""
        total, h, w = 0, H, W
        dummy = lambda C, h, w: Act(torch.empty((N, h, w, C), device="meta"), C)  # noqa: E731
        x = dummy(self.stem.Cpi, h, w)
        total += self.stem.flops(x)
        h, w = self.stem.out_hw(h, w)
        k, s, p = self.pool
        h, w = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        for b in self.blocks:
            hi, wi = h, w
            for c in b.convs:
                total += c.flops(dummy(c.Cpi, h, w))
                h, w = c.out_hw(h, w)
            if b.down is not None:
                total += b.down.flops(dummy(b.down.Cpi, hi, wi))
        for d in self.deconvs + [self.final]:
            total += d.flops(dummy(d.Cpi, h, w))
            h, w = d.out_hw(h, w)
        return total


def cached(module: nn.Module, dtype=torch.float32, algo: int | None = None) -> FvpPoseResNet:
    """FvpPoseResNet for ``module``, rebuilt whenever its parameters or buffers change."""
    sig = (dtype, algo) + tuple((t.data_ptr(), t._version) for t in list(module.parameters()) + list(module.buffers()))
    hit = getattr(module, "_fvp_backbone", None)
    if hit is None or hit[0] != sig:
        hit = (sig, FvpPoseResNet(module, dtype, algo))
        object.__setattr__(module, "_fvp_backbone", hit)
    return hit[1]
