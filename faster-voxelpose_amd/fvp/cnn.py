"""The HDN / JLN 2-D CNNs on the fp32 matrix cores.

:class:`FvpCNN` compiles an eval-mode reference module -- ``P2PNet``
(cnns_2d.py:185-232), ``CenterNet`` (:235-295) or any ``nn.Sequential`` /
``Basic2DBlock`` / ``Res2DBlock`` / ``Pool2DBlock`` / ``Upsample2DBlock`` /
``EncoderDecorder`` (:12-183) built from them -- into a sequence of
``fvp_conv2d_nhwc`` launches: NHWC fp32 activations (channels padded to 16),
BatchNorm folded with the conv bias into a per-channel scale/shift, the
Res2DBlock residual add and the ReLU fused into the conv epilogue, the
decoder's skip adds fused after the ReLU, ConvTranspose2d(2, 2) as a 1x1 conv
with a 2x scatter epilogue.  Modules are recognised by the reference's
attribute names, so the reference's own instances (and their state_dicts) are
used directly.  Eval mode only (BatchNorm with running statistics).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from .ops import _ptr, _stream


def _rup(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class Act:
    """NHWC activation [N,H,W,Cp] with C logical channels (padding channels are zero)."""

    def __init__(self, t: torch.Tensor, C: int):
        self.t, self.C = t, C

    @property
    def N(self):
        return self.t.shape[0]

    @property
    def H(self):
        return self.t.shape[1]

    @property
    def W(self):
        return self.t.shape[2]

    @property
    def Cp(self):
        return self.t.shape[3]


class ConvLayer:
    """A Conv2d / ConvTranspose2d(k=2,s=2) with its following BatchNorm folded.
    dtype torch.bfloat16: bf16 operands, fp32 accumulation (opt-in precision)."""

    def __init__(self, conv, bn=None, dtype=torch.float32):
        dev = conv.weight.device
        w = conv.weight.detach().float()
        self.up2 = isinstance(conv, nn.ConvTranspose2d)
        if self.up2:
            assert tuple(conv.kernel_size) == (2, 2) and tuple(conv.stride) == (2, 2) and tuple(conv.padding) == (0, 0)
            cin, cout = w.shape[0], w.shape[1]
            self.KH = self.KW = 1
        else:
            assert tuple(conv.stride) == (1, 1) and conv.groups == 1 and tuple(conv.dilation) == (1, 1)
            cout, cin, kh, kw = w.shape
            assert tuple(conv.padding) == ((kh - 1) // 2, (kw - 1) // 2) and kh % 2 == 1 and kw % 2 == 1
            self.KH, self.KW = kh, kw
        self.Cin, self.Cout = cin, cout
        self.Cpi, self.Cpo = _rup(cin, 16), _rup(cout, 16)
        ntot = 4 * self.Cpo if self.up2 else self.Cpo
        self.Cpo_w = _rup(ntot, 128)
        taps = self.KH * self.KW
        pack = torch.zeros((taps, self.Cpi, self.Cpo_w), dtype=torch.float32, device=dev)
        if self.up2:  # n = (dy*2+dx)*Cpo + co  <-  W[ci][co][dy][dx]
            for q in range(4):
                pack[0, :cin, q * self.Cpo:q * self.Cpo + cout] = w[:, :, q >> 1, q & 1]
        else:  # row (ky*KW+kx)*Cpi + ci  <-  W[co][ci][ky][kx]
            pack[:, :cin, :cout] = w.permute(2, 3, 1, 0).reshape(taps, cin, cout)
        self.wpack = pack.reshape(taps * self.Cpi, self.Cpo_w).contiguous()
        self.bf16 = dtype == torch.bfloat16
        if self.bf16:  # [Cpo_w][K], k contiguous
            self.wpack_bf16 = self.wpack.t().contiguous().to(torch.bfloat16)
        bias = conv.bias.detach().float() if conv.bias is not None else torch.zeros(cout, device=dev)
        if bn is not None:  # eval BatchNorm: (x - mean) / sqrt(var + eps) * gamma + beta
            s = bn.weight.detach().float() / torch.sqrt(bn.running_var.detach().float() + bn.eps)
            scale, shift = s, (bias - bn.running_mean.detach().float()) * s + bn.bias.detach().float()
        else:
            scale, shift = torch.ones(cout, device=dev), bias
        self.scale = torch.zeros(self.Cpo, device=dev)
        self.shift = torch.zeros(self.Cpo, device=dev)
        self.scale[:cout] = scale
        self.shift[:cout] = shift

    def __call__(self, x: Act, relu: bool, res_pre: Act | None = None, res_post: Act | None = None) -> Act:
        assert x.Cp == self.Cpi, (x.Cp, self.Cpi)
        Ho, Wo = (2 * x.H, 2 * x.W) if self.up2 else (x.H, x.W)
        out = torch.empty((x.N, Ho, Wo, self.Cpo), dtype=torch.float32, device=x.t.device)
        for r in (res_pre, res_post):
            assert r is None or tuple(r.t.shape) == tuple(out.shape), (None if r is None else r.t.shape, out.shape)
        fn, w = ("fvp_conv2d_nhwc_bf16", self.wpack_bf16) if self.bf16 else ("fvp_conv2d_nhwc", self.wpack)
        _lib.call(fn, _ptr(x.t), x.N, x.H, x.W, x.Cp, _ptr(w), self.KH, self.KW, self.Cpo,
                  self.Cpo_w, _ptr(self.scale), _ptr(self.shift), _ptr(res_pre.t) if res_pre else None,
                  _ptr(res_post.t) if res_post else None, int(relu), int(self.up2), _ptr(out), _stream(out))
        return Act(out, self.Cout)

    def flops(self, x: Act) -> int:
        n = 4 * self.Cout if self.up2 else self.Cout
        return 2 * x.N * x.H * x.W * n * self.Cin * self.KH * self.KW


def maxpool2(x: Act) -> Act:
    out = torch.empty((x.N, x.H // 2, x.W // 2, x.Cp), dtype=torch.float32, device=x.t.device)
    _lib.call("fvp_maxpool2_nhwc", _ptr(x.t), x.N, x.H, x.W, x.Cp, _ptr(out), _stream(out))
    return Act(out, x.C)


def to_nhwc(x: torch.Tensor) -> Act:
    x = x.float().contiguous()
    N, C, H, W = x.shape
    out = torch.empty((N, H, W, _rup(C, 16)), dtype=torch.float32, device=x.device)
    _lib.call("fvp_nchw_to_nhwc", _ptr(x), N, C, H, W, out.shape[3], _ptr(out), _stream(out))
    return Act(out, C)


def to_nchw(x: Act) -> torch.Tensor:
    out = torch.empty((x.N, x.C, x.H, x.W), dtype=torch.float32, device=x.t.device)
    _lib.call("fvp_nhwc_to_nchw", _ptr(x.t), x.N, x.C, x.H, x.W, x.Cp, _ptr(out), _stream(out))
    return out


# ---------------------------------------------------------------------------
def _seq_convs(seq: nn.Sequential, dtype=torch.float32):
    """[Conv(, BN)(, ReLU)]* of an nn.Sequential -> [(ConvLayer, relu)]."""
    mods = list(seq.children())
    out, i = [], 0
    while i < len(mods):
        m = mods[i]
        if not isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
            raise TypeError(f"FvpCNN: unsupported layer {type(m).__name__} in a Sequential")
        bn = mods[i + 1] if i + 1 < len(mods) and isinstance(mods[i + 1], nn.BatchNorm2d) else None
        j = i + 1 + (bn is not None)
        relu = j < len(mods) and isinstance(mods[j], nn.ReLU)
        out.append((ConvLayer(m, bn, dtype), relu))
        i = j + relu
    return out


class _Plan:
    """A compiled module: call(x: Act) -> Act."""

    def __init__(self, m: nn.Module, dtype=torch.float32):
        self.dtype = dtype
        self.kind, self.parts = self._compile(m)

    def _compile(self, m):
        if hasattr(m, "res_branch"):  # Res2DBlock (cnns_2d.py:32-64)
            (c1, r1), (c2, _) = _seq_convs(m.res_branch, self.dtype)
            skip = _seq_convs(m.skip_con, self.dtype) if len(list(m.skip_con.children())) else []
            return "res", (c1, c2, skip[0][0] if skip else None)
        if hasattr(m, "pool_size"):  # Pool2DBlock
            assert m.pool_size == 2
            return "pool", None
        if hasattr(m, "block"):  # Basic2DBlock / Upsample2DBlock: Sequential(conv, BN, ReLU)
            return "seq", _seq_convs(m.block, self.dtype)
        if hasattr(m, "encoder_pool1") and hasattr(m, "skip_res1"):  # EncoderDecorder (:123-183)
            names = ["skip_res1", "encoder_pool1", "encoder_res1", "skip_res2", "encoder_pool2", "encoder_res2",
                     "mid_res", "decoder_res2", "decoder_upsample2", "decoder_res1", "decoder_upsample1"]
            return "encdec", {n: _Plan(getattr(m, n), self.dtype) for n in names}
        if isinstance(m, nn.Sequential):
            kids = list(m.children())
            if kids and all(isinstance(k, (nn.Conv2d, nn.ConvTranspose2d, nn.BatchNorm2d, nn.ReLU)) for k in kids):
                return "seq", _seq_convs(m, self.dtype)
            return "chain", [_Plan(k, self.dtype) for k in kids]
        raise TypeError(f"FvpCNN: unsupported module {type(m).__name__}")

    def __call__(self, x: Act, res_post: Act | None = None) -> Act:
        k, p = self.kind, self.parts
        if k == "res":
            c1, c2, skip = p
            skip_x = x if skip is None else skip(x, relu=False)
            return c2(c1(x, relu=True), relu=True, res_pre=skip_x, res_post=res_post)
        if k == "pool":
            assert res_post is None
            return maxpool2(x)
        if k == "seq":
            for i, (c, relu) in enumerate(p):
                x = c(x, relu, res_post=res_post if i == len(p) - 1 else None)
            return x
        if k == "chain":
            for i, sub in enumerate(p):
                x = sub(x, res_post if i == len(p) - 1 else None)
            return x
        if k == "encdec":  # EncoderDecorder.forward (cnns_2d.py:156-180)
            skip_x1 = p["skip_res1"](x)
            x = p["encoder_pool1"](x)
            x = p["encoder_res1"](x)
            skip_x2 = p["skip_res2"](x)
            x = p["encoder_pool2"](x)
            x = p["encoder_res2"](x)
            x = p["mid_res"](x)
            x = p["decoder_res2"](x)
            x = p["decoder_upsample2"](x, res_post=skip_x2)  # x = upsample(x) + skip_x2
            x = p["decoder_res1"](x)
            x = p["decoder_upsample1"](x, res_post=skip_x1)  # x = upsample(x) + skip_x1
            assert res_post is None
            return x
        raise AssertionError(k)


class FvpCNN:
    """Eval-mode P2PNet / CenterNet (or a block of them) on fvp conv kernels.

    ``FvpCNN(p2pnet)(x[N,J,H,W]) -> [N,out,H,W]``;
    ``FvpCNN(center_net).from_xy(xy[B,J,X,Y]) -> (hm, size)`` (CenterNet.forward
    after its ``torch.max(x, dim=4)``, cnns_2d.py:291-295).  Weights are read
    once at construction; rebuild after loading a new state_dict."""

    def __init__(self, module: nn.Module, dtype=torch.float32):
        """dtype torch.bfloat16: bf16 operands with fp32 accumulation (opt-in; ~1e-2 relative)."""
        if dtype not in (torch.float32, torch.bfloat16):
            raise _lib.FvpError(f"FvpCNN: dtype {dtype} (float32 or bfloat16)")
        if module.training:
            raise _lib.FvpError("FvpCNN: eval mode only (BatchNorm folded with running statistics)")
        self.module = module
        if hasattr(module, "output_hm") and hasattr(module, "output_size"):  # CenterNet
            self.kind = "centernet"
            self.front = _Plan(module.front_layers, dtype)
            self.encdec = _Plan(module.encoder_decoder, dtype)
            self.hm = _seq_convs(module.output_hm, dtype)
            self.size = _seq_convs(module.output_size, dtype)
        elif hasattr(module, "output_layer"):  # P2PNet
            self.kind = "p2p"
            self.front = _Plan(module.front_layers, dtype)
            self.encdec = _Plan(module.encoder_decoder, dtype)
            self.out = ConvLayer(module.output_layer, None, dtype)
        else:
            self.kind = "plain"
            self.plan = _Plan(module, dtype)

    @staticmethod
    def _run_seq(seq, x):
        for c, relu in seq:
            x = c(x, relu)
        return x

    @torch.no_grad()
    def __call__(self, x: torch.Tensor):
        a = to_nhwc(x)
        if self.kind == "p2p":
            return to_nchw(self.out(self.encdec(self.front(a)), relu=False))
        if self.kind == "centernet":
            return self.from_xy(x)
        return to_nchw(self.plan(a))

    @torch.no_grad()
    def from_xy(self, xy: torch.Tensor):
        assert self.kind == "centernet"
        f = self.encdec(self.front(to_nhwc(xy)))
        return to_nchw(self._run_seq(self.hm, f)), to_nchw(self._run_seq(self.size, f))


def cached(module: nn.Module, dtype=torch.float32) -> FvpCNN:
    """FvpCNN for ``module``, rebuilt whenever its parameters or buffers change
    (storage or in-place version), e.g. after load_state_dict."""
    sig = (dtype,) + tuple((t.data_ptr(), t._version) for t in list(module.parameters()) + list(module.buffers()))
    hit = getattr(module, "_fvp_cnn", None)
    if hit is None or hit[0] != sig:
        hit = (sig, FvpCNN(module, dtype))
        object.__setattr__(module, "_fvp_cnn", hit)
    return hit[1]
