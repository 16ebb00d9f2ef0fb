"""Test-side restatement of the reference's 2-D CNN architectures
(lib/models/cnns_2d.py: Basic2DBlock :12-29, Res2DBlock :32-64, Pool2DBlock
:67-79, Upsample2DBlock :82-104, EncoderDecorder :123-183, P2PNet :185-232,
CenterNet :235-295), their 1-D twins (lib/models/cnns_1d.py: Basic1DBlock
:10-34, Res1DBlock :37-74, Pool1DBlock :77-93, Upsample1DBlock :96-123,
EncoderDecorder :125-179, C2CNet :182-241) and WeightNet (weight_net.py:48-80)
with the same module attribute names, so state_dicts are interchangeable with
the reference's.  Pinned to the reference by
tests/golden/cnn.npz (tools/gen_golden.py runs the reference's own classes on
the same seeded weights and inputs).  Used where the reference is absent (the
GPU box)."""
import torch
import torch.nn as nn
import torch.nn.functional as F


def _cbr(cin, cout, k, relu=True):
    layers = [nn.Conv2d(cin, cout, k, stride=1, padding=(k - 1) // 2), nn.BatchNorm2d(cout)]
    return layers + [nn.ReLU(True)] if relu else layers


class Basic2DBlock(nn.Module):
    def __init__(self, cin, cout, k):
        super().__init__()
        self.block = nn.Sequential(*_cbr(cin, cout, k))

    def forward(self, x):
        return self.block(x)


class Res2DBlock(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.res_branch = nn.Sequential(*_cbr(cin, cout, 3), *_cbr(cout, cout, 3, relu=False))
        self.skip_con = nn.Sequential() if cin == cout else nn.Sequential(*_cbr(cin, cout, 1, relu=False))

    def forward(self, x):
        return F.relu(self.res_branch(x) + self.skip_con(x), True)


class Pool2DBlock(nn.Module):
    def __init__(self, pool_size):
        super().__init__()
        self.pool_size = pool_size

    def forward(self, x):
        return F.max_pool2d(x, kernel_size=self.pool_size, stride=self.pool_size)


class Upsample2DBlock(nn.Module):
    def __init__(self, cin, cout, k, s):
        super().__init__()
        self.block = nn.Sequential(nn.ConvTranspose2d(cin, cout, k, stride=s), nn.BatchNorm2d(cout), nn.ReLU(True))

    def forward(self, x):
        return self.block(x)


class EncoderDecorder(nn.Module):
    def __init__(self):
        super().__init__()
        self.encoder_pool1 = Pool2DBlock(2)
        self.encoder_res1 = Res2DBlock(32, 64)
        self.encoder_pool2 = Pool2DBlock(2)
        self.encoder_res2 = Res2DBlock(64, 128)
        self.mid_res = Res2DBlock(128, 128)
        self.decoder_res2 = Res2DBlock(128, 128)
        self.decoder_upsample2 = Upsample2DBlock(128, 64, 2, 2)
        self.decoder_res1 = Res2DBlock(64, 64)
        self.decoder_upsample1 = Upsample2DBlock(64, 32, 2, 2)
        self.skip_res1 = Res2DBlock(32, 32)
        self.skip_res2 = Res2DBlock(64, 64)

    def forward(self, x):
        s1 = self.skip_res1(x)
        x = self.encoder_res1(self.encoder_pool1(x))
        s2 = self.skip_res2(x)
        x = self.decoder_res2(self.mid_res(self.encoder_res2(self.encoder_pool2(x))))
        x = self.decoder_res1(self.decoder_upsample2(x) + s2)
        return self.decoder_upsample1(x) + s1


class P2PNet(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.output_channels = cout
        self.front_layers = nn.Sequential(Basic2DBlock(cin, 16, 7), Res2DBlock(16, 32))
        self.encoder_decoder = EncoderDecorder()
        self.output_layer = nn.Conv2d(32, cout, kernel_size=1)

    def forward(self, x):
        return self.output_layer(self.encoder_decoder(self.front_layers(x)))


class CenterNet(nn.Module):
    def __init__(self, cin, cout, head_conv=32):
        super().__init__()
        self.output_channels = cout
        self.front_layers = nn.Sequential(Basic2DBlock(cin, 16, 7), Res2DBlock(16, 32))
        self.encoder_decoder = EncoderDecorder()
        self.output_hm = nn.Sequential(nn.Conv2d(32, head_conv, 3, padding=1), nn.ReLU(True),
                                       nn.Conv2d(head_conv, cout, 1))
        self.output_size = nn.Sequential(nn.Conv2d(32, head_conv, 3, padding=1), nn.ReLU(True),
                                         nn.Conv2d(head_conv, 2, 1))

    def forward(self, x):
        x, _ = torch.max(x, dim=4)
        x = self.encoder_decoder(self.front_layers(x))
        return self.output_hm(x), self.output_size(x)


# ---- 1-D (cnns_1d.py) ---------------------------------------------------------
def _cbr1(cin, cout, k, relu=True):
    layers = [nn.Conv1d(cin, cout, k, stride=1, padding=(k - 1) // 2), nn.BatchNorm1d(cout)]
    return layers + [nn.ReLU(True)] if relu else layers


class Basic1DBlock(nn.Module):
    def __init__(self, cin, cout, k):
        super().__init__()
        self.block = nn.Sequential(*_cbr1(cin, cout, k))

    def forward(self, x):
        return self.block(x)


class Res1DBlock(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.res_branch = nn.Sequential(*_cbr1(cin, cout, 3), *_cbr1(cout, cout, 3, relu=False))
        self.skip_con = nn.Sequential() if cin == cout else nn.Sequential(*_cbr1(cin, cout, 1, relu=False))

    def forward(self, x):
        return F.relu(self.res_branch(x) + self.skip_con(x), True)


class Pool1DBlock(nn.Module):
    def __init__(self, pool_size):
        super().__init__()
        self.pool_size = pool_size

    def forward(self, x):
        return F.max_pool1d(x, kernel_size=self.pool_size, stride=self.pool_size)


class Upsample1DBlock(nn.Module):
    def __init__(self, cin, cout, k, s):
        super().__init__()
        self.block = nn.Sequential(nn.ConvTranspose1d(cin, cout, k, stride=s), nn.BatchNorm1d(cout), nn.ReLU(True))

    def forward(self, x):
        return self.block(x)


class EncoderDecorder1D(EncoderDecorder):
    def __init__(self):
        nn.Module.__init__(self)
        self.encoder_pool1 = Pool1DBlock(2)
        self.encoder_res1 = Res1DBlock(32, 64)
        self.encoder_pool2 = Pool1DBlock(2)
        self.encoder_res2 = Res1DBlock(64, 128)
        self.mid_res = Res1DBlock(128, 128)
        self.decoder_res2 = Res1DBlock(128, 128)
        self.decoder_upsample2 = Upsample1DBlock(128, 64, 2, 2)
        self.decoder_res1 = Res1DBlock(64, 64)
        self.decoder_upsample1 = Upsample1DBlock(64, 32, 2, 2)
        self.skip_res1 = Res1DBlock(32, 32)
        self.skip_res2 = Res1DBlock(64, 64)


class C2CNet(nn.Module):
    def __init__(self, cin, cout, head_conv=32):
        super().__init__()
        self.output_channels = cout
        self.front_layers = nn.Sequential(Basic1DBlock(cin, 16, 7), Res1DBlock(16, 32))
        self.encoder_decoder = EncoderDecorder1D()
        self.output_hm = nn.Conv1d(32, cout, kernel_size=1)

    def forward(self, x):
        return self.output_hm(self.encoder_decoder(self.front_layers(x)))


# ---- WeightNet (weight_net.py:48-80) --------------------------------------------
class WeightNet(nn.Module):
    def __init__(self, num_joints, voxels=(64, 64), feat=32, hidden=64):
        super().__init__()
        self.voxels_per_axis = voxels
        self.num_joints = num_joints
        self.heatmap_feature_net = nn.Sequential(nn.Conv2d(1, feat, 3, stride=1, padding=1), nn.BatchNorm2d(feat),
                                                 nn.MaxPool2d(2), nn.ReLU(inplace=True))
        self.output = nn.Sequential(nn.Linear(feat, hidden), nn.ReLU(inplace=True), nn.Linear(hidden, 1),
                                    nn.Sigmoid())

    def forward(self, x):
        x = torch.flatten(x, 0, 1)
        b, j = x.shape[0], self.num_joints
        x = x.view(b * j, 1, self.voxels_per_axis[0], self.voxels_per_axis[1])
        x = F.adaptive_avg_pool2d(self.heatmap_feature_net(x), 1).view(b * j, -1)
        return self.output(x).view(b, j, 1)


# ---- PoseResNet (lib/models/resnet.py:19-215), same attribute names ------------------
def _bn(c):
    return nn.BatchNorm2d(c, momentum=0.1)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, planes, 3, stride, 1, bias=False)
        self.bn1 = _bn(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = _bn(planes)
        self.relu = nn.ReLU(inplace=True)
        self.downsample, self.stride = downsample, stride

    def forward(self, x):
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return self.relu(y + (x if self.downsample is None else self.downsample(x)))


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.bn1 = _bn(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = _bn(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = _bn(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample, self.stride = downsample, stride

    def forward(self, x):
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return self.relu(y + (x if self.downsample is None else self.downsample(x)))


RESNET_SPEC = {18: (BasicBlock, (2, 2, 2, 2)), 34: (BasicBlock, (3, 4, 6, 3)), 50: (Bottleneck, (3, 4, 6, 3)),
               101: (Bottleneck, (3, 4, 23, 3)), 152: (Bottleneck, (3, 8, 36, 3))}


class PoseResNet(nn.Module):
    """resnet.get(cfg): stem, four stages, deconvolution head, final conv."""

    def __init__(self, num_layers=50, num_joints=15, deconv_filters=(256, 256, 256), deconv_kernels=(4, 4, 4),
                 final_kernel=1, deconv_with_bias=False):
        super().__init__()
        block, counts = RESNET_SPEC[num_layers]
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = _bn(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        cin = 64
        for i, (planes, n) in enumerate(zip((64, 128, 256, 512), counts)):
            stride = 1 if i == 0 else 2
            down = None
            if stride != 1 or cin != planes * block.expansion:
                down = nn.Sequential(nn.Conv2d(cin, planes * block.expansion, 1, stride, bias=False),
                                     _bn(planes * block.expansion))
            blocks = [block(cin, planes, stride, down)]
            cin = planes * block.expansion
            blocks += [block(cin, planes) for _ in range(1, n)]
            setattr(self, f"layer{i + 1}", nn.Sequential(*blocks))
        head = []
        for f, k in zip(deconv_filters, deconv_kernels):
            pad, opad = {4: (1, 0), 3: (1, 1), 2: (0, 0)}[k]
            head += [nn.ConvTranspose2d(cin, f, k, 2, pad, opad, bias=deconv_with_bias), _bn(f), nn.ReLU(True)]
            cin = f
        self.deconv_layers = nn.Sequential(*head)
        self.final_layer = nn.Conv2d(cin, num_joints, final_kernel, 1, 1 if final_kernel == 3 else 0)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.final_layer(self.deconv_layers(x))
