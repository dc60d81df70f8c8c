"""Learned perceptual image patch similarity (API parity: reference ``functional/image/lpips.py:44-431``).

Backbones come from :mod:`torchmetrics_forked_amd.models` (torchvision-identical layer layout, randomly initialised
unless ``backbone_weights`` is given).  The per-layer head — channel L2-normalisation of both feature maps,
squared difference, 1×1 linear layer and spatial mean — runs as ONE fused gfx950 kernel per layer
(``tmx::lpips_head``) when no autograd graph is needed; with gradients (or on CPU) the eager formulation is used.
With ``pretrained=True`` the linear heads are the published LPIPS v0.1 weights shipped with the package
(``models/lpips_heads.safetensors``, the same values as the reference's ``lpips_models/{net}.pth``), or a LPIPS
``.pth`` given as ``model_path`` (loaded ``weights_only=True``).  The backbone trunks are random unless
``backbone_weights`` points at torchvision-layout weights (the reference downloads ImageNet weights; offline here).
"""
import os
from typing import List, NamedTuple, Optional, Tuple, Union

import torch
import torch.nn.functional as F
from torch import Tensor, nn
from typing_extensions import Literal

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.models.backbones import alexnet_features, squeezenet1_1_features, vgg16_features

_SLICES = {
    "alex": [range(0, 2), range(2, 5), range(5, 8), range(8, 10), range(10, 12)],
    "vgg": [range(0, 4), range(4, 9), range(9, 16), range(16, 23), range(23, 30)],
    "squeeze": [range(0, 2), range(2, 5), range(5, 8), range(8, 10), range(10, 11), range(11, 12), range(12, 13)],
}
_CHANNELS = {"alex": [64, 192, 384, 256, 256], "vgg": [64, 128, 256, 512, 512], "squeeze": [64, 128, 256, 384, 384, 512, 512]}
_FEATURES = {"alex": alexnet_features, "vgg": vgg16_features, "squeeze": squeezenet1_1_features}
# channels_last trunk on the fused GPU path (TMX_LPIPS_CHANNELS_LAST=0 keeps NCHW): MIOpen's NHWC convolutions run
# without its layout transposes (VGG16 trunk, 16 x 3 x 1024^2: 92.6 vs 101.1 ms, tools/lpips_layout_probe.py) and the
# head reads the channels_last maps in place with four threads per pixel; BASELINE config 4: 0.329 vs 0.303 updates/s
# (gpurun r7x; the first NHWC head, one thread per pixel, lost: 0.250, r7v / r7w)
_CHANNELS_LAST = os.environ.get("TMX_LPIPS_CHANNELS_LAST", "1") != "0"
# LPIPS v0.1 linear heads (``tools/convert_lpips_heads.py`` from the reference's lpips_models/*.pth): the default for
# ``pretrained=True``, as in the reference (``functional/image/lpips.py:318-325``)
_HEADS_FILE = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "models", "lpips_heads.safetensors")


class _SlicedBackbone(nn.Module):
    def __init__(self, net: str, requires_grad: bool = False, weights: Optional[str] = None) -> None:
        super().__init__()
        feats = _FEATURES[net]()
        if weights is not None:
            state = torch.load(weights, map_location="cpu", weights_only=True)
            state = {k[len("features."):]: v for k, v in state.items() if k.startswith("features.")} or state
            feats.load_state_dict(state)
        self.slices = nn.ModuleList(
            nn.Sequential(*[feats[i] for i in rng]) for rng in _SLICES[net]
        )
        for p in self.parameters():
            p.requires_grad_(requires_grad)

    def forward(self, x: Tensor) -> List[Tensor]:
        outs = []
        for s in self.slices:
            x = s(x)
            outs.append(x)
        return outs


class _NamedBackbone(_SlicedBackbone):
    """Public LPIPS trunks (reference ``functional/image/lpips.py:65-202``): ``forward`` returns a NamedTuple of
    the per-slice ReLU outputs.  ``pretrained=True`` loads torchvision-layout ``weights`` (a local file: nothing is
    downloaded); without a file the trunk stays randomly initialised."""

    _net = "alex"

    def __init__(self, requires_grad: bool = False, pretrained: bool = True, weights: Optional[str] = None) -> None:
        super().__init__(self._net, requires_grad=requires_grad, weights=weights if pretrained else None)
        self.N_slices = len(self.slices)
        fields = [(f"relu{i + 1}", Tensor) for i in range(self.N_slices)]
        if self._net == "vgg":
            fields = [(n, Tensor) for n in ("relu1_2", "relu2_2", "relu3_3", "relu4_3", "relu5_3")]
        self._out = NamedTuple(f"_{type(self).__name__}Output", fields)  # type: ignore[misc]

    def forward(self, x: Tensor) -> NamedTuple:  # type: ignore[override]
        return self._out(*super().forward(x))


class SqueezeNet(_NamedBackbone):
    """SqueezeNet-1.1 trunk, 7 slices."""

    _net = "squeeze"


class Alexnet(_NamedBackbone):
    """AlexNet trunk, 5 slices."""

    _net = "alex"


class Vgg16(_NamedBackbone):
    """VGG16 trunk, 5 slices."""

    _net = "vgg"


def _spatial_average(in_tens: Tensor, keep_dim: bool = True) -> Tensor:
    return in_tens.mean([2, 3], keepdim=keep_dim)


def _upsample(in_tens: Tensor, out_hw: Tuple[int, ...] = (64, 64)) -> Tensor:
    return F.interpolate(in_tens, size=out_hw, mode="bilinear", align_corners=False)


def _normalize_tensor(in_feat: Tensor, eps: float = 1e-8) -> Tensor:
    return in_feat / torch.sqrt(eps + torch.sum(in_feat**2, dim=1, keepdim=True))


def _resize_tensor(x: Tensor, size: int = 64) -> Tensor:
    if x.shape[-1] > size and x.shape[-2] > size:
        return F.interpolate(x, (size, size), mode="area")
    return F.interpolate(x, (size, size), mode="bilinear", align_corners=False)


class ScalingLayer(nn.Module):
    def __init__(self) -> None:
        super().__init__()
        self.register_buffer("shift", torch.tensor([-0.030, -0.088, -0.188])[None, :, None, None], persistent=False)
        self.register_buffer("scale", torch.tensor([0.458, 0.448, 0.450])[None, :, None, None], persistent=False)

    def forward(self, inp: Tensor) -> Tensor:
        return (inp - self.shift) / self.scale


class NetLinLayer(nn.Module):
    def __init__(self, chn_in: int, chn_out: int = 1, use_dropout: bool = False) -> None:
        super().__init__()
        layers: List[nn.Module] = [nn.Dropout()] if use_dropout else []
        layers += [nn.Conv2d(chn_in, chn_out, 1, stride=1, padding=0, bias=False)]
        self.model = nn.Sequential(*layers)

    def forward(self, x: Tensor) -> Tensor:
        return self.model(x)


class _LPIPS(nn.Module):
    def __init__(
        self,
        pretrained: bool = True,
        net: Literal["alex", "vgg", "squeeze"] = "alex",
        spatial: bool = False,
        pnet_rand: bool = False,
        pnet_tune: bool = False,
        use_dropout: bool = True,
        model_path: Optional[str] = None,
        eval_mode: bool = True,
        resize: Optional[int] = None,
        backbone_weights: Optional[str] = None,
    ) -> None:
        super().__init__()
        net = "vgg" if net == "vgg16" else net
        if net not in _CHANNELS:
            raise ValueError(f"Unknown LPIPS backbone {net}")
        self.pnet_type = net
        self.spatial = spatial
        self.resize = resize
        self.scaling_layer = ScalingLayer()
        self.chns = _CHANNELS[net]
        self.L = len(self.chns)
        self.net = _SlicedBackbone(net, requires_grad=pnet_tune, weights=backbone_weights)
        self.lins = nn.ModuleList(NetLinLayer(c, use_dropout=use_dropout) for c in self.chns)
        for i, lin in enumerate(self.lins):  # reference attribute names lin0..lin6 (state-dict compatible)
            setattr(self, f"lin{i}", lin)
        if pretrained:
            if model_path is not None:
                self.load_state_dict(torch.load(model_path, map_location="cpu", weights_only=True), strict=False)
            else:  # the published LPIPS v0.1 heads shipped with the package (reference lpips_models/{net}.pth)
                self._load_packaged_heads(net)
        if eval_mode:
            self.eval()

    def _load_packaged_heads(self, net: str) -> None:
        from safetensors.torch import load_file

        heads = load_file(_HEADS_FILE)
        with torch.no_grad():
            for i, lin in enumerate(self.lins):
                conv = lin.model[-1]
                conv.weight.copy_(heads[f"{net}.lin{i}"].reshape(conv.weight.shape))

    def forward(self, in0: Tensor, in1: Tensor, retperlayer: bool = False, normalize: bool = False) -> Union[Tensor, Tuple[Tensor, List[Tensor]]]:
        if normalize:
            in0, in1 = 2 * in0 - 1, 2 * in1 - 1
        x0, x1 = self.scaling_layer(in0), self.scaling_layer(in1)
        if self.resize is not None:
            x0, x1 = _resize_tensor(x0, size=self.resize), _resize_tensor(x1, size=self.resize)
        grad = torch.is_grad_enabled() and (in0.requires_grad or in1.requires_grad or any(p.requires_grad for p in self.parameters()))
        fused = (not self.spatial) and x0.is_cuda and not grad and not self.training and ops.use_native(x0)
        if fused and _CHANNELS_LAST and x0.dim() == 4:
            # channels_last trunk (see _CHANNELS_LAST): MIOpen's NHWC convolutions without its layout transposes; the
            # head reads the channels_last feature maps in place (tmx::lpips_head)
            if not self.__dict__.get("_trunk_cl"):
                self.net.to(memory_format=torch.channels_last)
                self.__dict__["_trunk_cl"] = True
            x0 = x0.contiguous(memory_format=torch.channels_last)
            x1 = x1.contiguous(memory_format=torch.channels_last)
        outs0, outs1 = self.net(x0), self.net(x1)
        res = []
        for kk in range(self.L):
            if fused:
                w = self.lins[kk].model[-1].weight.reshape(-1)
                res.append(torch.ops.tmx.lpips_head(outs0[kk], outs1[kk], w).to(outs0[kk].dtype).reshape(-1, 1, 1, 1))
                continue
            diff = (_normalize_tensor(outs0[kk]) - _normalize_tensor(outs1[kk])) ** 2
            if self.spatial:
                res.append(_upsample(self.lins[kk](diff), out_hw=tuple(in0.shape[2:])))
            else:
                res.append(_spatial_average(self.lins[kk](diff), keep_dim=True))
        val = sum(res)
        return (val, res) if retperlayer else val


class _NoTrainLpips(_LPIPS):
    def train(self, mode: bool = True) -> "_NoTrainLpips":
        return super().train(False)


def _valid_img(img: Tensor, normalize: bool) -> bool:
    value_check = img.max() <= 1.0 and img.min() >= 0.0 if normalize else img.min() >= -1
    return img.ndim == 4 and img.shape[1] == 3 and bool(value_check)


def _lpips_update(img1: Tensor, img2: Tensor, net: nn.Module, normalize: bool) -> Tuple[Tensor, Union[int, Tensor]]:
    if not (_valid_img(img1, normalize) and _valid_img(img2, normalize)):
        raise ValueError(
            "Expected both input arguments to be normalized tensors with shape [N, 3, H, W]."
            f" Got input with shape {img1.shape} and {img2.shape} and values in range"
            f" {[img1.min(), img1.max()]} and {[img2.min(), img2.max()]} when all values are"
            f" expected to be in the {[0, 1] if normalize else [-1, 1]} range."
        )
    n = img1.shape[0]
    chunk = _lpips_chunk(img1, net)
    if chunk >= n or torch.is_grad_enabled() and (img1.requires_grad or img2.requires_grad):
        loss = net(img1, img2, normalize=normalize).squeeze()
    else:  # bounded activation memory: the trunk's feature maps of a chunk, not of the whole batch
        loss = torch.cat([
            net(img1[i : i + chunk], img2[i : i + chunk], normalize=normalize).reshape(-1) for i in range(0, n, chunk)
        ]).squeeze()
    return loss, n


# feature-map channels kept alive per input pixel by each trunk (sum over the tapped stages of C / stride^2) — sizes
# the chunks of a large LPIPS batch (3x1024x1024 x 256 images through VGG16 would hold ~260 GB of activations)
_ACT_CHANNELS_PER_PIXEL = {"vgg": 128.0, "alex": 10.0, "squeeze": 12.0}
_LPIPS_ACT_BUDGET = float(os.environ.get("TMX_LPIPS_ACT_BUDGET_GB", "24")) * 2**30


def _lpips_chunk(img: Tensor, net: nn.Module) -> int:
    kind = getattr(net, "pnet_type", "vgg")
    per_image = 2 * 4 * img.shape[-1] * img.shape[-2] * _ACT_CHANNELS_PER_PIXEL.get(kind, 128.0) * 2  # both inputs, fp32, 2x slack
    return max(1, int(_LPIPS_ACT_BUDGET // per_image))


def _lpips_compute(sum_scores: Tensor, total: Union[Tensor, int], reduction: Literal["sum", "mean"] = "mean") -> Tensor:
    return sum_scores / total if reduction == "mean" else sum_scores


def learned_perceptual_image_patch_similarity(
    img1: Tensor,
    img2: Tensor,
    net_type: Literal["alex", "vgg", "squeeze"] = "alex",
    reduction: Literal["sum", "mean"] = "mean",
    normalize: bool = False,
) -> Tensor:
    net = _NoTrainLpips(net=net_type).to(img1.device)
    loss, total = _lpips_update(img1, img2, net, normalize)
    return _lpips_compute(loss.sum(), total, reduction)
