"""Model-based image metrics: LPIPS, FID, KID, Inception Score, MiFID, perceptual path length (API parity:
reference ``image/{lpip,fid,kid,inception,mifid,perceptual_path_length}.py``).

FID keeps the reference's fp64 ``sum`` states (feature sum + Gram ``XᵀX``), so DDP sync is one all-reduce; on the
GPU the update is one fused in-place launch (``fid_gram_update``: fp64 MFMA over the upper tiles, mirrored, plus the
feature sums, from the raw features -- no fp64 copy, no new F x F matrix).  ``trace(sqrtm(Σ1·Σ2))`` is evaluated through the symmetric
form ``√Σ1·Σ2·√Σ1`` with two symmetric eigensolvers (``eigh``), which stays on the GPU, instead of the general
non-symmetric ``eigvals`` of the reference (same eigenvalues).  KID's compute runs every subset in one fused launch
(``kid_poly_sums``: the three polynomial-kernel sums of ``poly_mmd`` with the subset rows gathered in the kernel)."""
from copy import deepcopy
from typing import Any, ClassVar, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from torch.nn import Module
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.image.lpips import _lpips_compute, _lpips_update, _NoTrainLpips
from torchmetrics_forked_amd.functional.image.perceptual_path_length import (
    GeneratorType,
    _perceptual_path_length_validate_arguments,
    _validate_generator_model,
    perceptual_path_length,
)
from torchmetrics_forked_amd.functional.image.lpips import _LPIPS
from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.models.inception import FeatureExtractorInceptionV3
from torchmetrics_forked_amd.utilities.data import dim_zero_cat
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE
from torchmetrics_forked_amd.utilities.prints import rank_zero_warn


class NoTrainInceptionV3(FeatureExtractorInceptionV3):
    """Inception-v3 ("inception-v3-compat" layout) feature extractor pinned to eval mode."""

    def __init__(self, name: str = "inception-v3-compat", features_list: Sequence[str] = ("2048",),
                 feature_extractor_weights_path: Optional[str] = None) -> None:
        super().__init__(features_list, weights_path=feature_extractor_weights_path)


def _sqrtm_psd(mat: Tensor) -> Tensor:
    w, v = torch.linalg.eigh(mat)
    return (v * w.clamp(min=0).sqrt().unsqueeze(0)) @ v.T


_GRAM_MAX_FEATURES = 16384  # csrc/pairwise.hip fid_gram_update's TORCH_CHECK


def _gram_kernel_ok(features: Tensor) -> bool:
    """Feature widths the fused Gram kernel takes: below 256 the triangle holds too few 64 x 64 tiles to fill the GPU
    (0.8x at 512 x 192 fp32), above 16384 the kernel refuses the width."""
    return features.dim() == 2 and 256 <= features.shape[1] <= _GRAM_MAX_FEATURES


def _fused_moments(features: Tensor, gram: Tensor, fsum: Tensor) -> bool:
    """``csrc/pairwise.hip`` ``fid_gram_update`` for GPU float features into contiguous fp64 states on their device
    (``profiles/fid_gram_r5.json``); otherwise the reference's ``double()`` + ``sum`` + ``addmm``."""
    return (features.is_cuda and features.is_floating_point() and _gram_kernel_ok(features)
            and gram.dtype == torch.float64
            and fsum.dtype == torch.float64 and gram.device == features.device and fsum.device == features.device
            and gram.is_contiguous() and fsum.is_contiguous() and ops.use_native(features, gram, fsum))


def _compute_fid(mu1: Tensor, sigma1: Tensor, mu2: Tensor, sigma2: Tensor) -> Tensor:
    """‖μ1−μ2‖² + tr Σ1 + tr Σ2 − 2·Σ√λ(Σ1Σ2), eigenvalues from the symmetric PSD product √Σ1·Σ2·√Σ1."""
    a = (mu1 - mu2).square().sum(dim=-1)
    b = sigma1.trace() + sigma2.trace()
    s1 = _sqrtm_psd((sigma1 + sigma1.T) / 2)
    m = s1 @ sigma2 @ s1
    c = torch.linalg.eigvalsh((m + m.T) / 2).clamp(min=0).sqrt().sum(dim=-1)
    return a + b - 2 * c


def _resolve_inception(feature: Union[int, str, Module], valid: Sequence[Any]) -> Tuple[Module, Optional[int]]:
    if isinstance(feature, (int, str)) and not isinstance(feature, bool):
        if feature not in valid:
            raise ValueError(f"Integer input to argument `feature` must be one of {tuple(valid)}, but got {feature}.")
        return NoTrainInceptionV3(features_list=[str(feature)]), None
    if isinstance(feature, Module):
        return feature, None
    raise TypeError("Got unknown input to argument `feature`")


class FrechetInceptionDistance(Metric):
    higher_is_better: bool = False
    is_differentiable: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0

    def __init__(self, feature: Union[int, Module] = 2048, reset_real_features: bool = True, normalize: bool = False,
                 **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.inception, _ = _resolve_inception(feature, (64, 192, 768, 2048))
        if isinstance(feature, int):
            num_features = feature
        else:
            num_features = self.inception(torch.randint(0, 255, (1, 3, 299, 299), dtype=torch.uint8)).shape[-1]
        if not isinstance(reset_real_features, bool):
            raise ValueError("Argument `reset_real_features` expected to be a bool")
        self.reset_real_features = reset_real_features
        if not isinstance(normalize, bool):
            raise ValueError("Argument `normalize` expected to be a bool")
        self.normalize = normalize
        mx = (num_features, num_features)
        self.add_state("real_features_sum", torch.zeros(num_features).double(), dist_reduce_fx="sum")
        self.add_state("real_features_cov_sum", torch.zeros(mx).double(), dist_reduce_fx="sum")
        self.add_state("real_features_num_samples", torch.tensor(0).long(), dist_reduce_fx="sum")
        self.add_state("fake_features_sum", torch.zeros(num_features).double(), dist_reduce_fx="sum")
        self.add_state("fake_features_cov_sum", torch.zeros(mx).double(), dist_reduce_fx="sum")
        self.add_state("fake_features_num_samples", torch.tensor(0).long(), dist_reduce_fx="sum")

    def update(self, imgs: Tensor, real: bool) -> None:
        imgs = (imgs * 255).byte() if self.normalize else imgs
        features = self.inception(imgs)
        self.orig_dtype = features.dtype
        if features.dim() == 1:
            features = features.unsqueeze(0)
        prefix = "real" if real else "fake"
        fsum, gram = getattr(self, f"{prefix}_features_sum"), getattr(self, f"{prefix}_features_cov_sum")
        if _fused_moments(features, gram, fsum):
            # one launch, in place: fp64 Gram (upper tiles, mirrored) + feature sums from the raw features
            torch.ops.tmx.fid_gram_update(features.detach(), gram, fsum)
        else:
            features = features.double()
            setattr(self, f"{prefix}_features_sum", fsum + features.sum(dim=0))
            setattr(self, f"{prefix}_features_cov_sum", gram.addmm(features.t(), features))
        setattr(self, f"{prefix}_features_num_samples", getattr(self, f"{prefix}_features_num_samples") + imgs.shape[0])

    def _moments(self, prefix: str) -> Tuple[Tensor, Tensor]:
        n = getattr(self, f"{prefix}_features_num_samples")
        mean = (getattr(self, f"{prefix}_features_sum") / n).unsqueeze(0)
        cov = (getattr(self, f"{prefix}_features_cov_sum") - n * mean.t().mm(mean)) / (n - 1)
        return mean.squeeze(0), cov

    def compute(self) -> Tensor:
        if self.real_features_num_samples < 2 or self.fake_features_num_samples < 2:
            raise RuntimeError("More than one sample is required for both the real and fake distributed to compute FID")
        mr, cr = self._moments("real")
        mf, cf = self._moments("fake")
        return _compute_fid(mr, cr, mf, cf).to(getattr(self, "orig_dtype", torch.float32))

    def reset(self) -> None:
        if not self.reset_real_features:
            keep = {k: deepcopy(getattr(self, k)) for k in ("real_features_sum", "real_features_cov_sum", "real_features_num_samples")}
            super().reset()
            for k, v in keep.items():
                setattr(self, k, v)
        else:
            super().reset()

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


def maximum_mean_discrepancy(k_xx: Tensor, k_xy: Tensor, k_yy: Tensor) -> Tensor:
    m = k_xx.shape[0]
    kt_xx = k_xx.sum() - torch.diag(k_xx).sum()
    kt_yy = k_yy.sum() - torch.diag(k_yy).sum()
    value = (kt_xx + kt_yy) / (m * (m - 1))
    return value - 2 * k_xy.sum() / m**2


def poly_kernel(f1: Tensor, f2: Tensor, degree: int = 3, gamma: Optional[float] = None, coef: float = 1.0) -> Tensor:
    if gamma is None:
        gamma = 1.0 / f1.shape[1]
    return (f1 @ f2.T * gamma + coef) ** degree


def poly_mmd(f_real: Tensor, f_fake: Tensor, degree: int = 3, gamma: Optional[float] = None, coef: float = 1.0) -> Tensor:
    return maximum_mean_discrepancy(
        poly_kernel(f_real, f_real, degree, gamma, coef), poly_kernel(f_real, f_fake, degree, gamma, coef),
        poly_kernel(f_fake, f_fake, degree, gamma, coef),
    )


class KernelInceptionDistance(Metric):
    higher_is_better: bool = False
    is_differentiable: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(self, feature: Union[str, int, Module] = 2048, subsets: int = 100, subset_size: int = 1000,
                 degree: int = 3, gamma: Optional[float] = None, coef: float = 1.0, reset_real_features: bool = True,
                 normalize: bool = False, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        rank_zero_warn(
            "Metric `Kernel Inception Distance` will save all extracted features in buffer."
            " For large datasets this may lead to large memory footprint.",
            UserWarning,
        )
        self.inception, _ = _resolve_inception(feature, ("logits_unbiased", 64, 192, 768, 2048))
        if not (isinstance(subsets, int) and subsets > 0):
            raise ValueError("Argument `subsets` expected to be integer larger than 0")
        self.subsets = subsets
        if not (isinstance(subset_size, int) and subset_size > 0):
            raise ValueError("Argument `subset_size` expected to be integer larger than 0")
        self.subset_size = subset_size
        if not (isinstance(degree, int) and degree > 0):
            raise ValueError("Argument `degree` expected to be integer larger than 0")
        self.degree = degree
        if gamma is not None and not (isinstance(gamma, float) and gamma > 0):
            raise ValueError("Argument `gamma` expected to be `None` or float larger than 0")
        self.gamma = gamma
        if not (isinstance(coef, float) and coef > 0):
            raise ValueError("Argument `coef` expected to be float larger than 0")
        self.coef = coef
        if not isinstance(reset_real_features, bool):
            raise ValueError("Argument `reset_real_features` expected to be a bool")
        self.reset_real_features = reset_real_features
        if not isinstance(normalize, bool):
            raise ValueError("Argument `normalize` expected to be a bool")
        self.normalize = normalize
        self.add_state("real_features", [], dist_reduce_fx=None)
        self.add_state("fake_features", [], dist_reduce_fx=None)

    def update(self, imgs: Tensor, real: bool) -> None:
        imgs = (imgs * 255).byte() if self.normalize else imgs
        features = self.inception(imgs)
        (self.real_features if real else self.fake_features).append(features)

    def compute(self) -> Tuple[Tensor, Tensor]:
        real = dim_zero_cat(self.real_features)
        fake = dim_zero_cat(self.fake_features)
        if real.shape[0] < self.subset_size:
            raise ValueError("Argument `subset_size` should be smaller than the number of samples")
        if fake.shape[0] < self.subset_size:
            raise ValueError("Argument `subset_size` should be smaller than the number of samples")
        scores = []
        if (real.is_cuda and real.is_floating_point() and real.dtype == fake.dtype and real.dim() == 2 and fake.dim() == 2
                and not torch.are_deterministic_algorithms_enabled() and ops.use_native(real, fake)):
            # every subset in one fused launch (csrc/pairwise.hip kid_poly_sums: the three polynomial-kernel sums per
            # subset, rows gathered through the subset indices); the subsets are the same host randperm draws, in the
            # same order, as the reference's loop.  The per-workgroup partials are combined by fp64 atomics, so the
            # last bits of a score can differ between runs (the reference's reduction order is fixed); under
            # torch.use_deterministic_algorithms(True) the reference's loop runs instead
            m = self.subset_size
            gamma = self.gamma if self.gamma is not None else 1.0 / real.shape[1]
            draws = [(torch.randperm(real.shape[0])[:m], torch.randperm(fake.shape[0])[:m]) for _ in range(self.subsets)]
            ir = torch.stack([d[0] for d in draws])
            jf = torch.stack([d[1] for d in draws])
            sums = torch.ops.tmx.kid_poly_sums(real, fake, ir, jf, int(self.degree), float(gamma), float(self.coef))
            scores = list(((sums[:, 0] + sums[:, 1]) / (m * (m - 1)) - 2 * sums[:, 2] / m**2).to(real.dtype))
        else:
            for _ in range(self.subsets):
                f_real = real[torch.randperm(real.shape[0])[: self.subset_size]]
                f_fake = fake[torch.randperm(fake.shape[0])[: self.subset_size]]
                scores.append(poly_mmd(f_real, f_fake, self.degree, self.gamma, self.coef))
        scores_t = torch.stack(scores)
        return scores_t.mean(), scores_t.std(unbiased=False)

    def reset(self) -> None:
        if not self.reset_real_features:
            value = self._defaults.pop("real_features")
            super().reset()
            self._defaults["real_features"] = value
        else:
            super().reset()

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        val = val if val is not None else self.compute()[0]
        return self._plot(val, ax)


class InceptionScore(Metric):
    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0

    def __init__(self, feature: Union[str, int, Module] = "logits_unbiased", splits: int = 10, normalize: bool = False,
                 **kwargs: Any) -> None:
        super().__init__(**kwargs)
        rank_zero_warn(
            "Metric `InceptionScore` will save all extracted features in buffer."
            " For large datasets this may lead to large memory footprint.",
            UserWarning,
        )
        self.inception, _ = _resolve_inception(feature, ("logits_unbiased", 64, 192, 768, 2048))
        if not isinstance(normalize, bool):
            raise ValueError("Argument `normalize` expected to be a bool")
        self.normalize = normalize
        self.splits = splits
        self.add_state("features", [], dist_reduce_fx=None)

    def update(self, imgs: Tensor) -> None:
        imgs = (imgs * 255).byte() if self.normalize else imgs
        self.features.append(self.inception(imgs))

    def compute(self) -> Tuple[Tensor, Tensor]:
        features = dim_zero_cat(self.features)
        features = features[torch.randperm(features.shape[0])]
        prob = features.softmax(dim=1).chunk(self.splits, dim=0)
        log_prob = features.log_softmax(dim=1).chunk(self.splits, dim=0)
        kl = torch.stack([
            (p * (lp - p.mean(dim=0, keepdim=True).log())).sum(dim=1).mean().exp() for p, lp in zip(prob, log_prob)
        ])
        return kl.mean(), kl.std()

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        val = val if val is not None else self.compute()[0]
        return self._plot(val, ax)


def _rowmax_fused_wins(f1: Tensor, f2: Tensor) -> bool:
    """The fused row-max kernel: fp32 with >= 256 128 x 128 tiles runs on f16 matrix cores (a two-plane split of
    every fp32 row, three products; 2.4x over normalise + hipBLASLt matmul + min at 10,000 x 10,000 x 2048); smaller
    fp32 / fp64 products take its exact fp32 / fp64 MFMA tiles while the launches and the N x M round trips dominate."""
    work = f1.shape[0] * f2.shape[0] * f1.shape[1]
    if f1.dtype == torch.float32 and ((f1.shape[0] + 127) // 128) * ((f2.shape[0] + 127) // 128) >= 256:
        return True  # the f16-split matrix-core route (10,000^2 x 2048: 1.64 vs 3.87 ms, profiles/mifid_rowmax_r6.json)
        return work <= (1 << 29) and f1.shape[1] <= 256
    if f1.dtype in (torch.bfloat16, torch.float16):
        return work <= (1 << 29)
    return work < (1 << 32) and f1.shape[1] <= 1024


def _compute_cosine_distance(features1: Tensor, features2: Tensor, cosine_distance_eps: float = 0.1) -> Tensor:
    f1 = features1[torch.sum(features1, dim=1) != 0]
    f2 = features2[torch.sum(features2, dim=1) != 0]
    if (f1.is_cuda and f1.is_floating_point() and f1.dtype == f2.dtype and f1.dim() == 2 and f2.shape[0] > 0
            and f1.shape[1] > 0 and _rowmax_fused_wins(f1, f2) and ops.use_native(f1, f2)):
        # one fused launch: the row maxima of |cos| without the N x M similarity matrix (csrc/pairwise.hip)
        mean_min_d = torch.mean(1.0 - torch.ops.tmx.pairwise_abs_cos_rowmax(f1, f2)).to(f1.dtype)
        # the kernel's fmax skips NaN cosines; the reference's ``min`` propagates them (any non-finite feature makes a
        # NaN row or column): restore that without a host sync
        finite = torch.isfinite(f1).all() & torch.isfinite(f2).all()
        mean_min_d = torch.where(finite, mean_min_d, torch.full_like(mean_min_d, float("nan")))
    else:
        n1 = f1 / torch.norm(f1, dim=1, keepdim=True)
        n2 = f2 / torch.norm(f2, dim=1, keepdim=True)
        d = 1.0 - torch.abs(n1 @ n2.t())
        mean_min_d = torch.mean(d.min(dim=1).values)
    return mean_min_d if mean_min_d < cosine_distance_eps else torch.ones_like(mean_min_d)


def _mifid_compute(mu1: Tensor, sigma1: Tensor, features1: Tensor, mu2: Tensor, sigma2: Tensor, features2: Tensor,
                   cosine_distance_eps: float = 0.1) -> Tensor:
    fid_value = _compute_fid(mu1, sigma1, mu2, sigma2)
    distance = _compute_cosine_distance(features1, features2, cosine_distance_eps)
    return fid_value / (distance + 10e-15) if fid_value > 1e-8 else torch.zeros_like(fid_value)


class MemorizationInformedFrechetInceptionDistance(Metric):
    higher_is_better: bool = False
    is_differentiable: bool = False
    full_state_update: bool = False

    def __init__(self, feature: Union[int, Module] = 2048, reset_real_features: bool = True, normalize: bool = False,
                 cosine_distance_eps: float = 0.1, **kwargs: Any) -> None:
        super().__init__(**kwargs)
        self.inception, _ = _resolve_inception(feature, (64, 192, 768, 2048))
        if not isinstance(reset_real_features, bool):
            raise ValueError("Argument `reset_real_features` expected to be a bool")
        self.reset_real_features = reset_real_features
        if not isinstance(normalize, bool):
            raise ValueError("Argument `normalize` expected to be a bool")
        self.normalize = normalize
        if not (isinstance(cosine_distance_eps, float) and 1 >= cosine_distance_eps > 0):
            raise ValueError("Argument `cosine_distance_eps` expected to be a float greater than 0 and less than 1")
        self.cosine_distance_eps = cosine_distance_eps
        self.add_state("real_features", [], dist_reduce_fx=None)
        self.add_state("fake_features", [], dist_reduce_fx=None)

    def update(self, imgs: Tensor, real: bool) -> None:
        imgs = (imgs * 255).byte() if self.normalize else imgs
        features = self.inception(imgs)
        self.orig_dtype = features.dtype
        (self.real_features if real else self.fake_features).append(features.double())

    def compute(self) -> Tensor:
        real, fake = dim_zero_cat(self.real_features), dim_zero_cat(self.fake_features)
        mr, mf = real.mean(dim=0), fake.mean(dim=0)
        cr, cf = torch.cov(real.t()), torch.cov(fake.t())
        return _mifid_compute(mr, cr, real, mf, cf, fake, cosine_distance_eps=self.cosine_distance_eps).to(self.orig_dtype)

    def reset(self) -> None:
        if not self.reset_real_features:
            value = self._defaults.pop("real_features")
            super().reset()
            self._defaults["real_features"] = value
        else:
            super().reset()

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class LearnedPerceptualImagePatchSimilarity(Metric):
    is_differentiable: bool = True
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    __jit_ignored_attributes__: ClassVar[List[str]] = ["device", "_fast_update", "net"]

    def __init__(self, net_type: Literal["vgg", "alex", "squeeze"] = "alex", reduction: Literal["sum", "mean"] = "mean",
                 normalize: bool = False, model_path: Optional[str] = None, backbone_weights: Optional[str] = None,
                 **kwargs: Any) -> None:
        super().__init__(**kwargs)
        valid = ("vgg", "alex", "squeeze")
        if net_type not in valid:
            raise ValueError(f"Argument `net_type` must be one of {valid}, but got {net_type}.")
        self.net = _NoTrainLpips(net=net_type, model_path=model_path, backbone_weights=backbone_weights)
        if reduction not in ("mean", "sum"):
            raise ValueError(f"Argument `reduction` must be one of {('mean', 'sum')}, but got {reduction}")
        self.reduction = reduction
        if not isinstance(normalize, bool):
            raise ValueError(f"Argument `normalize` should be an bool but got {normalize}")
        self.normalize = normalize
        self.add_state("sum_scores", torch.tensor(0.0), dist_reduce_fx="sum")
        self.add_state("total", torch.tensor(0.0), dist_reduce_fx="sum")

    def update(self, img1: Tensor, img2: Tensor, detach: bool = False) -> None:
        loss, total = _lpips_update(img1, img2, net=self.net, normalize=self.normalize)
        self.sum_scores += loss.sum().detach() if detach else loss.sum()
        self.total += total

    def compute(self) -> Tensor:
        return _lpips_compute(self.sum_scores, self.total, self.reduction)

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)


class PerceptualPathLength(Metric):
    is_differentiable: bool = False
    higher_is_better: Optional[bool] = True
    full_state_update: bool = True

    def __init__(self, num_samples: int = 10_000, conditional: bool = False, batch_size: int = 128,
                 interpolation_method: Literal["lerp", "slerp_any", "slerp_unit"] = "lerp", epsilon: float = 1e-4,
                 resize: Optional[int] = 64, lower_discard: Optional[float] = 0.01, upper_discard: Optional[float] = 0.99,
                 sim_net: Union[Module, Literal["alex", "vgg", "squeeze"]] = "vgg", **kwargs: Any) -> None:
        super().__init__(**kwargs)
        _perceptual_path_length_validate_arguments(num_samples, conditional, batch_size, interpolation_method, epsilon,
                                                   resize, lower_discard, upper_discard)
        self.num_samples = num_samples
        self.conditional = conditional
        self.batch_size = batch_size
        self.interpolation_method = interpolation_method
        self.epsilon = epsilon
        self.resize = resize
        self.lower_discard = lower_discard
        self.upper_discard = upper_discard
        if isinstance(sim_net, Module):
            self.net = sim_net
        elif sim_net in ("alex", "vgg", "squeeze"):
            self.net = _LPIPS(pretrained=True, net=sim_net, resize=resize)
        else:
            raise ValueError(f"sim_net must be a nn.Module or one of 'alex', 'vgg', 'squeeze', got {sim_net}")

    def update(self, generator: GeneratorType) -> None:
        _validate_generator_model(generator, self.conditional)
        self.generator = generator

    def compute(self) -> Tuple[Tensor, Tensor, Tensor]:
        return perceptual_path_length(
            generator=self.generator, num_samples=self.num_samples, conditional=self.conditional,
            interpolation_method=self.interpolation_method, epsilon=self.epsilon, resize=self.resize,
            lower_discard=self.lower_discard, upper_discard=self.upper_discard, sim_net=self.net, device=self.device,
        )
