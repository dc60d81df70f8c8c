"""Total variation (API parity: reference ``functional/image/tv.py:20-80``)."""
from typing import Optional, Tuple, Union

from torch import Tensor
from typing_extensions import Literal


def _total_variation_update(img: Tensor) -> Tuple[Tensor, int]:
    if img.ndim != 4:
        raise RuntimeError(f"Expected input `img` to be an 4D tensor, but got {img.shape}")
    res1 = (img[..., 1:, :] - img[..., :-1, :]).abs().sum([1, 2, 3])
    res2 = (img[..., :, 1:] - img[..., :, :-1]).abs().sum([1, 2, 3])
    return res1 + res2, img.shape[0]


def _total_variation_compute(score: Tensor, num_elements: Union[int, Tensor], reduction: Optional[Literal["mean", "sum", "none"]]) -> Tensor:
    if reduction == "mean":
        return score.sum() / num_elements
    if reduction == "sum":
        return score.sum()
    if reduction is None or reduction == "none":
        return score
    raise ValueError("Expected argument `reduction` to either be 'sum', 'mean', 'none' or None")


def total_variation(img: Tensor, reduction: Optional[Literal["mean", "sum", "none"]] = "sum") -> Tensor:
    score, n = _total_variation_update(img)
    return _total_variation_compute(score, n, reduction)
