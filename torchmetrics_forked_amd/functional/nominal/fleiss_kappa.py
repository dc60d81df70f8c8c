"""Fleiss kappa (API parity: reference ``functional/nominal/fleiss_kappa.py:20-110``)."""
import torch
from torch import Tensor
from typing_extensions import Literal


def _fleiss_kappa_update(ratings: Tensor, mode: Literal["counts", "probs"] = "counts") -> Tensor:
    """``[n_samples, n_categories]`` rater counts (``probs`` mode: per-rater argmax over the category dim)."""
    if mode == "probs":
        if ratings.ndim != 3 or not ratings.is_floating_point():
            raise ValueError(
                "If argument ``mode`` is 'probs', ratings must have 3 dimensions with the format"
                " [n_samples, n_categories, n_raters] and be floating point."
            )
        choice = ratings.argmax(dim=1)  # [n, raters]
        n_cat = max(ratings.shape[1], ratings.shape[2])
        counts = torch.zeros(choice.shape[0], n_cat, dtype=torch.long, device=ratings.device)
        counts.scatter_add_(1, choice, torch.ones_like(choice))
        return counts
    if mode == "counts" and (ratings.ndim != 2 or ratings.is_floating_point()):
        raise ValueError(
            "If argument ``mode`` is `counts`, ratings must have 2 dimensions with the format"
            " [n_samples, n_categories] and be none floating point."
        )
    return ratings


def _fleiss_kappa_compute(counts: Tensor) -> Tensor:
    total = counts.shape[0]
    num_raters = counts.sum(1).max()
    p_i = counts.sum(dim=0) / (total * num_raters)
    p_j = ((counts**2).sum(dim=1) - num_raters) / (num_raters * (num_raters - 1))
    p_bar = p_j.mean()
    pe_bar = (p_i**2).sum()
    return (p_bar - pe_bar) / (1 - pe_bar + 1e-5)


def fleiss_kappa(ratings: Tensor, mode: Literal["counts", "probs"] = "counts") -> Tensor:
    if mode not in ("counts", "probs"):
        raise ValueError("Argument ``mode`` must be one of ['counts', 'probs'].")
    return _fleiss_kappa_compute(_fleiss_kappa_update(ratings, mode))
