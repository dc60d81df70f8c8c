"""Python entry point for ``csrc/clustering.hip`` (expected mutual information on the GPU)."""
from torch import Tensor
import torch


def expected_mutual_info(a: Tensor, b: Tensor, n_samples: int) -> Tensor:
    """fp64 EMI of the row / column marginals ``a`` [R] and ``b`` [K] (one wave per cluster pair)."""
    return torch.ops.tmx.expected_mutual_info(a.double().contiguous(), b.double().contiguous(), float(n_samples))
