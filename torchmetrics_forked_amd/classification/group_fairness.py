"""Group-fairness modules (API parity: reference ``classification/group_fairness.py:35-330``).

States are per-group-id ``tp/fp/tn/fn [num_groups]`` counters filled by one bincount pass per update (see the
functional module).  Deliberate deviation: the reference adds each batch's *present* groups positionally
(``self.tp[i]`` for the i-th present group), which misattributes counts when a batch lacks some group; here
counts always land on their group id.  Both agree whenever every batch contains every group.
"""
from typing import Any, Dict, Optional

import torch
from torch import Tensor
from typing_extensions import Literal

from torchmetrics_forked_amd.functional.classification.group_fairness import (
    _compute_binary_demographic_parity,
    _compute_binary_equal_opportunity,
    _group_counts,
    _groups_validation,
)
from torchmetrics_forked_amd.functional.classification.stat_scores import (
    _binary_stat_scores_arg_validation,
    _binary_stat_scores_tensor_validation,
)
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE
from torchmetrics_forked_amd.utilities.prints import rank_zero_warn


class _AbstractGroupStatScores(Metric):
    tp: Tensor
    fp: Tensor
    tn: Tensor
    fn: Tensor

    def _create_states(self, num_groups: int) -> None:
        for s in ("tp", "fp", "tn", "fn"):
            self.add_state(s, torch.zeros(num_groups, dtype=torch.long), dist_reduce_fx="sum")

    def _update_groups(self, preds: Tensor, target: Tensor, groups: Tensor) -> None:
        if self.validate_args:
            _binary_stat_scores_tensor_validation(preds, target, "global", self.ignore_index)
            _groups_validation(groups, self.num_groups)
        counts = _group_counts(preds, target, groups, self.num_groups, self.threshold, self.ignore_index)
        self.tp += counts[:, 0]
        self.fp += counts[:, 1]
        self.tn += counts[:, 2]
        self.fn += counts[:, 3]


class BinaryGroupStatRates(_AbstractGroupStatScores):
    is_differentiable: bool = False
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(
        self,
        num_groups: int,
        threshold: float = 0.5,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if validate_args:
            _binary_stat_scores_arg_validation(threshold, "global", ignore_index)
        if not isinstance(num_groups, int) and num_groups < 2:
            raise ValueError(f"Expected argument `num_groups` to be an int larger than 1, but got {num_groups}")
        self.num_groups = num_groups
        self.threshold = threshold
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._create_states(num_groups)

    def update(self, preds: Tensor, target: Tensor, groups: Tensor) -> None:
        self._update_groups(preds, target, groups)

    def compute(self) -> Dict[str, Tensor]:
        results = torch.stack((self.tp, self.fp, self.tn, self.fn), dim=1)
        return {f"group_{i}": g / g.sum() for i, g in enumerate(results)}


class BinaryFairness(_AbstractGroupStatScores):
    is_differentiable: bool = False
    higher_is_better: bool = False
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0

    def __init__(
        self,
        num_groups: int,
        task: Literal["demographic_parity", "equal_opportunity", "all"] = "all",
        threshold: float = 0.5,
        ignore_index: Optional[int] = None,
        validate_args: bool = True,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        if task not in ("demographic_parity", "equal_opportunity", "all"):
            raise ValueError(
                f"Expected argument `task` to either be ``demographic_parity``,"
                f"``equal_opportunity`` or ``all`` but got {task}."
            )
        if validate_args:
            _binary_stat_scores_arg_validation(threshold, "global", ignore_index)
        if not isinstance(num_groups, int) and num_groups < 2:
            raise ValueError(f"Expected argument `num_groups` to be an int larger than 1, but got {num_groups}")
        self.num_groups = num_groups
        self.task = task
        self.threshold = threshold
        self.ignore_index = ignore_index
        self.validate_args = validate_args
        self._create_states(num_groups)

    def update(self, preds: Tensor, target: Optional[Tensor], groups: Tensor) -> None:
        if self.task == "demographic_parity":
            if target is not None:
                rank_zero_warn("The task demographic_parity does not require a target.", UserWarning)
            target = torch.zeros(preds.shape, dtype=torch.long, device=preds.device)
        self._update_groups(preds, target, groups)

    def compute(self) -> Dict[str, Tensor]:
        st = (self.tp, self.fp, self.tn, self.fn)
        if self.task == "demographic_parity":
            return _compute_binary_demographic_parity(*st)
        if self.task == "equal_opportunity":
            return _compute_binary_equal_opportunity(*st)
        return {**_compute_binary_demographic_parity(*st), **_compute_binary_equal_opportunity(*st)}

    def plot(self, val: Optional[Any] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        return self._plot(val, ax)
