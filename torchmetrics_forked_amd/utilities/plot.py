"""Matplotlib rendering of metric values, confusion matrices and curves.

Public surface as in the reference (``utilities/plot.py``: ``plot_single_or_multi_val``, ``plot_confusion_matrix``,
``plot_curve``, ``trim_axs``, ``_AX_TYPE``, ``_PLOT_OUT_TYPE``).  Plotting is host-side presentation: every input is
first normalised into plain NumPy series (one device->host copy per tensor), then drawn by one renderer per kind.
"""
from itertools import product
from math import ceil, isqrt
from typing import Any, Dict, Iterator, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from torch import Tensor

from torchmetrics_forked_amd.utilities.imports import _MATPLOTLIB_AVAILABLE

if _MATPLOTLIB_AVAILABLE:
    import matplotlib

    matplotlib.use("Agg", force=False)
    import matplotlib.axes
    import matplotlib.pyplot as plt

    _PLOT_OUT_TYPE = Tuple[plt.Figure, Union[matplotlib.axes.Axes, np.ndarray]]
    _AX_TYPE = matplotlib.axes.Axes
else:  # pragma: no cover
    _PLOT_OUT_TYPE = Tuple[object, object]  # type: ignore[misc]
    _AX_TYPE = object  # type: ignore[misc]

_MARKER = {"marker": "o", "markersize": 10}


def _error_on_missing_matplotlib() -> None:
    if not _MATPLOTLIB_AVAILABLE:
        raise ModuleNotFoundError(
            "Plot function expects `matplotlib` to be installed. Please install with `pip install matplotlib`"
        )


def _host(x: Any) -> np.ndarray:
    return x.detach().cpu().numpy() if isinstance(x, Tensor) else np.asarray(x)


def _figure(ax: Optional[_AX_TYPE]) -> Tuple[Any, _AX_TYPE]:
    return plt.subplots() if ax is None else (None, ax)


# --------------------------------------------------------------------------------------------------------------
# metric values
# --------------------------------------------------------------------------------------------------------------
class _Series:
    """One drawable: y values at x positions, a legend label and whether points are joined."""

    __slots__ = ("x", "y", "label", "joined")

    def __init__(self, x: Sequence[float], y: Sequence[float], label: Optional[str], joined: bool) -> None:
        self.x, self.y, self.label, self.joined = x, y, label, joined


def _indexed_label(i: int, legend_name: Optional[str]) -> str:
    return f"{legend_name} {i}" if legend_name else f"{i}"


def _value_series(val: Any, legend_name: Optional[str]) -> Tuple[List[_Series], bool]:
    """Normalise the accepted value layouts into series; the flag says whether the x axis counts steps.

    * scalar tensor -> one point;  vector tensor -> one unjoined point per entry (class / label values);
    * dict of tensors -> one point per key, or a joined line per key when a value holds several steps;
    * sequence of tensors / dicts -> one joined line per entry (key) over the steps."""
    if isinstance(val, Tensor):
        if val.numel() == 1:
            return [_Series([0], [float(val.detach().cpu())], None, False)], False
        flat = _host(val).reshape(-1)
        return [_Series([i], [float(v)], _indexed_label(i, legend_name), False) for i, v in enumerate(flat)], False
    if isinstance(val, dict):
        out, steps = [], False
        for i, (key, v) in enumerate(val.items()):
            if v.numel() == 1:
                out.append(_Series([i], [float(v.detach().cpu())], key, False))
            else:
                ys = _host(v).reshape(-1)
                out.append(_Series(list(range(len(ys))), ys, key, True))
                steps = True
        return out, steps
    if isinstance(val, Sequence):
        if isinstance(val[0], dict):
            stacked = {k: _host(torch.stack([step[k] for step in val])) for k in val[0]}
            return [_Series(list(range(len(v))), v, k, True) for k, v in stacked.items()], True
        steps_by_entry = _host(torch.stack(list(val), 0))
        if steps_by_entry.ndim == 1:
            return [_Series(list(range(len(steps_by_entry))), steps_by_entry, "", True)], True
        return [
            _Series(list(range(steps_by_entry.shape[0])), col, _indexed_label(i, legend_name), True)
            for i, col in enumerate(steps_by_entry.T)
        ], True
    raise ValueError(f"Cannot plot a value of type {type(val)}")


def _mark_bounds(
    ax: _AX_TYPE, lower: Optional[float], upper: Optional[float], higher_is_better: Optional[bool]
) -> None:
    """Pad the y range by 10 %, draw the metric's bounds as dashed lines and flag the optimal one."""
    y0, y1 = ax.get_ylim()
    pad = 0.1 * ((upper - lower) if lower is not None and upper is not None else (y1 - y0))
    ax.set_ylim(bottom=(lower if lower is not None else y0) - pad, top=(upper if upper is not None else y1) + pad)
    x0, x1 = ax.get_xlim()
    ax.hlines([lower, upper] if lower and upper else (y0, y1), x0, x1, linestyles="dashed", colors="k")
    optimum = None
    if higher_is_better is True and upper is not None:
        optimum = upper
    elif higher_is_better is False and lower is not None:
        optimum = lower
    if optimum is not None:
        ax.set_xlim(x0 - 0.1 * (x1 - x0), x1)
        ax.text(x0, optimum, s="Optimal \n value", horizontalalignment="center", verticalalignment="center")


def plot_single_or_multi_val(
    val: Union[Tensor, Sequence[Tensor], Dict[str, Tensor], Sequence[Dict[str, Tensor]]],
    ax: Optional[_AX_TYPE] = None,
    higher_is_better: Optional[bool] = None,
    lower_bound: Optional[float] = None,
    upper_bound: Optional[float] = None,
    legend_name: Optional[str] = None,
    name: Optional[str] = None,
) -> _PLOT_OUT_TYPE:
    """Plot one metric value (a point per class / key) or a history of values (a line per class / key over steps)."""
    _error_on_missing_matplotlib()
    fig, ax = _figure(ax)
    series, over_steps = _value_series(val, legend_name)
    for s in series:
        style = {"linestyle": "-"} if s.joined else {"linestyle": "None"} if s.label is not None else {}
        ax.plot(s.x, s.y, label=s.label, **_MARKER, **style)
    ax.get_xaxis().set_visible(True)
    if over_steps:
        ax.set_xlabel("Step")
        ax.set_xticks(range(max(len(s.x) for s in series)))
    handles, labels = ax.get_legend_handles_labels()
    if handles and any(labels):
        ax.legend(handles, labels, loc="upper center", bbox_to_anchor=(0.5, 1.15), ncol=3, fancybox=True, shadow=True)
    _mark_bounds(ax, lower_bound, upper_bound, higher_is_better)
    ax.grid(True)
    ax.set_ylabel(name)
    return fig, ax


# --------------------------------------------------------------------------------------------------------------
# confusion matrices
# --------------------------------------------------------------------------------------------------------------
def _get_col_row_split(n: int) -> Tuple[int, int]:
    """(rows, cols) of the smallest near-square grid holding ``n`` panels."""
    side = isqrt(n)
    if side * side == n:
        return side, side
    return (side, side + 1) if side * (side + 1) >= n else (side + 1, side + 1)


def trim_axs(axs: Any, nb: int) -> Any:
    """Keep the first ``nb`` axes of a subplot grid and remove the others."""
    if isinstance(axs, _AX_TYPE):
        return axs
    flat = axs.flat
    for extra in flat[nb:]:
        extra.remove()
    return flat[:nb]


def _panels(axs: Any, n: int) -> Iterator[_AX_TYPE]:
    for i in range(n):
        yield axs if isinstance(axs, _AX_TYPE) else axs[i]


def _draw_confmat(a: _AX_TYPE, mat: np.ndarray, names: List[Any], add_text: bool, cmap: Optional[Any]) -> None:
    k = mat.shape[0]
    a.imshow(mat, cmap=cmap)
    a.set_xlabel("Predicted class", fontsize=15)
    a.set_ylabel("True class", fontsize=15)
    a.set_xticks(list(range(k)))
    a.set_yticks(list(range(k)))
    a.set_xticklabels(names, rotation=45, fontsize=10)
    a.set_yticklabels(names, rotation=25, fontsize=10)
    if add_text:
        for r, c in product(range(k), range(k)):
            v = mat[r, c].item()
            a.text(c, r, str(round(v, 2) if isinstance(v, float) else v), ha="center", va="center", fontsize=15)


def plot_confusion_matrix(
    confmat: Tensor,
    ax: Optional[_AX_TYPE] = None,
    add_text: bool = True,
    labels: Optional[List[Union[int, str]]] = None,
    cmap: Optional[Any] = None,
) -> _PLOT_OUT_TYPE:
    """Heatmap of a ``[C, C]`` confusion matrix, or one 2x2 panel per label of a ``[L, 2, 2]`` stack."""
    _error_on_missing_matplotlib()
    stacked = confmat.ndim == 3
    n_panels = confmat.shape[0] if stacked else 1
    k = 2 if stacked else confmat.shape[0]
    if labels is not None and not stacked and len(labels) != k:
        raise ValueError(
            "Expected number of elements in arg `labels` to match number of labels in confmat but "
            f"got {len(labels)} and {k}"
        )
    panel_titles = (labels or list(range(n_panels))) if stacked else None
    tick_names = [str(i) for i in range(k)] if stacked else (labels or list(range(k)))
    rows, cols = _get_col_row_split(n_panels) if stacked else (1, 1)
    fig, axs = plt.subplots(nrows=rows, ncols=cols) if ax is None else (ax.get_figure(), ax)
    axs = trim_axs(axs, n_panels)
    mats = _host(confmat)
    for i, a in enumerate(_panels(axs, n_panels)):
        if panel_titles is not None:
            a.set_title(f"Label {panel_titles[i]}", fontsize=15)
        _draw_confmat(a, mats[i] if stacked else mats, tick_names, add_text, cmap)
    return fig, axs


# --------------------------------------------------------------------------------------------------------------
# curves
# --------------------------------------------------------------------------------------------------------------
def plot_curve(
    curve: Union[Tuple[Tensor, Tensor, Tensor], Tuple[Tensor, Tensor], Tuple[List[Tensor], List[Tensor]]],
    score: Optional[Tensor] = None,
    ax: Optional[_AX_TYPE] = None,
    label_names: Optional[Tuple[str, str]] = None,
    legend_name: Optional[str] = None,
    name: Optional[str] = None,
) -> _PLOT_OUT_TYPE:
    """Plot an (x, y[, thresholds]) curve, or one curve per class / label, with the area score in the legend."""
    _error_on_missing_matplotlib()
    if len(curve) < 2:
        raise ValueError(f"Expected 2 or 3 elements in curve but got {len(curve)}")
    x, y = curve[0], curve[1]
    single = isinstance(x, Tensor) and isinstance(y, Tensor) and x.ndim == 1 and y.ndim == 1
    several = (isinstance(x, list) and isinstance(y, list)) or (isinstance(x, Tensor) and x.ndim == 2)
    if not (single or several):
        raise ValueError(
            f"Unknown format for argument `x` and `y`. Expected either list or tensors but got {type(x)} and {type(y)}."
        )
    fig, ax = _figure(ax)
    if single:
        label = f"AUC={score.item():0.3f}" if score is not None else None
        ax.plot(_host(x), _host(y), linestyle="-", linewidth=2, label=label)
        if label_names is not None:
            ax.set_xlabel(label_names[0])
            ax.set_ylabel(label_names[1])
        if label is not None:
            ax.legend()
    else:
        for i, (xi, yi) in enumerate(zip(x, y)):
            label = f"{legend_name}_{i}" if legend_name is not None else str(i)
            if score is not None:
                label += f" AUC={score[i].item():0.3f}"
            ax.plot(_host(xi), _host(yi), linestyle="-", linewidth=2, label=label)
        ax.legend()
    ax.grid(True)
    ax.set_title(name)
    return fig, ax
