"""Every plot entry point renders (Agg backend) for the value layouts metrics produce."""
import matplotlib
import pytest
import torch

matplotlib.use("Agg")

import torchmetrics_forked_amd as tm  # noqa: E402
from torchmetrics_forked_amd.utilities.plot import (  # noqa: E402
    _get_col_row_split,
    plot_confusion_matrix,
    plot_curve,
    plot_single_or_multi_val,
)


@pytest.fixture(autouse=True)
def _close_figures():
    yield
    import matplotlib.pyplot as plt

    plt.close("all")


@pytest.mark.parametrize(
    "val",
    [
        torch.tensor(0.5),
        torch.rand(4),
        {"a": torch.tensor(0.1), "b": torch.tensor(0.7)},
        {"a": torch.rand(5)},
        [torch.tensor(0.1), torch.tensor(0.4), torch.tensor(0.3)],
        [torch.rand(3) for _ in range(4)],
        [{"a": torch.tensor(0.1), "b": torch.tensor(0.2)}, {"a": torch.tensor(0.3), "b": torch.tensor(0.1)}],
    ],
)
@pytest.mark.parametrize("hib", [None, True, False])
def test_value_layouts(val, hib):
    fig, ax = plot_single_or_multi_val(val, higher_is_better=hib, lower_bound=0.0, upper_bound=1.0, legend_name="Class", name="m")
    assert ax.get_ylabel() == "m"
    lo, hi = ax.get_ylim()
    assert lo <= 0.0 and hi >= 1.0


def test_confusion_matrix_and_curves():
    _, ax = plot_confusion_matrix(torch.randint(0, 9, (3, 3)), labels=["x", "y", "z"])
    assert [t.get_text() for t in ax.get_xticklabels()] == ["x", "y", "z"]
    _, axs = plot_confusion_matrix(torch.randint(0, 9, (5, 2, 2)))
    assert len(axs) == 5
    with pytest.raises(ValueError, match="labels"):
        plot_confusion_matrix(torch.zeros(3, 3), labels=["a"])
    x = torch.linspace(0, 1, 10)
    _, ax = plot_curve((x, x**2), score=torch.tensor(0.33), label_names=("FPR", "TPR"))
    assert ax.get_xlabel() == "FPR"
    _, ax = plot_curve(([x, x], [x, x**2]), score=torch.tensor([0.5, 0.33]), legend_name="Class")
    assert len(ax.get_legend().get_texts()) == 2
    with pytest.raises(ValueError):
        plot_curve((x,))
    assert [_get_col_row_split(n) for n in (1, 2, 4, 5, 7, 10)] == [(1, 1), (1, 2), (2, 2), (2, 3), (3, 3), (3, 4)]


def test_metric_plot_methods():
    m = tm.MulticlassAccuracy(num_classes=3, average=None)
    m.update(torch.randn(20, 3), torch.randint(0, 3, (20,)))
    m.plot()
    cm = tm.MulticlassConfusionMatrix(num_classes=3)
    cm.update(torch.randn(20, 3), torch.randint(0, 3, (20,)))
    cm.plot()
    roc = tm.BinaryROC()
    roc.update(torch.rand(30), torch.randint(0, 2, (30,)))
    roc.plot(score=True)
    coll = tm.MetricCollection([tm.BinaryAccuracy(), tm.BinaryPrecision()])
    coll.update(torch.rand(10), torch.randint(0, 2, (10,)))
    coll.plot()
    tr = tm.wrappers.MetricTracker(tm.BinaryAccuracy())
    for _ in range(3):
        tr.increment()
        tr.update(torch.rand(10), torch.randint(0, 2, (10,)))
    tr.plot()
