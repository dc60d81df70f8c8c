"""``cat_dict_columns`` (csrc/py_columns.cpp, the library's CPython entry point): MeanAveragePrecision's batched update
reads the per-image dict columns in one C pass.  Host test (CPU tensors; the function is device-agnostic)."""
import pytest
import torch

from torchmetrics_forked_amd import ops

K, W = ("boxes", "scores", "labels"), (4, 0, 0)
GK, GW = ("boxes", "labels", "iscrowd", "area"), (4, 0, -1, -1)


@pytest.fixture(scope="module")
def pym():
    m = ops.py_module()
    if m is None:
        pytest.skip("native library not built")
    return m


def _batch(n=6, k=5):
    g = torch.Generator().manual_seed(0)
    return torch.rand(n, k, 4, generator=g), torch.rand(n, k, generator=g), torch.randint(0, 9, (n, k), generator=g)


def test_chained_items_give_views(pym):
    box, sc, lab = _batch()
    preds = [{"boxes": box[i], "scores": sc[i], "labels": lab[i]} for i in range(6)]
    (fb, fs, fl), rows = pym.cat_dict_columns(preds, K, W)
    assert rows == [5] * 6
    assert fb.data_ptr() == box.data_ptr() and fb.shape == (30, 4) and torch.equal(fb, box.view(-1, 4))
    assert fs.data_ptr() == sc.data_ptr() and torch.equal(fl, lab.view(-1))


def test_ragged_separate_items_are_concatenated(pym):
    items = [{"boxes": torch.rand(k, 4), "scores": torch.rand(k), "labels": torch.arange(k)} for k in (3, 1, 7)]
    (fb, fs, fl), rows = pym.cat_dict_columns(items, K, W)
    assert rows == [3, 1, 7]
    assert torch.equal(fb, torch.cat([i["boxes"] for i in items])) and torch.equal(fl, torch.cat([i["labels"] for i in items]))


def test_optional_columns(pym):
    box, _, lab = _batch()
    tg = [{"boxes": box[i], "labels": lab[i]} for i in range(6)]
    (fb, fl, crowd, area), rows = pym.cat_dict_columns(tg, GK, GW)
    assert crowd is None and area is None and rows == [5] * 6
    for i in range(6):
        tg[i]["iscrowd"] = torch.zeros(5, dtype=torch.long)
    (_, _, crowd, area), _ = pym.cat_dict_columns(tg, GK, GW)
    assert crowd.shape == (30,) and area is None


@pytest.mark.parametrize(
    "mutate",
    [
        lambda it: it[2].__setitem__("labels", it[2]["labels"][:3]),  # row count differs between columns
        lambda it: it[1].__setitem__("scores", it[1]["scores"].double()),  # mixed dtype in a column
        lambda it: it[0].__setitem__("boxes", it[0]["boxes"][:, :3]),  # wrong width
        lambda it: it[3].__setitem__("labels", [1, 2, 3, 4, 5]),  # not a tensor
        lambda it: it[4].pop("scores"),  # missing required key
        lambda it: it.__setitem__(1, 5),  # not a dict
        lambda it: [d.__setitem__(k, d[k][:0]) for d in it[:1] for k in K],  # an empty image
        lambda it: it[0].__setitem__("scores", it[0]["scores"].clone().requires_grad_()),
    ],
)
def test_non_uniform_batches_are_refused(pym, mutate):
    box, sc, lab = _batch()
    preds = [{"boxes": box[i], "scores": sc[i], "labels": lab[i]} for i in range(6)]
    mutate(preds)
    assert pym.cat_dict_columns(preds, K, W) is None


def test_partly_present_optional_column_is_refused(pym):
    box, _, lab = _batch()
    tg = [{"boxes": box[i], "labels": lab[i]} for i in range(6)]
    tg[2]["area"] = torch.ones(5)
    assert pym.cat_dict_columns(tg, GK, GW) is None


def test_bad_arguments_raise(pym):
    with pytest.raises(TypeError):
        pym.cat_dict_columns((), K, W)
    with pytest.raises(TypeError):
        pym.cat_dict_columns([], K, (4, 0))
