"""Run every ``>>>`` example in the package's docstrings (the reference runs its examples as doctests,
pyproject.toml:13-20).  Examples are CPU-only and deterministic; they are generated from the library's own output by
``tools/gen_doc_examples.py``."""
import doctest
import importlib
import pkgutil

import pytest

import torchmetrics_forked_amd


def _modules_with_examples():
    out = []
    for info in pkgutil.walk_packages(torchmetrics_forked_amd.__path__, "torchmetrics_forked_amd."):
        if ".ops." in info.name or info.name.endswith(".ops"):
            continue
        try:
            mod = importlib.import_module(info.name)
        except Exception:  # optional-dependency modules
            continue
        src = getattr(mod, "__file__", None)
        if src and src.endswith(".py") and ">>>" in open(src).read():
            out.append(info.name)
    return sorted(set(out))


MODULES = _modules_with_examples()


def test_examples_exist():
    assert len(MODULES) >= 15, MODULES


@pytest.mark.parametrize("name", MODULES)
def test_docstring_examples(name):
    mod = importlib.import_module(name)
    res = doctest.testmod(mod, optionflags=doctest.NORMALIZE_WHITESPACE | doctest.ELLIPSIS, verbose=False)
    assert res.failed == 0, f"{res.failed} of {res.attempted} doctest lines failed in {name}"
