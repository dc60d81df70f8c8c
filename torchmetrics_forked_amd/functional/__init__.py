"""Functional (stateless) metrics (API parity: reference ``functional/__init__.py``)."""
from torchmetrics_forked_amd.functional import classification, regression, retrieval  # noqa: F401
from torchmetrics_forked_amd.functional.classification import *  # noqa: F401,F403
from torchmetrics_forked_amd.functional.regression import *  # noqa: F401,F403
