"""Functional (stateless) metrics (API parity: reference ``functional/__init__.py``)."""
from torchmetrics_forked_amd.functional import (  # noqa: F401
    classification,
    clustering,
    image,
    nominal,
    pairwise,
    regression,
    retrieval,
)
from torchmetrics_forked_amd.functional.classification import *  # noqa: F401,F403
from torchmetrics_forked_amd.functional.image import *  # noqa: F401,F403
from torchmetrics_forked_amd.functional.nominal import *  # noqa: F401,F403
from torchmetrics_forked_amd.functional.pairwise import *  # noqa: F401,F403
from torchmetrics_forked_amd.functional.regression import *  # noqa: F401,F403
