"""Optional-dependency flags (parity: reference ``utilities/imports.py:23-67``).

Every flag is computed with ``importlib.util.find_spec`` so importing the framework never imports heavy
optional packages eagerly.
"""
import importlib
import importlib.util
import operator
import shutil
import sys
from typing import Callable

import torch
from packaging.version import Version


def package_available(name: str) -> bool:
    try:
        return importlib.util.find_spec(name) is not None
    except (ModuleNotFoundError, ValueError):
        return False


def compare_version(package: str, op: Callable, version: str) -> bool:
    if not package_available(package):
        return False
    try:
        mod = importlib.import_module(package)
        return op(Version(Version(mod.__version__).base_version), Version(version))
    except Exception:  # pragma: no cover - broken installs
        return False


_PYTHON_VERSION = ".".join(map(str, sys.version_info[:3]))
_TORCH_VERSION = Version(Version(torch.__version__).base_version)
_TORCH_GREATER_EQUAL_1_11 = _TORCH_VERSION >= Version("1.11")
_TORCH_GREATER_EQUAL_1_12 = _TORCH_VERSION >= Version("1.12")
_TORCH_GREATER_EQUAL_1_13 = _TORCH_VERSION >= Version("1.13")
_TORCH_GREATER_EQUAL_2_0 = _TORCH_VERSION >= Version("2.0")
_TORCH_GREATER_EQUAL_2_1 = _TORCH_VERSION >= Version("2.1")
_ROCM = torch.version.hip is not None

_NLTK_AVAILABLE = package_available("nltk")
_ROUGE_SCORE_AVAILABLE = package_available("rouge_score")
_BERTSCORE_AVAILABLE = package_available("bert_score")
_SCIPY_AVAILABLE = package_available("scipy")
_SKLEARN_AVAILABLE = package_available("sklearn")
_TORCH_FIDELITY_AVAILABLE = package_available("torch_fidelity")
_LPIPS_AVAILABLE = package_available("lpips")
_PYCOCOTOOLS_AVAILABLE = package_available("pycocotools")
_FASTER_COCO_EVAL_AVAILABLE = package_available("faster_coco_eval")
_TORCHVISION_AVAILABLE = package_available("torchvision")
_TORCHAUDIO_AVAILABLE = package_available("torchaudio")
_TRANSFORMERS_AVAILABLE = package_available("transformers")
_REGEX_AVAILABLE = package_available("regex")
_PESQ_AVAILABLE = package_available("pesq")
_GAMMATONE_AVAILABLE = package_available("gammatone")
_PYSTOI_AVAILABLE = package_available("pystoi")
_FAST_BSS_EVAL_AVAILABLE = package_available("fast_bss_eval")
_MATPLOTLIB_AVAILABLE = package_available("matplotlib")
_SCIENCEPLOT_AVAILABLE = package_available("scienceplots")
_MULTIPROCESSING_AVAILABLE = package_available("multiprocessing")
_XLA_AVAILABLE = package_available("torch_xla")
_PIQ_GREATER_EQUAL_0_8 = compare_version("piq", operator.ge, "0.8.0")
_MECAB_AVAILABLE = package_available("MeCab")
_MECAB_KO_AVAILABLE = package_available("mecab_ko")
_MECAB_KO_DIC_AVAILABLE = package_available("mecab_ko_dic")
_IPADIC_AVAILABLE = package_available("ipadic")
_SENTENCEPIECE_AVAILABLE = package_available("sentencepiece")
_LATEX_AVAILABLE = shutil.which("latex") is not None
_TORCHVISION_GREATER_EQUAL_0_8 = compare_version("torchvision", operator.ge, "0.8.0")
_TORCHVISION_GREATER_EQUAL_0_13 = compare_version("torchvision", operator.ge, "0.13.0")
_TRANSFORMERS_GREATER_EQUAL_4_4 = compare_version("transformers", operator.ge, "4.4.0")
_TRANSFORMERS_GREATER_EQUAL_4_10 = compare_version("transformers", operator.ge, "4.10.0")
