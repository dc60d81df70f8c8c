import importlib
import importlib.util
import operator
from typing import Callable

from packaging.version import Version


def package_available(name: str) -> bool:
    try:
        return importlib.util.find_spec(name) is not None
    except (ModuleNotFoundError, ValueError):
        return False


def compare_version(package: str, op: Callable, version: str, use_base_version: bool = False) -> bool:
    try:
        pkg = importlib.import_module(package)
    except Exception:
        return False
    try:
        pkg_version = Version(pkg.__version__)
    except Exception:
        return True
    if use_base_version:
        pkg_version = Version(pkg_version.base_version)
    return op(pkg_version, Version(version))
