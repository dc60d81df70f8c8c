"""Minimal stand-in for ``lightning_utilities`` so the read-only reference package can be
imported as a *test oracle* (parity checks only; never used by the framework itself)."""
from lightning_utilities.core.apply_func import apply_to_collection  # noqa: F401
