"""Framework exception / warning types (parity: reference ``utilities/exceptions.py:16-21``)."""


class TorchMetricsUserError(Exception):
    """Raised on misuse of the metric runtime (double sync, forward while synced, ...)."""


class TorchMetricsUserWarning(Warning):
    """Warning category for user-facing runtime advisories."""
