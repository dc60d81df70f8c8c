"""Cross-rank machinery: the coalesced state-sync engine (RCCL over xGMI / gloo) and its failure detection."""
from torchmetrics_forked_amd.parallel.sync import (
    SyncTimeoutError,
    sync_states,
    sync_states_async,
    sync_states_many,
    sync_timeout,
)

__all__ = ["SyncTimeoutError", "sync_states", "sync_states_async", "sync_states_many", "sync_timeout"]
