"""BERTScore module (API parity: reference ``text/bert.py``).

States are the tokenised ``input_ids`` / ``attention_mask`` (``cat``), so DDP gathers token ids (small) and the
embedding model runs once at ``compute`` on each rank's device; scoring uses the MFMA greedy-matching kernel."""
from typing import Any, Callable, Dict, List, Optional, Sequence, Union

import torch
from torch import Tensor
from torch.nn import Module

from torchmetrics_forked_amd.functional.text.bert import _DEFAULT_MODEL, bert_score
from torchmetrics_forked_amd.functional.text.helper_embedding_metric import _TRANSFORMERS_AVAILABLE, _preprocess_text
from torchmetrics_forked_amd.metric import Metric
from torchmetrics_forked_amd.utilities import rank_zero_warn
from torchmetrics_forked_amd.utilities.data import dim_zero_cat
from torchmetrics_forked_amd.utilities.plot import _AX_TYPE, _PLOT_OUT_TYPE


class BERTScore(Metric):
    """BERTScore precision / recall / F1 per sentence pair."""

    is_differentiable: bool = False
    higher_is_better: bool = True
    full_state_update: bool = False
    plot_lower_bound: float = 0.0
    plot_upper_bound: float = 1.0
    preds_input_ids: List[Tensor]
    preds_attention_mask: List[Tensor]
    target_input_ids: List[Tensor]
    target_attention_mask: List[Tensor]

    def __init__(
        self,
        model_name_or_path: Optional[str] = None,
        num_layers: Optional[int] = None,
        all_layers: bool = False,
        model: Optional[Module] = None,
        user_tokenizer: Optional[Any] = None,
        user_forward_fn: Optional[Callable[[Module, Dict[str, Tensor]], Tensor]] = None,
        verbose: bool = False,
        idf: bool = False,
        device: Optional[Union[str, torch.device]] = None,
        max_length: int = 512,
        batch_size: int = 64,
        num_threads: int = 0,
        return_hash: bool = False,
        lang: str = "en",
        rescale_with_baseline: bool = False,
        baseline_path: Optional[str] = None,
        baseline_url: Optional[str] = None,
        **kwargs: Any,
    ) -> None:
        super().__init__(**kwargs)
        self.model_name_or_path = model_name_or_path or _DEFAULT_MODEL
        self.num_layers = num_layers
        self.all_layers = all_layers
        self.model = model
        self.user_forward_fn = user_forward_fn
        self.verbose = verbose
        self.idf = idf
        self.embedding_device = device
        self.max_length = max_length
        self.batch_size = batch_size
        self.num_threads = num_threads
        self.return_hash = return_hash
        self.lang = lang
        self.rescale_with_baseline = rescale_with_baseline
        self.baseline_path = baseline_path
        self.baseline_url = baseline_url
        if user_tokenizer:
            self.tokenizer = user_tokenizer
            self.user_tokenizer = True
        else:
            if not _TRANSFORMERS_AVAILABLE:
                raise ModuleNotFoundError("`BERTScore` metric with default tokenizers requires `transformers` package be installed.")
            if model_name_or_path is None:
                rank_zero_warn(
                    "The argument `model_name_or_path` was not specified while it is required when the default"
                    f" `transformers` model is used. It will use the default recommended model - {_DEFAULT_MODEL!r}."
                )
            from transformers import AutoTokenizer

            self.tokenizer = AutoTokenizer.from_pretrained(self.model_name_or_path)
            self.user_tokenizer = False
        self.add_state("preds_input_ids", [], dist_reduce_fx="cat")
        self.add_state("preds_attention_mask", [], dist_reduce_fx="cat")
        self.add_state("target_input_ids", [], dist_reduce_fx="cat")
        self.add_state("target_attention_mask", [], dist_reduce_fx="cat")

    def update(self, preds: Union[str, Sequence[str]], target: Union[str, Sequence[str]]) -> None:
        preds = [preds] if isinstance(preds, str) else list(preds)
        target = [target] if isinstance(target, str) else list(target)
        own = self.user_tokenizer and not hasattr(self.tokenizer, "pad_token")
        p, _ = _preprocess_text(preds, self.tokenizer, self.max_length, truncation=False, sort_according_length=False, own_tokenizer=own)
        t, _ = _preprocess_text(target, self.tokenizer, self.max_length, truncation=False, sort_according_length=False, own_tokenizer=own)
        self.preds_input_ids.append(p["input_ids"].to(self.device))
        self.preds_attention_mask.append(p["attention_mask"].to(self.device))
        self.target_input_ids.append(t["input_ids"].to(self.device))
        self.target_attention_mask.append(t["attention_mask"].to(self.device))

    # ------------------------------------------------------------------------------------- sharded compute
    # ``sharded_compute=True`` under DDP (and ``idf=False``: IDF weights need the whole target corpus): the token
    # states are not gathered; every rank embeds and scores only its own sentence pairs and the per-pair
    # precision / recall / F1 are all-gathered afterwards (rank-major, the order of the replicated ``cat`` gather).
    # The reference gathers every pair to every rank and runs the full model forward on all of them
    # (``text/bert.py:229-260``): W x the embedding work for W ranks.
    _bert_sharded: Optional[Any] = None

    def _sync_dist(self, dist_sync_fn: Any = None, process_group: Optional[Any] = None) -> None:
        from torchmetrics_forked_amd.utilities.distributed import gather_all_tensors

        if self.sharded_compute and not self.idf and (dist_sync_fn is None or dist_sync_fn is gather_all_tensors):
            self._bert_sharded = [process_group or self.process_group]
            return
        super()._sync_dist(dist_sync_fn, process_group)

    def unsync(self, should_unsync: bool = True) -> None:
        super().unsync(should_unsync)
        if should_unsync:
            self._bert_sharded = None

    def _gather_scores(self, out: Dict[str, Any]) -> Dict[str, Any]:
        from torchmetrics_forked_amd.utilities.distributed import gather_all_tensors

        group = self._bert_sharded[0]
        res = dict(out)
        for key in ("precision", "recall", "f1"):
            val = out[key]
            t = val if isinstance(val, Tensor) else torch.tensor(val, dtype=torch.float32)
            comm = t.to(self.device).reshape(-1)
            parts = gather_all_tensors(comm, group)
            merged = torch.cat([p.to(t.device) for p in parts])
            res[key] = merged if isinstance(val, Tensor) else merged.tolist()
        return res

    def compute(self) -> Dict[str, Union[Tensor, List[float], str]]:
        if self._bert_sharded is not None and not self.preds_input_ids:
            empty = torch.zeros(0, dtype=torch.float32, device=self.device)
            local: Dict[str, Any] = {"precision": empty, "recall": empty, "f1": empty}
            return self._gather_scores(local)
        preds = {"input_ids": dim_zero_cat(self.preds_input_ids), "attention_mask": dim_zero_cat(self.preds_attention_mask)}
        target = {"input_ids": dim_zero_cat(self.target_input_ids), "attention_mask": dim_zero_cat(self.target_attention_mask)}
        out = bert_score(
            preds=preds, target=target, model_name_or_path=self.model_name_or_path, num_layers=self.num_layers,
            all_layers=self.all_layers, model=self.model, user_tokenizer=self.tokenizer if self.user_tokenizer else None,
            user_forward_fn=self.user_forward_fn, verbose=self.verbose, idf=self.idf, device=self.embedding_device,
            max_length=self.max_length, batch_size=self.batch_size, num_threads=self.num_threads, return_hash=self.return_hash,
            lang=self.lang, rescale_with_baseline=self.rescale_with_baseline, baseline_path=self.baseline_path,
            baseline_url=self.baseline_url,
        )
        return self._gather_scores(out) if self._bert_sharded is not None else out

    def plot(self, val: Optional[Union[Tensor, Sequence[Tensor]]] = None, ax: Optional[_AX_TYPE] = None) -> _PLOT_OUT_TYPE:
        if val is None:
            val = self.compute()
        val = val.get("f1", val) if isinstance(val, dict) else val
        return self._plot(val, ax)
