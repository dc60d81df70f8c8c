"""BERTScore (API parity: reference ``functional/text/bert.py``; Zhang et al., 2020).

MI355X path: embeddings stay on the model's device (the reference copies every batch to the CPU), the greedy
matching runs in the MFMA kernel ``tmx::bert_greedy_match`` (row / column maxima of P·Rᵀ without materialising the
[B, Lp, Lr] similarity tensor), and the IDF-weighted reductions are batched tensor ops.  CPU inputs use a chunked
``bmm`` + ``max`` with the same semantics.

Documented deviation: every prediction is scored against *its own* reference and results come back in input
order.  (The reference sorts predictions and references by length independently and pairs them by sorted
position, so sentences are mismatched whenever the two length orders differ.)
"""
import csv
import urllib.request
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor
from torch.nn import Module

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.functional.text.helper_embedding_metric import (
    _TQDM_AVAILABLE,
    _TRANSFORMERS_AVAILABLE,
    _check_shape_of_model_output,
    _get_progress_bar,
    _idf_table,
    _lookup_idf,
    _preprocess_text,
    _process_attention_mask_for_special_tokens,
)
from torchmetrics_forked_amd.utilities import rank_zero_warn

_DEFAULT_MODEL = "roberta-large"


def _model_device(model: Module, device: Optional[Union[str, torch.device]]) -> torch.device:
    if device is not None:
        return torch.device(device)
    try:
        return next(model.parameters()).device
    except StopIteration:
        return torch.device("cpu")


def _embed(
    input_ids: Tensor,
    attention_mask: Tensor,
    model: Module,
    device: torch.device,
    batch_size: int,
    num_layers: Optional[int],
    all_layers: bool,
    verbose: bool,
    user_forward_fn: Optional[Callable[[Module, Dict[str, Tensor]], Tensor]],
) -> Tuple[Tensor, Tensor]:
    """Normalised, special-token-masked embeddings ``[N, layers, L, D]`` (input order) and the processed mask."""
    n, length = input_ids.shape
    order = attention_mask.sum(1).argsort()
    chunks: List[Tensor] = []
    for s in _get_progress_bar(range(0, n, batch_size), verbose):
        idx = order[s : s + batch_size]
        ids, mask = input_ids[idx], attention_mask[idx]
        max_len = int(mask.sum(1).max().item())
        batch = {"input_ids": ids[:, :max_len].to(device), "attention_mask": mask[:, :max_len].to(device)}
        with torch.no_grad():
            if not all_layers:
                if user_forward_fn is None:
                    out = model(batch["input_ids"], batch["attention_mask"], output_hidden_states=True)
                    out = out.hidden_states[num_layers if num_layers is not None else -1]
                else:
                    out = user_forward_fn(model, batch)
                    _check_shape_of_model_output(out, batch["input_ids"])
                out = out.unsqueeze(1)
            else:
                if user_forward_fn is not None:
                    raise ValueError("The option `all_layers=True` can be used only with default `transformers` models.")
                out = model(batch["input_ids"], batch["attention_mask"], output_hidden_states=True)
                out = torch.stack(out.hidden_states, dim=1)
        out = out / out.norm(dim=-1, keepdim=True)
        if max_len < length:
            out = torch.nn.functional.pad(out, (0, 0, 0, length - max_len))
        chunks.append(out)
    emb = torch.cat(chunks)
    inv = torch.empty_like(order)
    inv[order] = torch.arange(n, device=order.device)
    emb = emb[inv.to(emb.device)]
    mask = _process_attention_mask_for_special_tokens(attention_mask.clone().to(emb.device))
    emb = emb * mask[:, None, :, None].to(emb.dtype)
    return emb, mask


def _greedy_max(p: Tensor, r: Tensor) -> Tuple[Tensor, Tensor]:
    """Row maxima ``[B, Lp]`` and column maxima ``[B, Lr]`` of ``p @ rᵀ`` per pair."""
    if p.is_cuda and ops.use_native(p):
        return torch.ops.tmx.bert_greedy_match(p.contiguous(), r.contiguous())
    rows, cols = [], []
    step = max(1, int(2**26 // max(1, p.shape[1] * r.shape[1])))
    for s in range(0, p.shape[0], step):
        sim = torch.bmm(p[s : s + step], r[s : s + step].transpose(1, 2))
        rows.append(sim.max(dim=2).values)
        cols.append(sim.max(dim=1).values)
    return torch.cat(rows).float(), torch.cat(cols).float()


def _scores(
    p_emb: Tensor, r_emb: Tensor, p_scale: Tensor, r_scale: Tensor
) -> Tuple[Tensor, Tensor, Tensor]:
    """p_emb / r_emb ``[N, layers, L, D]``; scales ``[N, L]`` -> precision / recall / f1 ``[layers, N]``."""
    n, layers = p_emb.shape[:2]
    pf = p_emb.transpose(0, 1).reshape(n * layers, p_emb.shape[2], p_emb.shape[3])
    rf = r_emb.transpose(0, 1).reshape(n * layers, r_emb.shape[2], r_emb.shape[3])
    rowmax, colmax = _greedy_max(pf, rf)
    rowmax = rowmax.reshape(layers, n, -1)
    colmax = colmax.reshape(layers, n, -1)
    precision = (rowmax * p_scale[None].to(rowmax)).sum(-1)
    recall = (colmax * r_scale[None].to(colmax)).sum(-1)
    f1 = 2 * precision * recall / (precision + recall)
    f1 = f1.masked_fill(torch.isnan(f1), 0.0)
    return precision, recall, f1


def _get_hash(model_name_or_path: Optional[str] = None, num_layers: Optional[int] = None, idf: bool = False) -> str:
    return f"{model_name_or_path}_L{num_layers}{'_idf' if idf else '_no-idf'}"


def _read_csv_from_local_file(baseline_path: str) -> Tensor:
    with open(baseline_path) as f:
        rows = [[float(x) for x in row] for i, row in enumerate(csv.reader(f)) if i > 0]
    return torch.tensor(rows)[:, 1:]


def _read_csv_from_url(baseline_url: str) -> Tensor:
    with urllib.request.urlopen(baseline_url) as req:  # noqa: S310
        rows = [[float(x) for x in row.strip().decode("utf-8").split(",")] for i, row in enumerate(req) if i > 0]
    return torch.tensor(rows)[:, 1:]


def _load_baseline(
    lang: str = "en", model_name_or_path: Optional[str] = None, baseline_path: Optional[str] = None, baseline_url: Optional[str] = None
) -> Optional[Tensor]:
    if baseline_path:
        return _read_csv_from_local_file(baseline_path)
    if baseline_url:
        return _read_csv_from_url(baseline_url)
    if lang and model_name_or_path:
        url = f"https://raw.githubusercontent.com/Tiiiger/bert_score/master/bert_score/rescale_baseline/{lang}/{model_name_or_path}.tsv"
        return _read_csv_from_url(url)
    rank_zero_warn("Baseline was not successfully loaded. No baseline is going to be used.")
    return None


def _rescale_metrics_with_baseline(
    precision: Tensor, recall: Tensor, f1_score: Tensor, baseline: Tensor, num_layers: Optional[int] = None, all_layers: bool = False
) -> Tuple[Tensor, Tensor, Tensor]:
    if num_layers is None and all_layers is False:
        num_layers = -1
    allm = torch.stack([precision, recall, f1_score], dim=-1)
    scale = baseline.unsqueeze(1) if all_layers else baseline[num_layers]
    allm = (allm - scale.to(allm)) / (1 - scale.to(allm))
    return allm[..., 0], allm[..., 1], allm[..., 2]


def _tokenize(text: Any, tokenizer: Any, max_length: int, own: bool) -> Dict[str, Tensor]:
    if isinstance(text, dict):
        return {"input_ids": text["input_ids"], "attention_mask": text["attention_mask"]}
    out, _ = _preprocess_text(list(text), tokenizer, max_length, truncation=True, sort_according_length=False, own_tokenizer=own)
    return out


def bert_score(
    preds: Union[str, Sequence[str], Dict[str, Tensor]],
    target: Union[str, Sequence[str], Dict[str, Tensor]],
    model_name_or_path: Optional[str] = None,
    num_layers: Optional[int] = None,
    all_layers: bool = False,
    model: Optional[Module] = None,
    user_tokenizer: Any = None,
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
) -> Dict[str, Union[Tensor, List[float], str]]:
    """Token-matching BERTScore precision / recall / F1 per sentence pair."""
    if len(preds) != len(target):
        raise ValueError("Number of predicted and reference sententes must be the same!")
    if isinstance(preds, str):
        preds = [preds]
    if isinstance(target, str):
        target = [target]
    if not isinstance(preds, (list, dict)):
        preds = list(preds)
    if not isinstance(target, (list, dict)):
        target = list(target)
    if verbose and not _TQDM_AVAILABLE:
        raise ModuleNotFoundError("An argument `verbose = True` requires `tqdm` package be installed.")
    if model is None:
        if not _TRANSFORMERS_AVAILABLE:
            raise ModuleNotFoundError("`bert_score` metric with default models requires `transformers` package be installed.")
        from transformers import AutoModel, AutoTokenizer

        if model_name_or_path is None:
            rank_zero_warn(
                "The argument `model_name_or_path` was not specified while it is required when default"
                f" `transformers` model are used. It is, therefore, used the default recommended model - {_DEFAULT_MODEL}."
            )
        tokenizer = AutoTokenizer.from_pretrained(model_name_or_path or _DEFAULT_MODEL)
        model = AutoModel.from_pretrained(model_name_or_path or _DEFAULT_MODEL)
        own = False
    else:
        tokenizer = user_tokenizer
        own = user_tokenizer is not None and not hasattr(user_tokenizer, "pad_token")
    model.eval()
    if device is not None:
        model.to(device)
    dev = _model_device(model, device)
    try:
        if num_layers and num_layers > model.config.num_hidden_layers:
            raise ValueError(
                f"num_layers={num_layers} is forbidden for {model_name_or_path}."
                f" Please use num_layers <= {model.config.num_hidden_layers}"
            )
    except AttributeError:
        rank_zero_warn("It was not possible to retrieve the parameter `num_layers` from the model specification.")

    empty = all(isinstance(t, list) and len(t) == 0 for t in (preds, target))
    if empty:
        rank_zero_warn("Predictions and references are empty.")
        out: Dict[str, Union[Tensor, List[float], str]] = {"precision": [0.0], "recall": [0.0], "f1": [0.0]}
        if return_hash:
            out["hash"] = _get_hash(model_name_or_path, num_layers, idf)
        return out
    valid_lists = all(isinstance(t, list) and len(t) > 0 and isinstance(t[0], str) for t in (preds, target))
    valid_tensors = all(isinstance(t, dict) and isinstance(t["input_ids"], Tensor) for t in (preds, target))
    if not (valid_lists or valid_tensors):
        raise ValueError("Invalid input provided.")
    if valid_lists and tokenizer is None:
        raise ValueError("A tokenizer is required to score raw sentences with a user-provided model.")

    baseline = _load_baseline(lang, model_name_or_path, baseline_path, baseline_url) if rescale_with_baseline else None
    t_tok = _tokenize(target, tokenizer, max_length, own)
    p_tok = _tokenize(preds, tokenizer, max_length, own)
    if valid_tensors:  # trim to the longest attended sequence, like the reference's TokenizedDataset
        for tok in (t_tok, p_tok):
            ml = int(tok["attention_mask"].sum(1).max().item())
            tok["input_ids"], tok["attention_mask"] = tok["input_ids"][:, :ml], tok["attention_mask"][:, :ml]

    r_emb, r_mask = _embed(t_tok["input_ids"], t_tok["attention_mask"], model, dev, batch_size, num_layers, all_layers, verbose, user_forward_fn)
    p_emb, p_mask = _embed(p_tok["input_ids"], p_tok["attention_mask"], model, dev, batch_size, num_layers, all_layers, verbose, user_forward_fn)
    if idf:
        table, default = _idf_table(t_tok["input_ids"].to(dev), len(t_tok["input_ids"]))
        r_w = _lookup_idf(t_tok["input_ids"], table, default).to(r_emb.device) * r_mask
        p_w = _lookup_idf(p_tok["input_ids"], table, default).to(p_emb.device) * p_mask
    else:
        r_w, p_w = r_mask.to(r_emb.dtype), p_mask.to(p_emb.dtype)
    r_scale = r_w / r_w.sum(-1, keepdim=True)
    p_scale = p_w / p_w.sum(-1, keepdim=True)
    precision, recall, f1 = _scores(p_emb, r_emb, p_scale.float(), r_scale.float())
    if not all_layers:
        precision, recall, f1 = precision[0], recall[0], f1[0]
    if baseline is not None:
        precision, recall, f1 = _rescale_metrics_with_baseline(precision, recall, f1, baseline, num_layers, all_layers)
    output: Dict[str, Union[Tensor, List[float], str]] = {"precision": precision, "recall": recall, "f1": f1}
    if return_hash:
        output["hash"] = _get_hash(model_name_or_path, num_layers, idf)
    return output
