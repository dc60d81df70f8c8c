"""CLIPScore / CLIP-IQA vs the reference with a tiny random-init CLIP saved to a local directory (no downloads)."""
import json

import pytest
import torch

transformers = pytest.importorskip("transformers")


@pytest.fixture(scope="module")
def tiny_clip(tmp_path_factory):
    d = tmp_path_factory.mktemp("tinyclip")
    # GPT-2 byte -> unicode table (printable bytes map to themselves, the rest to 256+i)
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("\xa1"), ord("\xac") + 1)) + list(range(ord("\xae"), ord("\xff") + 1))
    cs = bs[:]
    k = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + k)
            k += 1
    chars = [chr(c) for c in cs]
    vocab = {c: i for i, c in enumerate(chars)}
    for c in chars:
        vocab[c + "</w>"] = len(vocab)
    vocab["<|startoftext|>"] = len(vocab)
    vocab["<|endoftext|>"] = len(vocab)
    (d / "vocab.json").write_text(json.dumps(vocab))
    (d / "merges.txt").write_text("#version: 0.2\n")
    tok = transformers.CLIPTokenizer(str(d / "vocab.json"), str(d / "merges.txt"))
    imgp = transformers.CLIPImageProcessor(size={"shortest_edge": 32}, crop_size={"height": 32, "width": 32})
    proc = transformers.CLIPProcessor(image_processor=imgp, tokenizer=tok)
    cfg = transformers.CLIPConfig(
        text_config={"vocab_size": len(vocab), "hidden_size": 32, "intermediate_size": 64, "num_hidden_layers": 2,
                     "num_attention_heads": 2, "max_position_embeddings": 64},
        vision_config={"hidden_size": 32, "intermediate_size": 64, "num_hidden_layers": 2, "num_attention_heads": 2,
                       "image_size": 32, "patch_size": 8},
        projection_dim=16,
    )
    torch.manual_seed(0)
    transformers.CLIPModel(cfg).eval().save_pretrained(str(d))
    proc.save_pretrained(str(d))
    return str(d)


class _TensorCLIP(transformers.CLIPModel):
    """Test-only adapter: this transformers version returns output objects from ``get_*_features``; the reference
    expects tensors (our implementation accepts both)."""

    def get_image_features(self, *a, **k):
        out = super().get_image_features(*a, **k)
        return out if isinstance(out, torch.Tensor) else out.pooler_output

    def get_text_features(self, *a, **k):
        out = super().get_text_features(*a, **k)
        return out if isinstance(out, torch.Tensor) else out.pooler_output


@pytest.fixture(autouse=True)
def _ref_tensor_clip(reference, monkeypatch):
    import importlib

    for mod in ("torchmetrics.functional.multimodal.clip_score", "torchmetrics.functional.multimodal.clip_iqa"):
        m = importlib.import_module(mod)
        if hasattr(m, "_CLIPModel"):
            monkeypatch.setattr(m, "_CLIPModel", _TensorCLIP)


def _images(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 255, (n, 3, 40, 36), generator=g, dtype=torch.uint8)


def test_clip_score_vs_reference(reference, tiny_clip):
    from torchmetrics.functional.multimodal import clip_score as ref

    from torchmetrics_forked_amd.functional.multimodal import clip_score

    imgs = _images(3)
    text = ["a photo of a cat", "a dog", "something else entirely"]
    torch.testing.assert_close(clip_score(imgs, text, tiny_clip), ref(imgs, text, tiny_clip))


def test_clip_score_module(reference, tiny_clip):
    from torchmetrics.multimodal import CLIPScore as Ref

    from torchmetrics_forked_amd.multimodal import CLIPScore

    a, b = CLIPScore(tiny_clip), Ref(tiny_clip)
    for s in range(2):
        imgs = list(_images(2, s))
        a.update(imgs, ["red", "blue sky"])
        b.update(imgs, ["red", "blue sky"])
    torch.testing.assert_close(a.compute(), b.compute())
    with pytest.raises(ValueError, match="same"):
        a.update(list(_images(2)), ["only one"])


@pytest.mark.parametrize("prompts", [("quality",), ("quality", "brightness"), (("nice", "ugly"), "sharpness")])
def test_clip_iqa_vs_reference(reference, tiny_clip, prompts):
    from torchmetrics.functional.multimodal import clip_image_quality_assessment as ref

    from torchmetrics_forked_amd.functional.multimodal import clip_image_quality_assessment
    from torchmetrics_forked_amd.multimodal import CLIPImageQualityAssessment

    imgs = _images(4).float() / 255
    a = clip_image_quality_assessment(imgs, tiny_clip, prompts=prompts)
    b = ref(imgs, tiny_clip, prompts=prompts)
    if isinstance(a, dict):
        for k in b:
            torch.testing.assert_close(a[k], b[k])
    else:
        torch.testing.assert_close(a, b)
    m = CLIPImageQualityAssessment(tiny_clip, prompts=prompts)
    m.update(imgs[:2])
    m.update(imgs[2:])
    out = m.compute()
    if isinstance(out, dict):
        for k in b:
            torch.testing.assert_close(out[k], b[k])
    else:
        torch.testing.assert_close(out, b)


def test_clip_iqa_errors(tiny_clip):
    from torchmetrics_forked_amd.functional.multimodal.clip_iqa import _clip_iqa_format_prompts

    with pytest.raises(ValueError, match="must be a tuple"):
        _clip_iqa_format_prompts(["quality"])
    with pytest.raises(ValueError, match="must be one of"):
        _clip_iqa_format_prompts(("nope",))
    with pytest.raises(ValueError, match="length 2"):
        _clip_iqa_format_prompts((("a", "b", "c"),))
