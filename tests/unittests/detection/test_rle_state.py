"""Segmentation mAP keeps the reference's RLE state format (``mean_ap.py:811-816``: per image a tuple of
``((H, W), counts bytes)``), encoded by ``tmx::rle_encode``; IoUs come from ``tmx::rle_decode_bits`` +
``tmx::mask_iou_tiles``.  CPU ops vs the pure-Python COCO encoder / dense mask IoU, the state_dict format, and a gloo
world-2 sync that must equal the single-process result."""
import numpy as np
import pytest
import torch

from tests.helpers.multirank import run_multirank
from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.detection import MeanAveragePrecision
from torchmetrics_forked_amd.detection._mask_utils import (
    _tiles,
    encode_mask_batch,
    mask_iou,
    rle_decode,
    rle_encode,
    rle_segm_ious,
)

pytestmark = pytest.mark.skipif(not ops.load(), reason="native library not built")


def _masks(k, h, w, seed):
    g = torch.Generator().manual_seed(seed)
    m = torch.rand(k, h, w, generator=g) > 0.55
    if k > 2:
        m[0] = True        # all foreground: counts [0, H W]
        m[1] = False       # all background: counts [H W]
        m[2, 0, 0] = True  # leading foreground pixel
    return m


@pytest.mark.parametrize("h,w", [(1, 1), (5, 3), (37, 23), (64, 64), (65, 130), (128, 70)])
def test_rle_encode_op_matches_python_encoder(h, w):
    m = _masks(6, h, w, seed=h * 131 + w)
    chars, off = torch.ops.tmx.rle_encode(m)
    buf = chars.numpy().tobytes()
    for k in range(m.shape[0]):
        assert buf[off[k]:off[k + 1]] == rle_encode(m[k])["counts"].encode("ascii")
    bits, area = torch.ops.tmx.rle_decode_bits(chars, off, h, w)
    for k in range(m.shape[0]):
        assert int(area[k]) == int(m[k].sum())
        flat = m[k].t().reshape(-1).numpy()
        words = bits[k].numpy().view(np.uint64)
        got = ((words[np.arange(flat.size) // 64] >> (np.arange(flat.size) % 64).astype(np.uint64)) & 1).astype(bool)
        assert np.array_equal(got, flat)
        assert np.array_equal(rle_decode({"size": [h, w], "counts": buf[off[k]:off[k + 1]]}), m[k].numpy().astype(np.uint8))


def test_state_format_and_checkpoint():
    preds = [{"masks": _masks(3, 20, 30, 1), "scores": torch.tensor([0.9, 0.5, 0.2]), "labels": torch.tensor([0, 1, 0])},
             {"masks": torch.zeros(0, 20, 30, dtype=torch.bool), "scores": torch.zeros(0), "labels": torch.zeros(0, dtype=torch.long)}]
    target = [{"masks": _masks(2, 20, 30, 2), "labels": torch.tensor([0, 1])},
              {"masks": _masks(1, 20, 30, 3), "labels": torch.tensor([1])}]
    m = MeanAveragePrecision(iou_type="segm")
    m.update(preds, target)
    assert m.detection_mask[1] == ()
    entry = m.detection_mask[0][0]
    assert isinstance(entry, tuple) and entry[0] == (20, 30) and isinstance(entry[1], bytes)
    assert entry[1] == rle_encode(preds[0]["masks"][0])["counts"].encode("ascii")
    m.persistent(True)
    sd = m.state_dict()
    assert sd["groundtruth_mask"] == list(m.groundtruth_mask)
    m2 = MeanAveragePrecision(iou_type="segm")
    m2.load_state_dict(sd)
    a, b = m.compute(), m2.compute()
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_rle_ious_match_dense_mask_iou():
    gen = torch.Generator().manual_seed(7)
    imgs = [(_masks(int(torch.randint(0, 20, (1,), generator=gen)), 33, 41, 10 + i),
             _masks(int(torch.randint(0, 19, (1,), generator=gen)), 33, 41, 50 + i)) for i in range(6)]
    crowd = [torch.randint(0, 2, (g.shape[0],), generator=gen) for _, g in imgs]
    det = encode_mask_batch([d for d, _ in imgs])
    gt = encode_mask_batch([g for _, g in imgs])
    ious, off, darea, garea = rle_segm_ious(det, gt, crowd, torch.device("cpu"), max_bits_bytes=2048)  # forces chunks
    pos = 0
    for i, (d, g) in enumerate(imgs):
        if d.shape[0] and g.shape[0]:
            ref = mask_iou(d, g, crowd[i]).reshape(-1)
            assert int(off[i]) == pos
            torch.testing.assert_close(ious[pos:pos + ref.numel()], ref, rtol=0, atol=0)
            pos += ref.numel()
    assert pos == ious.numel()
    torch.testing.assert_close(darea, torch.cat([d.flatten(1).sum(1) for d, _ in imgs]).double())
    torch.testing.assert_close(garea, torch.cat([g.flatten(1).sum(1) for _, g in imgs]).double())


def test_tiles_cover_every_block():
    t = _tiles([0, 17, 3, 40], [5, 2, 0, 33])
    covered = {(int(i), d, g) for i, d0, g0 in t for d in range(d0, d0 + 16) for g in range(g0, g0 + 16)}
    for i, (dn, gn) in enumerate(zip([0, 17, 3, 40], [5, 2, 0, 33])):
        for d in range(dn):
            for g in range(gn):
                assert (i, d, g) in covered


def _segm_batch(rank, n_img, seed):
    gen = torch.Generator().manual_seed(seed + rank)
    preds, target = [], []
    for _ in range(n_img):
        nd, ng = int(torch.randint(1, 5, (1,), generator=gen)), int(torch.randint(1, 4, (1,), generator=gen))
        base = torch.rand(ng, 24, 24, generator=gen) > 0.5
        det = torch.cat([base, torch.rand(max(0, nd - ng), 24, 24, generator=gen) > 0.5])[:nd]
        det = det ^ (torch.rand(det.shape, generator=gen) > 0.9)
        preds.append({"masks": det, "scores": torch.rand(nd, generator=gen), "labels": torch.randint(0, 2, (nd,), generator=gen)})
        target.append({"masks": base, "labels": torch.randint(0, 2, (ng,), generator=gen)})
    return preds, target


def check_segm_sync(rank, world, device):
    m = MeanAveragePrecision(iou_type="segm")
    p, t = _segm_batch(rank, 4, 100)
    m.update(p, t)
    out = m.compute()
    # single process over every rank's images in the synced (element-major, rank-interleaved) order
    ref = MeanAveragePrecision(iou_type="segm")
    per_rank = [_segm_batch(r, 4, 100) for r in range(world)]
    for e in range(4):
        for r in range(world):
            ref.update([per_rank[r][0][e]], [per_rank[r][1][e]])
    expect = ref.compute()
    for k in expect:
        assert torch.equal(out[k], expect[k]), k
    assert isinstance(m.detection_mask[0][0][1], bytes)  # unsync restored the local RLE tuples
    assert len(m.detection_mask) == 4


def test_segm_sync_gloo():
    run_multirank(check_segm_sync, 2, "gloo")
