"""gfx950 detection kernels (tiled box-overlap matrices, bit-packed mask IoU) vs fp64 PyTorch references, and
MeanAveragePrecision / IoU modules with GPU-resident states vs the same metric on CPU."""
import pytest
import torch

from torchmetrics_forked_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


def _boxes(n, g):
    xy = torch.rand(n, 2, generator=g) * 500
    return torch.cat([xy, xy + torch.rand(n, 2, generator=g) * 200 + 0.5], 1)


@pytest.mark.parametrize("mode", ["iou", "giou", "diou", "ciou"])
@pytest.mark.parametrize("nm", [(1, 1), (17, 70), (300, 257), (2000, 1500), (0, 5)])
def test_box_pairwise_kernel(mode, nm):
    from torchmetrics_forked_amd.functional.detection._box_ops import _eager, pairwise_box_overlap

    g = torch.Generator().manual_seed(nm[0] * 7 + nm[1])
    a, b = _boxes(nm[0], g), _boxes(nm[1], g)
    got = pairwise_box_overlap(a.cuda(), b.cuda(), mode)
    ref = _eager(a.double(), b.double(), mode)
    assert got.shape == ref.shape and got.dtype == torch.float32
    torch.testing.assert_close(got.cpu().double(), ref, atol=2e-5, rtol=0)


@pytest.mark.parametrize("shape", [(5, 7, 33, 29), (40, 12, 480, 640), (1, 1, 8, 8), (64, 3, 100, 100)])
def test_mask_iou_kernel(shape):
    from torchmetrics_forked_amd.detection._mask_utils import mask_iou

    d_n, g_n, h, w = shape
    g = torch.Generator().manual_seed(h * w)
    det = torch.rand(d_n, h, w, generator=g) < 0.3
    gt = torch.rand(g_n, h, w, generator=g) < 0.3
    crowd = torch.rand(g_n, generator=g) < 0.3
    got = mask_iou(det.cuda(), gt.cuda(), crowd.cuda())
    ref = mask_iou(det, gt, crowd)
    torch.testing.assert_close(got.cpu(), ref, atol=1e-12, rtol=0)


def _batch(g, n_img):
    preds, target = [], []
    for _ in range(n_img):
        ng = int(torch.randint(1, 8, (1,), generator=g))
        gt = _boxes(ng, g)
        lab = torch.randint(0, 5, (ng,), generator=g)
        det = torch.cat([gt + torch.randn(ng, 4, generator=g) * 10, _boxes(3, g)])
        det[:, 2:] = torch.maximum(det[:, 2:], det[:, :2] + 1)
        preds.append({"boxes": det, "scores": torch.rand(ng + 3, generator=g),
                      "labels": torch.cat([lab, torch.randint(0, 5, (3,), generator=g)])})
        target.append({"boxes": gt, "labels": lab})
    return preds, target


def _to(batch, dev):
    return [[{k: v.to(dev) for k, v in d.items()} for d in lst] for lst in batch]


def test_map_gpu_states_match_cpu():
    from torchmetrics_forked_amd.detection import MeanAveragePrecision

    g = torch.Generator().manual_seed(0)
    batches = [_batch(g, 8) for _ in range(3)]
    gpu = MeanAveragePrecision(class_metrics=True).cuda()
    cpu = MeanAveragePrecision(class_metrics=True)
    for b in batches:
        gpu.update(*_to(b, "cuda"))
        cpu.update(*b)
    a, c = gpu.compute(), cpu.compute()
    for k in c:
        torch.testing.assert_close(a[k].cpu(), c[k], atol=1e-6, rtol=0, msg=k)


def test_map_segm_gpu_matches_cpu():
    from torchmetrics_forked_amd.detection import MeanAveragePrecision

    g = torch.Generator().manual_seed(1)
    preds, target = [], []
    for _ in range(4):
        gm = torch.rand(3, 64, 48, generator=g) < 0.4
        dm = gm ^ (torch.rand(3, 64, 48, generator=g) < 0.1)
        target.append({"masks": gm, "labels": torch.tensor([0, 1, 1])})
        preds.append({"masks": dm, "scores": torch.rand(3, generator=g), "labels": torch.tensor([0, 1, 0])})
    gpu = MeanAveragePrecision(iou_type="segm").cuda()
    gpu.update(*_to((preds, target), "cuda"))
    cpu = MeanAveragePrecision(iou_type="segm")
    cpu.update(preds, target)
    a, c = gpu.compute(), cpu.compute()
    for k in c:
        torch.testing.assert_close(a[k].cpu(), c[k], atol=1e-6, rtol=0, msg=k)


def _box_masks(k, h, w, g):
    """Rectangle masks (realistic run counts) plus the corner cases of the encoder: all / none / first pixel."""
    x0 = torch.randint(0, w, (k, 1, 1), generator=g)
    y0 = torch.randint(0, h, (k, 1, 1), generator=g)
    x1 = x0 + torch.randint(1, max(w, 2), (k, 1, 1), generator=g)
    y1 = y0 + torch.randint(1, max(h, 2), (k, 1, 1), generator=g)
    yy = torch.arange(h).view(1, h, 1)
    xx = torch.arange(w).view(1, 1, w)
    m = (yy >= y0) & (yy < y1) & (xx >= x0) & (xx < x1)
    if k > 3:
        m[0] = True
        m[1] = False
        m[2] = torch.rand(h, w, generator=g) > 0.5
        m[3, 0, 0] = True
    return m


@pytest.mark.parametrize("h,w", [(1, 1), (37, 23), (64, 64), (100, 190), (257, 129)])
def test_rle_encode_decode_gpu_matches_cpu(h, w):
    """csrc/rle.hip encode (change words, positions, COCO strings) and decode bits are byte-identical to the CPU ops."""
    g = torch.Generator().manual_seed(h * 7 + w)
    m = _box_masks(9, h, w, g)
    cg, og = torch.ops.tmx.rle_encode(m.cuda())
    cc, oc = torch.ops.tmx.rle_encode(m)
    assert torch.equal(og, oc) and torch.equal(cg, cc)
    bg, ag = torch.ops.tmx.rle_decode_bits(cc.cuda(), oc.cuda(), h, w)
    bc, ac = torch.ops.tmx.rle_decode_bits(cc, oc, h, w)
    assert torch.equal(bg.cpu(), bc) and torch.equal(ag.cpu(), ac)


def test_mask_iou_tiles_gpu_matches_cpu_and_dense():
    from torchmetrics_forked_amd.detection._mask_utils import encode_mask_batch, mask_iou, rle_segm_ious

    g = torch.Generator().manual_seed(3)
    imgs = [(_box_masks(int(torch.randint(0, 40, (1,), generator=g)), 96, 80, g),
             _box_masks(int(torch.randint(0, 30, (1,), generator=g)), 96, 80, g)) for _ in range(12)]
    crowd = [torch.randint(0, 2, (gm.shape[0],), generator=g) for _, gm in imgs]
    det = encode_mask_batch([d.cuda() for d, _ in imgs])
    gt = encode_mask_batch([gm.cuda() for _, gm in imgs])
    assert det == encode_mask_batch([d for d, _ in imgs])
    on_gpu = rle_segm_ious(det, gt, crowd, torch.device("cuda"))
    on_cpu = rle_segm_ious(det, gt, crowd, torch.device("cpu"))
    for a, b in zip(on_gpu, on_cpu):
        assert torch.equal(a.cpu(), b)
    pos = 0
    for i, (d, gm) in enumerate(imgs):
        if d.shape[0] and gm.shape[0]:
            ref = mask_iou(d, gm, crowd[i]).reshape(-1)
            assert torch.equal(on_cpu[0][pos:pos + ref.numel()], ref)
            pos += ref.numel()


def test_map_segm_rle_device_path_equals_host_evaluator():
    """Segm mAP with RLE states on the device (one decode + one IoU launch per mask size) equals the host evaluator."""
    from torchmetrics_forked_amd.detection import MeanAveragePrecision

    g = torch.Generator().manual_seed(11)
    preds, target = [], []
    for _ in range(24):
        ng = int(torch.randint(1, 8, (1,), generator=g))
        gm = _box_masks(ng, 128, 96, g)
        dm = torch.cat([gm, _box_masks(3, 128, 96, g)]) ^ (torch.rand(ng + 3, 128, 96, generator=g) > 0.97)
        target.append({"masks": gm, "labels": torch.randint(0, 3, (ng,), generator=g), "iscrowd": torch.randint(0, 2, (ng,), generator=g) * (torch.rand(ng, generator=g) > 0.8)})
        preds.append({"masks": dm, "scores": torch.rand(ng + 3, generator=g), "labels": torch.randint(0, 3, (ng + 3,), generator=g)})
    gpu = MeanAveragePrecision(iou_type="segm", class_metrics=True).cuda()
    gpu.update(*_to((preds, target), "cuda"))
    cpu = MeanAveragePrecision(iou_type="segm", class_metrics=True)
    cpu.update(preds, target)
    assert gpu.detection_mask == cpu.detection_mask
    a, c = gpu.compute(), cpu.compute()
    for k in c:
        assert torch.equal(a[k].cpu(), c[k]), k


def _coco_inputs(seed, n_img, n_cls, max_det_img, max_gt_img, tie_scores):
    """Flat COCO evaluator inputs with crowds, zero/huge areas, score ties and >100 detections in some pairs."""
    g = torch.Generator().manual_seed(seed)
    d_img, g_img, d_box, g_box = [], [], [], []
    for i in range(n_img):
        ng = int(torch.randint(0, max_gt_img + 1, (1,), generator=g))
        nd = int(torch.randint(0, max_det_img + 1, (1,), generator=g))
        gb = _boxes(ng, g) if ng else torch.zeros(0, 4)
        src = gb[torch.randint(0, max(ng, 1), (nd,), generator=g)] if ng else _boxes(nd, g)
        db = src + torch.randn(nd, 4, generator=g) * 8
        db[:, 2:] = torch.maximum(db[:, 2:], db[:, :2] + 1)
        g_box.append(gb); d_box.append(db)
        g_img += [i] * ng; d_img += [i] * nd
    xyxy2xywh = lambda b: torch.cat([b[:, :2], b[:, 2:] - b[:, :2]], 1).double()
    det_boxes, gt_boxes = xyxy2xywh(torch.cat(d_box)), xyxy2xywh(torch.cat(g_box))
    nd, ng = det_boxes.shape[0], gt_boxes.shape[0]
    scores = torch.rand(nd, generator=g).double()
    if tie_scores:
        scores = (scores * 8).floor() / 8
    det_labels = torch.randint(0, n_cls, (nd,), generator=g) * 3 + 1  # sparse category ids
    gt_labels = torch.randint(0, n_cls, (ng,), generator=g) * 3 + 1
    gt_crowd = (torch.rand(ng, generator=g) < 0.1).long()
    gt_area = torch.where(torch.rand(ng, generator=g) < 0.3, torch.zeros(ng).double(), gt_boxes[:, 2] * gt_boxes[:, 3] * 1.3)
    gt_area = torch.where(gt_area > 0, gt_area, gt_boxes[:, 2] * gt_boxes[:, 3])
    det_area = det_boxes[:, 2] * det_boxes[:, 3]
    return dict(det_boxes=det_boxes, det_scores=scores, det_labels=det_labels, det_img=torch.tensor(d_img, dtype=torch.long),
                det_area=det_area, gt_boxes=gt_boxes, gt_labels=gt_labels, gt_img=torch.tensor(g_img, dtype=torch.long),
                gt_crowd=gt_crowd, gt_area=gt_area)


@pytest.mark.parametrize("cfg", [
    dict(seed=0, n_img=40, n_cls=6, max_det_img=30, max_gt_img=12, tie_scores=False, max_dets=[1, 10, 100]),
    dict(seed=1, n_img=25, n_cls=3, max_det_img=260, max_gt_img=70, tie_scores=True, max_dets=[1, 10, 100]),
    dict(seed=2, n_img=60, n_cls=10, max_det_img=15, max_gt_img=6, tie_scores=True, max_dets=[2, 5, 300]),
    dict(seed=3, n_img=7, n_cls=2, max_det_img=0, max_gt_img=5, tie_scores=False, max_dets=[1, 10, 100]),
    dict(seed=4, n_img=9, n_cls=2, max_det_img=12, max_gt_img=0, tie_scores=False, max_dets=[1, 10, 100]),
])
@pytest.mark.parametrize("score_dtype", [torch.float64, torch.float32])
def test_coco_evaluate_gpu_matches_host(cfg, score_dtype):
    """Device matcher + accumulator (csrc/coco_match.hip) against the host evaluator (coco_eval.cpp): precision,
    recall, score tables and exported IoUs are bit-identical (same double arithmetic).  fp32 scores take the
    composite-key radix orderings, fp64 the two stable sorts."""
    from torchmetrics_forked_amd.detection.mean_ap import _AREA_RANGES

    x = _coco_inputs(cfg["seed"], cfg["n_img"], cfg["n_cls"], cfg["max_det_img"], cfg["max_gt_img"], cfg["tie_scores"])
    x["det_scores"] = x["det_scores"].to(score_dtype)
    if score_dtype == torch.float32 and x["det_scores"].numel() > 3:
        x["det_scores"][:3] = torch.tensor([0.0, -0.0, 0.5])  # signed zeros tie
    cats = torch.cat([x["det_labels"], x["gt_labels"]]).unique()
    iou_thr = torch.linspace(0.5, 0.95, 10, dtype=torch.float64)
    rec_thr = torch.linspace(0.0, 1.0, 101, dtype=torch.float64)
    max_dets = torch.tensor(cfg["max_dets"], dtype=torch.long)
    area = torch.tensor(_AREA_RANGES, dtype=torch.float64)
    host = torch.ops.tmx.coco_evaluate(
        x["det_boxes"], x["det_scores"], x["det_labels"], x["det_img"], x["det_area"], x["gt_boxes"], x["gt_labels"],
        x["gt_img"], x["gt_crowd"], x["gt_area"], cats, cfg["n_img"], iou_thr, rec_thr, max_dets, area, None, None)
    c = lambda t: t.cuda()
    dev = torch.ops.tmx.coco_evaluate_gpu(
        c(x["det_boxes"]), c(x["det_scores"]), c(torch.searchsorted(cats, x["det_labels"])), c(x["det_img"]),
        c(x["det_area"]), c(x["gt_boxes"]), c(torch.searchsorted(cats, x["gt_labels"])), c(x["gt_img"]),
        c(x["gt_crowd"]), c(x["gt_area"]), cats.numel(), cfg["n_img"], c(iou_thr), c(rec_thr), max_dets, c(area),
        None, None, None, None, None, True)
    for name, h, d in zip(("precision", "recall", "scores"), host[:3], dev[:3]):
        assert torch.equal(h, d.cpu()), (name, (h - d.cpu()).abs().max())
    # exported IoU blocks: device lists non-empty pairs only
    hv, hi = host[3], host[4]
    dv, di = dev[3].cpu(), dev[4].cpu()
    hmap = {(int(r[0]), int(r[1])): hv[r[4]: r[4] + r[2] * r[3]] for r in hi if r[2] and r[3]}
    dmap = {(int(r[0]), int(r[1])): dv[r[4]: r[4] + r[2] * r[3]] for r in di if r[2] and r[3]}
    assert hmap.keys() == dmap.keys()
    for key in hmap:
        assert torch.equal(hmap[key], dmap[key]), key


@pytest.mark.parametrize("cfg", [
    dict(seed=0, n_img=40, n_cls=6, max_det_img=30, max_gt_img=12, tie_scores=False, max_dets=[1, 10, 100]),
    dict(seed=1, n_img=25, n_cls=3, max_det_img=260, max_gt_img=70, tie_scores=True, max_dets=[1, 10, 100]),
    dict(seed=2, n_img=60, n_cls=10, max_det_img=15, max_gt_img=6, tie_scores=True, max_dets=[2, 5, 300]),
    dict(seed=3, n_img=7, n_cls=2, max_det_img=0, max_gt_img=5, tie_scores=False, max_dets=[1, 10, 100]),
    dict(seed=4, n_img=9, n_cls=2, max_det_img=12, max_gt_img=0, tie_scores=False, max_dets=[1, 10, 100]),
    dict(seed=5, n_img=6, n_cls=4, max_det_img=256, max_gt_img=256, tie_scores=True, max_dets=[1, 10, 100]),
])
@pytest.mark.parametrize("score_dtype", [torch.float32, torch.bfloat16])
def test_coco_evaluate_gpu_img_matches_host(cfg, score_dtype):
    """Per-image route (one workgroup per image ranks, orders and matches its rows; csrc/coco_match.hip
    coco_image_match_kernel) against the host evaluator: precision, recall and score tables bit-identical."""
    from torchmetrics_forked_amd.detection.mean_ap import _AREA_RANGES

    x = _coco_inputs(cfg["seed"], cfg["n_img"], cfg["n_cls"], cfg["max_det_img"], cfg["max_gt_img"], cfg["tie_scores"])
    x["det_scores"] = x["det_scores"].to(score_dtype)
    if x["det_scores"].numel() > 3:
        x["det_scores"][:3] = torch.tensor([0.0, -0.0, 0.5], dtype=score_dtype)  # signed zeros tie
    cats = torch.cat([x["det_labels"], x["gt_labels"]]).unique()
    iou_thr = torch.linspace(0.5, 0.95, 10, dtype=torch.float64)
    rec_thr = torch.linspace(0.0, 1.0, 101, dtype=torch.float64)
    max_dets = torch.tensor(cfg["max_dets"], dtype=torch.long)
    area = torch.tensor(_AREA_RANGES, dtype=torch.float64)
    host = torch.ops.tmx.coco_evaluate(
        x["det_boxes"], x["det_scores"].double(), x["det_labels"], x["det_img"], x["det_area"], x["gt_boxes"],
        x["gt_labels"], x["gt_img"], x["gt_crowd"], x["gt_area"], cats, cfg["n_img"], iou_thr, rec_thr, max_dets, area,
        None, None)
    offs = lambda img: torch.cat([torch.zeros(1, dtype=torch.long),
                                  torch.bincount(img, minlength=cfg["n_img"]).cumsum(0)])
    c = lambda t: t.cuda()
    # (the op derives detection areas from the boxes, as _coco_inputs does; ground-truth areas are all > 0 here)
    dev = torch.ops.tmx.coco_evaluate_gpu_img(
        c(x["det_boxes"]), c(x["det_scores"]), c(torch.searchsorted(cats, x["det_labels"])), c(offs(x["det_img"])),
        c(x["gt_boxes"]), c(torch.searchsorted(cats, x["gt_labels"])), c(x["gt_crowd"]), c(x["gt_area"]),
        c(offs(x["gt_img"])), cats.numel(), c(iou_thr), c(rec_thr), max_dets, c(max_dets) if cfg["seed"] % 2 else None,
        c(area))
    if cfg["max_det_img"] > 256:  # past the per-image LDS tables: flagged (the module then takes another route)
        assert int(dev[3]) == 1 or x["det_img"].bincount().max() <= 256
        return
    assert int(dev[3]) == 0
    for name, h, d in zip(("precision", "recall", "scores"), host[:3], dev[:3]):
        assert torch.equal(h, d.cpu()), (name, (h - d.cpu()).abs().max())


def test_map_module_img_route_equals_grid_route(monkeypatch):
    """Module level, bbox, no extended summary: the per-image route and the (image, class)-grid route give identical
    results (macro with class metrics, and micro)."""
    import torchmetrics_forked_amd.detection.mean_ap as mod
    from torchmetrics_forked_amd.detection import MeanAveragePrecision

    g = torch.Generator().manual_seed(11)
    preds, target = [], []
    for _ in range(30):
        ng = int(torch.randint(0, 25, (1,), generator=g))
        gt = _boxes(ng, g) if ng else torch.zeros(0, 4)
        nd = int(torch.randint(0, 140, (1,), generator=g))
        det = (gt[torch.randint(0, ng, (nd,), generator=g)] if ng else _boxes(nd, g)) + torch.randn(nd, 4, generator=g) * 9
        det[:, 2:] = torch.maximum(det[:, 2:], det[:, :2] + 1)
        preds.append({"boxes": det, "scores": (torch.rand(nd, generator=g) * 32).floor() / 32,
                      "labels": torch.randint(0, 7, (nd,), generator=g)})
        target.append({"boxes": gt, "labels": torch.randint(0, 7, (ng,), generator=g),
                       "iscrowd": (torch.rand(ng, generator=g) < 0.1).long()})
    batch = _to((preds, target), "cuda")
    for avg in ("macro", "micro"):
        out = []
        for route in (True, False):
            monkeypatch.setattr(mod, "_IMG_ROUTE", route)
            m = MeanAveragePrecision(class_metrics=True, average=avg).cuda()
            m.warn_on_many_detections = False
            m.update(*batch)
            out.append(m.compute())
        for k in out[1]:
            torch.testing.assert_close(out[0][k].cpu(), out[1][k].cpu(), atol=0, rtol=0, msg=k)


def test_map_module_gpu_many_dets_crowds_matches_cpu():
    """Module level: crowd ground truth, supplied areas, > max_det detections, extended summary and micro average."""
    from torchmetrics_forked_amd.detection import MeanAveragePrecision

    g = torch.Generator().manual_seed(5)
    preds, target = [], []
    for _ in range(12):
        ng = int(torch.randint(1, 30, (1,), generator=g))
        gt = _boxes(ng, g)
        lab = torch.randint(0, 4, (ng,), generator=g)
        nd = int(torch.randint(50, 160, (1,), generator=g))
        det = gt[torch.randint(0, ng, (nd,), generator=g)] + torch.randn(nd, 4, generator=g) * 12
        det[:, 2:] = torch.maximum(det[:, 2:], det[:, :2] + 1)
        preds.append({"boxes": det, "scores": (torch.rand(nd, generator=g) * 16).floor() / 16,
                      "labels": torch.randint(0, 4, (nd,), generator=g)})
        target.append({"boxes": gt, "labels": lab, "iscrowd": (torch.rand(ng, generator=g) < 0.15).long(),
                       "area": torch.rand(ng, generator=g) * 20000})
    for avg in ("macro", "micro"):
        kw = dict(class_metrics=True, extended_summary=True, average=avg)
        gpu, cpu = MeanAveragePrecision(**kw).cuda(), MeanAveragePrecision(**kw)
        gpu.warn_on_many_detections = cpu.warn_on_many_detections = False
        gpu.update(*_to((preds, target), "cuda"))
        cpu.update(preds, target)
        a, c = gpu.compute(), cpu.compute()
        for k in c:
            if k == "ious":
                assert a[k].keys() == c[k].keys()
                for key in c[k]:
                    va, vc = a[k][key], c[k][key]
                    assert (isinstance(va, list) and isinstance(vc, list)) or torch.equal(va.cpu(), vc), key
            else:
                torch.testing.assert_close(a[k].cpu(), c[k], atol=0, rtol=0, msg=k)


@pytest.mark.parametrize("cls_name", ["IntersectionOverUnion", "GeneralizedIntersectionOverUnion",
                                      "DistanceIntersectionOverUnion", "CompleteIntersectionOverUnion"])
def test_iou_modules_gpu(cls_name):
    import torchmetrics_forked_amd.detection as D

    g = torch.Generator().manual_seed(2)
    preds, target = _batch(g, 6)
    preds = [{k: v for k, v in d.items() if k != "scores"} for d in preds]
    gpu = getattr(D, cls_name)(class_metrics=True).cuda()
    gpu.update(*_to((preds, target), "cuda"))
    cpu = getattr(D, cls_name)(class_metrics=True)
    cpu.update(preds, target)
    a, c = gpu.compute(), cpu.compute()
    for k in c:
        torch.testing.assert_close(a[k].cpu(), c[k], atol=2e-5, rtol=0, msg=k)


@pytest.mark.parametrize("modified", [False, True])
def test_panoptic_quality_gpu_matches_cpu(modified):
    from torchmetrics_forked_amd.functional.detection import modified_panoptic_quality, panoptic_quality

    g = torch.Generator().manual_seed(3)
    cats = torch.tensor([0, 1, 6, 7])
    def rand():
        c = cats[torch.randint(0, 4, (4, 32, 32), generator=g)].repeat_interleave(4, 1).repeat_interleave(4, 2)
        i = torch.randint(0, 3, (4, 32, 32), generator=g).repeat_interleave(4, 1).repeat_interleave(4, 2)
        return torch.stack([c, i], -1)
    p, t = rand(), rand()
    fn = modified_panoptic_quality if modified else panoptic_quality
    a = fn(p.cuda(), t.cuda(), things={0, 1}, stuffs={6, 7})
    b = fn(p, t, things={0, 1}, stuffs={6, 7})
    torch.testing.assert_close(a.cpu(), b, atol=1e-12, rtol=0)


@pytest.mark.parametrize("big_ids", [False, True])
def test_panoptic_segment_keys_kernel_paths(big_ids):
    """csrc/panoptic.hip packed keys (and the row-unique fallback when an instance id needs more than 32 bits) give
    the CPU result, with unknown prediction categories mapped to void."""
    from torchmetrics_forked_amd.detection import PanopticQuality

    g = torch.Generator().manual_seed(5)
    cats = torch.tensor([0, 1, 6, 7, 9])  # 9: unknown
    def rand():
        c = cats[torch.randint(0, 5, (3, 40, 24), generator=g)]
        i = torch.randint(0, 5, (3, 40, 24), generator=g)
        if big_ids:
            i = i + (1 << 33)
        return torch.stack([c, i], -1)
    mg = PanopticQuality(things={0, 1}, stuffs={6, 7}, allow_unknown_preds_category=True).cuda()
    mc = PanopticQuality(things={0, 1}, stuffs={6, 7}, allow_unknown_preds_category=True)
    for _ in range(2):
        p, t = rand(), rand()
        t[t[..., 0] == 9] = torch.tensor([0, 1])
        mg.update(p.cuda(), t.cuda())
        mc.update(p, t)
    torch.testing.assert_close(mg.compute().cpu(), mc.compute(), atol=1e-12, rtol=0)
    keys = torch.ops.tmx.panoptic_segment_keys(p.reshape(3, -1, 2).cuda(), t.reshape(3, -1, 2).cuda(), torch.tensor([0, 1, 6, 7]).cuda(), torch.tensor([0, 1, 2, 3, 4]).cuda())
    assert int(keys[2].item()) == int(big_ids)


def test_upload_i64_pinned_staging():
    """tmx::upload_i64: host int64 -> device through the reused pinned buffer, back-to-back calls of growing size (the
    buffer is reused only after the previous copy completed)."""
    like = torch.zeros(1, device="cuda")
    outs = []
    for n in (0, 5, 1000, 70000, 3):
        h = torch.arange(n, dtype=torch.long) * 7 - 3
        d = torch.ops.tmx.upload_i64(h, like)
        outs.append((h, d))
    for h, d in outs:
        assert d.is_cuda and d.dtype == torch.long and torch.equal(d.cpu(), h)


@pytest.mark.parametrize("labels", [[], [0], [3, 3, 1, 65535, 7, 1], list(range(0, 65536, 97)), [5, -1], [70000, 2]])
def test_class_presence_bitmap_and_ids(labels):
    """tmx::class_presence: the bitmap's set bits and the compacted device ids are torch.unique of the labels; a
    label outside [0, 65536) sets the flag word."""
    import numpy as np

    lab = torch.tensor(labels, dtype=torch.long, device="cuda")
    bm, ids = torch.ops.tmx.class_presence(lab)
    words = bm.numpy().view(np.uint32)
    inside = sorted({v for v in labels if 0 <= v < 65536})
    assert bool(words[-1]) == any(not 0 <= v < 65536 for v in labels)
    got = [32 * w + b for w in np.flatnonzero(words[:-1]) for b in range(32) if (int(words[w]) >> b) & 1]
    assert got == inside
    assert ids[: len(inside)].cpu().tolist() == inside


def test_coco_summary_tables_kernel_matches_composition():
    """tmx::coco_summary_tables (one kernel + one pinned copy) against the ATen composition of
    MeanAveragePrecision._summary_tables on the same tables (CPU path), including the overflow word."""
    import numpy as np

    from torchmetrics_forked_amd.detection import MeanAveragePrecision

    g = torch.Generator().manual_seed(4)
    T, R, K, A, M = 10, 101, 7, 4, 3
    prec = torch.rand(T, R, K, A, M, generator=g, dtype=torch.float64)
    prec[torch.rand(T, R, K, A, M, generator=g) < 0.3] = -1.0
    rec = torch.rand(T, K, A, M, generator=g, dtype=torch.float64)
    rec[torch.rand(T, K, A, M, generator=g) < 0.3] = -1.0
    m = MeanAveragePrecision()
    ref = m._summary_tables(prec, rec)
    got = m._summary_tables(prec.cuda(), rec.cuda(), torch.zeros(1, dtype=torch.long, device="cuda"))
    np.testing.assert_allclose(got, ref, rtol=1e-15, atol=0)
    assert m._summary_tables(prec.cuda(), rec.cuda(), torch.ones(1, dtype=torch.long, device="cuda")) is None
