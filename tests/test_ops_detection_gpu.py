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
