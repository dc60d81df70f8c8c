"""Straight-line Python statement of the COCO evaluate / accumulate / summarize algorithm (per-image,
per-category greedy matching, envelope precision, recall-threshold sampling).  Used as an independent oracle
for the native evaluator; deliberately written loop-by-loop without any vectorisation."""
import numpy as np

AREA = [[0, 1e10], [0, 32**2], [32**2, 96**2], [96**2, 1e10]]


def _iou(d, g, crowd):
    out = np.zeros((len(d), len(g)))
    for i, a in enumerate(d):
        for j, b in enumerate(g):
            w = min(a[0] + a[2], b[0] + b[2]) - max(a[0], b[0])
            h = min(a[1] + a[3], b[1] + b[3]) - max(a[1], b[1])
            if w <= 0 or h <= 0:
                continue
            inter = w * h
            u = a[2] * a[3] if crowd[j] else a[2] * a[3] + b[2] * b[3] - inter
            out[i, j] = inter / u
    return out


def coco_eval(dets, gts, cats, n_img, iou_thrs, rec_thrs, max_dets, iou_fn=None):
    """dets: list of dicts(img, cat, box(xywh), score, area); gts: list of dicts(img, cat, box, crowd, area)."""
    T, R, K, A, M = len(iou_thrs), len(rec_thrs), len(cats), len(AREA), len(max_dets)
    evals = {}
    ious = {}
    for i in range(n_img):
        for k, c in enumerate(cats):
            d = [x for x in dets if x["img"] == i and x["cat"] == c]
            g = [x for x in gts if x["img"] == i and x["cat"] == c]
            order = sorted(range(len(d)), key=lambda j: -d[j]["score"])  # python sort is stable
            d = [d[j] for j in order][: max_dets[-1]]
            if iou_fn is None:
                ious[(i, k)] = _iou([x["box"] for x in d], [x["box"] for x in g], [x["crowd"] for x in g])
            else:
                ious[(i, k)] = iou_fn(d, g)
            for a, (lo, hi) in enumerate(AREA):
                if not d and not g:
                    evals[(k, a, i)] = None
                    continue
                gig = [1 if (x["crowd"] or x["area"] < lo or x["area"] > hi) else 0 for x in g]
                gorder = sorted(range(len(g)), key=lambda j: gig[j])
                gs = [g[j] for j in gorder]
                gig = [gig[j] for j in gorder]
                crowd = [x["crowd"] for x in gs]
                io = ious[(i, k)][:, gorder] if len(d) and len(g) else np.zeros((len(d), len(g)))
                gtm = np.zeros((T, len(g)))
                dtm = np.zeros((T, len(d)))
                dig = np.zeros((T, len(d)))
                for t, thr in enumerate(iou_thrs):
                    for di in range(len(d)):
                        best = min(thr, 1 - 1e-10)
                        m = -1
                        for gi in range(len(g)):
                            if gtm[t, gi] > 0 and not crowd[gi]:
                                continue
                            if m > -1 and gig[m] == 0 and gig[gi] == 1:
                                break
                            if io[di, gi] < best:
                                continue
                            best = io[di, gi]
                            m = gi
                        if m == -1:
                            continue
                        dig[t, di] = gig[m]
                        dtm[t, di] = 1
                        gtm[t, m] = 1
                for di, x in enumerate(d):
                    if x["area"] < lo or x["area"] > hi:
                        for t in range(T):
                            if dtm[t, di] == 0:
                                dig[t, di] = 1
                evals[(k, a, i)] = dict(scores=[x["score"] for x in d], dtm=dtm, dig=dig, gig=np.array(gig))
    precision = -np.ones((T, R, K, A, M))
    recall = -np.ones((T, K, A, M))
    for k in range(K):
        for a in range(A):
            for m, md in enumerate(max_dets):
                E = [evals[(k, a, i)] for i in range(n_img) if evals[(k, a, i)] is not None]
                if not E:
                    continue
                sc = np.concatenate([np.array(e["scores"][:md], dtype=np.float64) for e in E])
                inds = np.argsort(-sc, kind="mergesort")
                dtm = np.concatenate([e["dtm"][:, :md] for e in E], axis=1)[:, inds]
                dig = np.concatenate([e["dig"][:, :md] for e in E], axis=1)[:, inds]
                gig = np.concatenate([e["gig"] for e in E])
                npig = np.count_nonzero(gig == 0)
                if npig == 0:
                    continue
                tps = np.logical_and(dtm, np.logical_not(dig))
                fps = np.logical_and(np.logical_not(dtm), np.logical_not(dig))
                tp_sum = np.cumsum(tps, axis=1).astype(float)
                fp_sum = np.cumsum(fps, axis=1).astype(float)
                for t in range(T):
                    tp, fp = tp_sum[t], fp_sum[t]
                    nd = len(tp)
                    rc = tp / npig
                    pr = (tp / (fp + tp + np.spacing(1))).tolist()
                    recall[t, k, a, m] = rc[-1] if nd else 0
                    for j in range(nd - 1, 0, -1):
                        if pr[j] > pr[j - 1]:
                            pr[j - 1] = pr[j]
                    q = np.zeros(R)
                    idx = np.searchsorted(rc, rec_thrs, side="left")
                    for ri, pi in enumerate(idx):
                        if pi >= nd:
                            break
                        q[ri] = pr[pi]
                    precision[t, :, k, a, m] = q
    return precision, recall, ious


def summarize(precision, recall, iou_thrs, max_dets, first_max_det=100):
    def s(ap, thr=None, area=0, md=100):
        mind = [i for i, v in enumerate(max_dets) if v == md]
        x = precision[..., area, mind] if ap else recall[..., area, mind]
        if thr is not None:
            x = x[[i for i, v in enumerate(iou_thrs) if v == thr]]
        v = x[x > -1]
        return -1.0 if v.size == 0 else float(np.mean(v))

    m2 = max_dets[2]
    return [
        s(1, md=first_max_det), s(1, 0.5, md=m2), s(1, 0.75, md=m2), s(1, area=1, md=m2), s(1, area=2, md=m2),
        s(1, area=3, md=m2), s(0, md=max_dets[0]), s(0, md=max_dets[1]), s(0, md=m2), s(0, area=1, md=m2),
        s(0, area=2, md=m2), s(0, area=3, md=m2),
    ]
