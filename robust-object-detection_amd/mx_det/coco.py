"""COCO index + COCOeval (bbox) restatement — the metric behind the reference's mAP numbers.

pycocotools (unpinned, README.md:229) is not installed in this image or on the GPU box; the
reference calls it at train_frcnn_baseline.py:92-96 (COCO(ann).loadRes -> COCOeval(bbox).evaluate /
accumulate / summarize, stats[0] = mAP@[.5:.95], stats[1] = mAP@.5) and eval_all.py:131-156
(per-class AP50 = mean(precision[0, :, k, 0, 2] > -1)). This module restates pycocotools' published
algorithm (cocoeval.py evaluate/evaluateImg/accumulate/summarize, maskApi bbIou in double precision)
with the same parameters: iouThrs linspace(.5,.95,10), recThrs linspace(0,1,101), maxDets
(1,10,100), area ranges all/small/medium/large, crowd gts as ignore regions. It is host code
(a few hundred detections per image); when pycocotools is importable the scripts use it instead.
"""
import copy
import json
from collections import defaultdict

import numpy as np


class COCO:
    def __init__(self, annotation_file=None):
        self.dataset, self.anns, self.cats, self.imgs = {}, {}, {}, {}
        self.imgToAnns, self.catToImgs = defaultdict(list), defaultdict(list)
        if annotation_file is not None:
            d = annotation_file if isinstance(annotation_file, dict) else json.load(open(annotation_file))
            self.dataset = d
            self.createIndex()

    def createIndex(self):
        self.anns, self.cats, self.imgs = {}, {}, {}
        self.imgToAnns, self.catToImgs = defaultdict(list), defaultdict(list)
        for ann in self.dataset.get("annotations", []):
            self.imgToAnns[ann["image_id"]].append(ann)
            self.anns[ann["id"]] = ann
        for img in self.dataset.get("images", []):
            self.imgs[img["id"]] = img
        for cat in self.dataset.get("categories", []):
            self.cats[cat["id"]] = cat
        for ann in self.dataset.get("annotations", []):
            self.catToImgs[ann["category_id"]].append(ann["image_id"])

    def getAnnIds(self, imgIds=(), catIds=(), areaRng=(), iscrowd=None):
        imgIds = imgIds if isinstance(imgIds, (list, tuple)) else [imgIds]
        catIds = catIds if isinstance(catIds, (list, tuple)) else [catIds]
        if len(imgIds) == 0:
            anns = self.dataset.get("annotations", [])
        else:
            anns = [a for i in imgIds if i in self.imgToAnns for a in self.imgToAnns[i]]
        if len(catIds):
            anns = [a for a in anns if a["category_id"] in catIds]
        if len(areaRng):
            anns = [a for a in anns if areaRng[0] < a["area"] < areaRng[1]]
        if iscrowd is not None:
            return [a["id"] for a in anns if a["iscrowd"] == iscrowd]
        return [a["id"] for a in anns]

    def getCatIds(self, catNms=(), supNms=(), catIds=()):
        cats = self.dataset.get("categories", [])
        if catNms:
            cats = [c for c in cats if c["name"] in catNms]
        if catIds:
            cats = [c for c in cats if c["id"] in catIds]
        return [c["id"] for c in cats]

    def getImgIds(self, imgIds=(), catIds=()):
        ids = set(imgIds) if imgIds else set(self.imgs.keys())
        for c in catIds:
            ids &= set(self.catToImgs[c])
        return list(ids)

    def loadAnns(self, ids=()):
        ids = ids if isinstance(ids, (list, tuple)) else [ids]
        return [self.anns[i] for i in ids]

    def loadCats(self, ids=()):
        ids = ids if isinstance(ids, (list, tuple)) else [ids]
        return [self.cats[i] for i in ids]

    def loadImgs(self, ids=()):
        ids = ids if isinstance(ids, (list, tuple)) else [ids]
        return [self.imgs[i] for i in ids]

    def loadRes(self, resFile):
        """bbox results list -> result COCO (pycocotools loadRes, bbox branch)."""
        res = COCO()
        res.dataset["images"] = [img for img in self.dataset["images"]]
        anns = json.load(open(resFile)) if isinstance(resFile, str) else resFile
        assert isinstance(anns, list), "results is not an array of objects"
        annsImgIds = [a["image_id"] for a in anns]
        assert set(annsImgIds) == (set(annsImgIds) & set(self.getImgIds())), \
            "Results do not correspond to current coco set"
        res.dataset["categories"] = copy.deepcopy(self.dataset["categories"])
        for i, ann in enumerate(anns):
            ann = dict(ann)
            bb = ann["bbox"]
            x1, x2, y1, y2 = [bb[0], bb[0] + bb[2], bb[1], bb[1] + bb[3]]
            if "segmentation" not in ann:
                ann["segmentation"] = [[x1, y1, x1, y2, x2, y2, x2, y1]]
            ann["area"] = bb[2] * bb[3]
            ann["id"] = i + 1
            ann["iscrowd"] = 0
            anns[i] = ann
        res.dataset["annotations"] = anns
        res.createIndex()
        return res


def bbox_iou(d, g, iscrowd):
    """maskApi bbIou: xywh boxes, double precision; crowd gt -> union = dt area."""
    d = np.asarray(d, dtype=np.float64).reshape(-1, 4)
    g = np.asarray(g, dtype=np.float64).reshape(-1, 4)
    if len(d) == 0 or len(g) == 0:
        return []
    crowd = np.asarray(iscrowd, dtype=bool)
    dx2, dy2 = d[:, 0] + d[:, 2], d[:, 1] + d[:, 3]
    gx2, gy2 = g[:, 0] + g[:, 2], g[:, 1] + g[:, 3]
    w = np.minimum(dx2[:, None], gx2[None]) - np.maximum(d[:, 0][:, None], g[:, 0][None])
    h = np.minimum(dy2[:, None], gy2[None]) - np.maximum(d[:, 1][:, None], g[:, 1][None])
    inter = np.where((w > 0) & (h > 0), w * h, 0.0)
    da = (d[:, 2] * d[:, 3])[:, None]
    ga = (g[:, 2] * g[:, 3])[None]
    union = np.where(crowd[None], da, da + ga - inter)
    return inter / union


class Params:
    def __init__(self):
        self.imgIds, self.catIds = [], []
        self.iouThrs = np.linspace(.5, 0.95, int(np.round((0.95 - .5) / .05)) + 1, endpoint=True)
        self.recThrs = np.linspace(.0, 1.00, int(np.round((1.00 - .0) / .01)) + 1, endpoint=True)
        self.maxDets = [1, 10, 100]
        self.areaRng = [[0 ** 2, 1e5 ** 2], [0 ** 2, 32 ** 2], [32 ** 2, 96 ** 2], [96 ** 2, 1e5 ** 2]]
        self.areaRngLbl = ["all", "small", "medium", "large"]
        self.useCats = 1
        self.iouType = "bbox"


class COCOeval:
    def __init__(self, cocoGt=None, cocoDt=None, iouType="bbox"):
        assert iouType == "bbox", "only bbox evaluation is restated"
        self.cocoGt, self.cocoDt = cocoGt, cocoDt
        self.params = Params()
        self.evalImgs, self.eval, self.stats, self.ious = [], {}, [], {}
        if cocoGt is not None:
            self.params.imgIds = sorted(cocoGt.getImgIds())
            self.params.catIds = sorted(cocoGt.getCatIds())

    def _prepare(self):
        p = self.params
        gts = self.cocoGt.loadAnns(self.cocoGt.getAnnIds(imgIds=p.imgIds, catIds=p.catIds))
        dts = self.cocoDt.loadAnns(self.cocoDt.getAnnIds(imgIds=p.imgIds, catIds=p.catIds))
        for gt in gts:
            gt["ignore"] = gt.get("ignore", 0)
            gt["ignore"] = "iscrowd" in gt and gt["iscrowd"]
        self._gts, self._dts = defaultdict(list), defaultdict(list)
        for gt in gts:
            self._gts[gt["image_id"], gt["category_id"]].append(gt)
        for dt in dts:
            self._dts[dt["image_id"], dt["category_id"]].append(dt)

    def computeIoU(self, imgId, catId):
        gt, dt = self._gts[imgId, catId], self._dts[imgId, catId]
        if len(gt) == 0 and len(dt) == 0:
            return []
        inds = np.argsort([-d["score"] for d in dt], kind="mergesort")
        dt = [dt[i] for i in inds][: self.params.maxDets[-1]]
        return bbox_iou([d["bbox"] for d in dt], [g["bbox"] for g in gt], [int(o["iscrowd"]) for o in gt])

    def evaluateImg(self, imgId, catId, aRng, maxDet):
        p = self.params
        gt, dt = self._gts[imgId, catId], self._dts[imgId, catId]
        if len(gt) == 0 and len(dt) == 0:
            return None
        for g in gt:
            g["_ignore"] = 1 if (g["ignore"] or g["area"] < aRng[0] or g["area"] > aRng[1]) else 0
        gtind = np.argsort([g["_ignore"] for g in gt], kind="mergesort")
        gt = [gt[i] for i in gtind]
        dtind = np.argsort([-d["score"] for d in dt], kind="mergesort")
        dt = [dt[i] for i in dtind[0:maxDet]]
        iscrowd = [int(o["iscrowd"]) for o in gt]
        ious = self.ious[imgId, catId]
        ious = ious[:, gtind] if len(ious) > 0 else ious
        T, G, D = len(p.iouThrs), len(gt), len(dt)
        gtm, dtm = np.zeros((T, G)), np.zeros((T, D))
        gtIg = np.array([g["_ignore"] for g in gt])
        dtIg = np.zeros((T, D))
        if len(ious) != 0:
            for tind, t in enumerate(p.iouThrs):
                for dind, d in enumerate(dt):
                    iou = min([t, 1 - 1e-10])
                    m = -1
                    for gind, g in enumerate(gt):
                        if gtm[tind, gind] > 0 and not iscrowd[gind]:
                            continue
                        if m > -1 and gtIg[m] == 0 and gtIg[gind] == 1:
                            break
                        if ious[dind, gind] < iou:
                            continue
                        iou = ious[dind, gind]
                        m = gind
                    if m == -1:
                        continue
                    dtIg[tind, dind] = gtIg[m]
                    dtm[tind, dind] = gt[m]["id"]
                    gtm[tind, m] = d["id"]
        a = np.array([d["area"] < aRng[0] or d["area"] > aRng[1] for d in dt]).reshape((1, len(dt)))
        dtIg = np.logical_or(dtIg, np.logical_and(dtm == 0, np.repeat(a, T, 0)))
        return {"image_id": imgId, "category_id": catId, "aRng": aRng, "maxDet": maxDet,
                "dtIds": [d["id"] for d in dt], "gtIds": [g["id"] for g in gt], "dtMatches": dtm, "gtMatches": gtm,
                "dtScores": [d["score"] for d in dt], "gtIgnore": gtIg, "dtIgnore": dtIg}

    def evaluate(self):
        p = self.params
        p.imgIds = list(np.unique(p.imgIds))
        p.catIds = list(np.unique(p.catIds))
        p.maxDets = sorted(p.maxDets)
        self._prepare()
        self.ious = {(i, c): self.computeIoU(i, c) for i in p.imgIds for c in p.catIds}
        md = p.maxDets[-1]
        self.evalImgs = [self.evaluateImg(i, c, a, md) for c in p.catIds for a in p.areaRng for i in p.imgIds]

    def accumulate(self):
        p = self.params
        T, R, K, A, M = len(p.iouThrs), len(p.recThrs), len(p.catIds), len(p.areaRng), len(p.maxDets)
        precision = -np.ones((T, R, K, A, M))
        recall = -np.ones((T, K, A, M))
        scores = -np.ones((T, R, K, A, M))
        I0, A0 = len(p.imgIds), len(p.areaRng)
        for k in range(K):
            Nk = k * A0 * I0
            for a in range(A):
                Na = a * I0
                for m, maxDet in enumerate(p.maxDets):
                    E = [self.evalImgs[Nk + Na + i] for i in range(I0)]
                    E = [e for e in E if e is not None]
                    if len(E) == 0:
                        continue
                    dtScores = np.concatenate([e["dtScores"][0:maxDet] for e in E])
                    inds = np.argsort(-dtScores, kind="mergesort")
                    dtScoresSorted = dtScores[inds]
                    dtm = np.concatenate([e["dtMatches"][:, 0:maxDet] for e in E], axis=1)[:, inds]
                    dtIg = np.concatenate([e["dtIgnore"][:, 0:maxDet] for e in E], axis=1)[:, inds]
                    gtIg = np.concatenate([e["gtIgnore"] for e in E])
                    npig = np.count_nonzero(gtIg == 0)
                    if npig == 0:
                        continue
                    tps = np.logical_and(dtm, np.logical_not(dtIg))
                    fps = np.logical_and(np.logical_not(dtm), np.logical_not(dtIg))
                    tp_sum = np.cumsum(tps, axis=1).astype(dtype=float)
                    fp_sum = np.cumsum(fps, axis=1).astype(dtype=float)
                    for t, (tp, fp) in enumerate(zip(tp_sum, fp_sum)):
                        nd = len(tp)
                        rc = tp / npig
                        pr = tp / (fp + tp + np.spacing(1))
                        q, ss = np.zeros((R,)), np.zeros((R,))
                        recall[t, k, a, m] = rc[-1] if nd else 0
                        pr = pr.tolist()
                        q = q.tolist()
                        for i in range(nd - 1, 0, -1):
                            if pr[i] > pr[i - 1]:
                                pr[i - 1] = pr[i]
                        idx = np.searchsorted(rc, p.recThrs, side="left")
                        try:
                            for ri, pi in enumerate(idx):
                                q[ri] = pr[pi]
                                ss[ri] = dtScoresSorted[pi]
                        except IndexError:
                            pass
                        precision[t, :, k, a, m] = np.array(q)
                        scores[t, :, k, a, m] = np.array(ss)
        self.eval = {"params": p, "counts": [T, R, K, A, M], "precision": precision, "recall": recall,
                     "scores": scores}

    def _summarize(self, ap=1, iouThr=None, areaRng="all", maxDets=100):
        p = self.params
        aind = [i for i, a in enumerate(p.areaRngLbl) if a == areaRng]
        mind = [i for i, m in enumerate(p.maxDets) if m == maxDets]
        if ap == 1:
            s = self.eval["precision"]
            if iouThr is not None:
                s = s[np.where(iouThr == p.iouThrs)[0]]
            s = s[:, :, :, aind, mind]
        else:
            s = self.eval["recall"]
            if iouThr is not None:
                s = s[np.where(iouThr == p.iouThrs)[0]]
            s = s[:, :, aind, mind]
        mean_s = -1 if len(s[s > -1]) == 0 else np.mean(s[s > -1])
        name = "Average Precision" if ap == 1 else "Average Recall"
        thr = f"{p.iouThrs[0]:0.2f}:{p.iouThrs[-1]:0.2f}" if iouThr is None else f"{iouThr:0.2f}"
        print(f" {name:<18} @[ IoU={thr:<9} | area={areaRng:>6s} | maxDets={maxDets:>3d} ] = {mean_s:0.3f}")
        return mean_s

    def summarize(self):
        md = self.params.maxDets[2]
        st = np.zeros((12,))
        st[0] = self._summarize(1)
        st[1] = self._summarize(1, iouThr=.5, maxDets=md)
        st[2] = self._summarize(1, iouThr=.75, maxDets=md)
        st[3] = self._summarize(1, areaRng="small", maxDets=md)
        st[4] = self._summarize(1, areaRng="medium", maxDets=md)
        st[5] = self._summarize(1, areaRng="large", maxDets=md)
        st[6] = self._summarize(0, maxDets=self.params.maxDets[0])
        st[7] = self._summarize(0, maxDets=self.params.maxDets[1])
        st[8] = self._summarize(0, maxDets=md)
        st[9] = self._summarize(0, areaRng="small", maxDets=md)
        st[10] = self._summarize(0, areaRng="medium", maxDets=md)
        st[11] = self._summarize(0, areaRng="large", maxDets=md)
        self.stats = st


def get_coco_api():
    """(COCO, COCOeval): pycocotools when importable, else this restatement."""
    try:
        from pycocotools.coco import COCO as PC
        from pycocotools.cocoeval import COCOeval as PE
        return PC, PE
    except ImportError:
        return COCO, COCOeval
