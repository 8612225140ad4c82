"""Training / evaluation runners behind the drop-in scripts (scripts/train_frcnn_*.py, eval_*.py).

Behaviour follows the reference entry points:
  train: scripts/train_frcnn_baseline.py:110-223 / train_frcnn_augmented.py:120-216 — SGD(lr, momentum,
    weight_decay) over trainable params, StepLR(8, 0.1) per epoch, loss = sum(loss_dict.values()),
    epoch_loss += loss.item(); history.jsonl records {epoch, train_loss_sum, lr, mAP50, mAP50_95,
    elapsed_sec}; last.pth {"model", "epoch"} every epoch; final COCOeval on the val split; best.pth
    {"model", "epoch": "final", "metrics"}; a final history record with epoch "final".
  eval: scripts/eval_all.py:97-156 — bs=1 inference, xyxy -> xywh result dicts, COCOeval bbox,
    stats[0]/[1], per-class AP50 from precision[0, :, k, 0, 2].
MI355X-side differences: images stay uint8 until the device (ToImage/ToDtype scaling, corruption and
normalisation run as HIP kernels); with WORLD_SIZE > 1 (torchrun) every rank trains on its shard of
each epoch's permutation (DistributedSampler, drop_last: no padded duplicates in the loss sum) with
RCCL gradient all-reduce, and evaluation shards images by rank and gathers detections to rank 0.

Multi-GPU recipe: each rank keeps the reference's BATCH_SIZE (2) so every GPU's
BatchNorm sees the reference's bs-2 statistics; the global batch is 2 x world and an epoch has 1/world
as many optimizer steps. LR_SCALING (cfg key, or env MX_LR_SCALING) chooses the learning rate:
"none" (default) keeps the reference's 0.005 (its per-image gradient scale, StepLR(8) per epoch);
"linear" uses LR x world with a linear warm-up over WARMUP_ITERS (default 500) optimizer steps (the
large-batch rule). The choice changes mAP; neither is the reference's single-GPU run.
"""
import json
import os
import random
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import DataLoader, DistributedSampler

from . import frcnn
from .coco import get_coco_api


def set_seed(seed):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)


def dist_info():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def init_device():
    if not torch.cuda.is_available():
        raise RuntimeError("mx_det runs its hot path on MI355X (HIP); no GPU is visible")
    world, rank, local = dist_info()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("nccl", device_id=dev)
    return dev, world, rank


def build_frcnn(num_classes=7, weights=None, trainable_backbone_layers=None):
    """fasterrcnn_resnet50_fpn_v2(weights) + FastRCNNPredictor(in_features, num_classes)
    (train_frcnn_baseline.py:139-143). weights: None or a local state_dict / checkpoint path
    (stand-in for the reference's COCO "DEFAULT" download, unavailable offline)."""
    model = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None)
    in_features = model.roi_heads.box_predictor.cls_score.in_features
    if weights is not None:
        sd = weights if isinstance(weights, dict) else torch.load(weights, map_location="cpu", weights_only=True)
        sd = sd.get("model", sd)
        pred_shape = sd.get("roi_heads.box_predictor.cls_score.weight", torch.empty(0)).shape
        if len(pred_shape) and pred_shape[0] == num_classes:
            model.roi_heads.box_predictor = frcnn.FastRCNNPredictor(in_features, num_classes)
            model.load_state_dict(sd)
        else:  # COCO-pretrained body/FPN/RPN, fresh predictor (reference: head replaced after load)
            model.load_state_dict(sd)
            model.roi_heads.box_predictor = frcnn.FastRCNNPredictor(in_features, num_classes)
        trainable = 3 if trainable_backbone_layers is None else trainable_backbone_layers
    else:
        model.roi_heads.box_predictor = frcnn.FastRCNNPredictor(in_features, num_classes)
        trainable = 5 if trainable_backbone_layers is None else trainable_backbone_layers
    frcnn.set_trainable_layers(model.backbone.body, trainable)
    return model


class ShardSampler(torch.utils.data.Sampler):
    """Per-image eval sharding without padding (every image evaluated exactly once across ranks)."""

    def __init__(self, n, world, rank):
        self.idx = list(range(rank, n, world))

    def __iter__(self):
        return iter(self.idx)

    def __len__(self):
        return len(self.idx)


def _to_device_batch(images, targets, dev):
    imgs = [im.to(dev, non_blocking=True) for im in images]
    tgs = [{k: v.to(dev, non_blocking=True) for k, v in t.items()} for t in targets]
    return imgs, tgs


def _append_jsonl(path, rec):
    with open(path, "a", encoding="utf-8") as f:
        f.write(json.dumps(rec, ensure_ascii=False) + "\n")


@torch.no_grad()
def evaluate(model, loader, ann_file, dev, per_class=False):
    """COCOeval of a model over a loader of (uint8 HWC image, target) with bs=1."""
    world, rank, _ = dist_info()
    COCO, COCOeval = get_coco_api()
    model.eval()
    results = []
    for images, targets in loader:
        imgs = [im.to(dev, non_blocking=True) for im in images]
        outs = model(imgs)
        for out, tgt in zip(outs, targets):
            img_id = int(tgt["image_id"].item())
            b = out["boxes"].float().cpu().numpy()
            s = out["scores"].float().cpu().numpy()
            lab = out["labels"].cpu().numpy()
            for (x1, y1, x2, y2), sc, lb in zip(b.tolist(), s.tolist(), lab.tolist()):
                results.append({"image_id": img_id, "category_id": int(lb), "bbox": [x1, y1, x2 - x1, y2 - y1],
                                "score": float(sc)})
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, results)
        results = [r for part in gathered for r in part]
    if rank != 0:
        return None
    if not results:
        return {"mAP50_95": 0.0, "mAP50": 0.0, **({"per_class_ap50": {}} if per_class else {})}
    gt = COCO(ann_file)
    ev = COCOeval(gt, gt.loadRes(results), iouType="bbox")
    ev.evaluate()
    ev.accumulate()
    ev.summarize()
    out = {"mAP50_95": float(ev.stats[0]), "mAP50": float(ev.stats[1])}
    if per_class:
        prec = ev.eval["precision"]
        pc = {}
        for k, cat_id in enumerate(gt.getCatIds()):
            name = gt.loadCats(cat_id)[0]["name"]
            ap = prec[0, :, k, 0, 2]
            ap = ap[ap > -1]
            pc[name] = float(np.mean(ap)) if len(ap) else 0.0
        out["per_class_ap50"] = pc
    return out


def train_frcnn(cfg):
    """cfg: dict with SEED, EPOCHS, BATCH_SIZE, LR, WEIGHT_DECAY, MOMENTUM, TRAIN_IMG, TRAIN_ANN, VAL_IMG,
    VAL_ANN, OUT_DIR, AUGMENT (bool), optional WEIGHTS (checkpoint path), NUM_WORKERS."""
    from .dataset import COCODetectionDataset, collate_fn, uint8_transform
    from .augment import RandomCorruptionGPU

    set_seed(cfg["SEED"])
    dev, world, rank = init_device()
    out_dir = Path(cfg["OUT_DIR"])
    if rank == 0:
        out_dir.mkdir(parents=True, exist_ok=True)
        print("Device:", dev, f"(world {world})", flush=True)
        if cfg.get("AUGMENT"):
            print("Mode: AUGMENTED training (corruption p=0.5, on GPU)\n", flush=True)
    # device input pipeline (MX_DEVICE_JPEG, default on): the loader yields file bytes, the host
    # entropy decode is prefetched on threads and the pixel stage runs on the GPU (PrefetchJpegLoader)
    device_jpeg = cfg.get("DEVICE_JPEG", os.environ.get("MX_DEVICE_JPEG", "1") != "0")
    train_ds = COCODetectionDataset(str(cfg["TRAIN_IMG"]), str(cfg["TRAIN_ANN"]), transforms=uint8_transform,
                                    raw=device_jpeg)
    val_ds = COCODetectionDataset(str(cfg["VAL_IMG"]), str(cfg["VAL_ANN"]), transforms=uint8_transform,
                                  raw=device_jpeg)
    sampler = (DistributedSampler(train_ds, world, rank, shuffle=True, seed=cfg["SEED"], drop_last=True)
               if world > 1 else None)
    train_loader = DataLoader(train_ds, batch_size=cfg["BATCH_SIZE"], shuffle=sampler is None, sampler=sampler,
                              num_workers=cfg.get("NUM_WORKERS", 0), collate_fn=collate_fn,
                              pin_memory=not device_jpeg)
    if device_jpeg:
        train_loader = PrefetchJpegLoader(train_loader, dev, workers=cfg.get("DECODE_THREADS", 4))
        if cfg.get("TIMER") is not None:
            cfg["TIMER"]["loader"] = train_loader
    if cfg.get("PRELOAD_DEVICE"):  # diagnostics (bench.py --mode script): every batch decoded up front
        train_loader = [(list(im), [dict(t) for t in tg]) for im, tg in train_loader]
    val_sampler = ShardSampler(len(val_ds), world, rank) if world > 1 else None
    val_loader = DataLoader(val_ds, batch_size=1, shuffle=False, sampler=val_sampler,
                            num_workers=cfg.get("NUM_WORKERS", 0), collate_fn=collate_fn,
                            pin_memory=not device_jpeg)
    if device_jpeg:
        val_loader = PrefetchJpegLoader(val_loader, dev, workers=cfg.get("DECODE_THREADS", 4))
    model = build_frcnn(7, cfg.get("WEIGHTS"), trainable_backbone_layers=cfg.get("TRAINABLE_LAYERS")).to(dev)
    ddp = model
    if world > 1:  # DDP(broadcast_buffers=False) semantics, HIP graphs kept (gradients averaged after backward)
        from .dp import DataParallel
        ddp = DataParallel(model)
        # parameters are identical on every rank now (rank-0 broadcast); the per-rank random streams
        # (corruption choice / noise seeds, RPN and RoI sampler keys) must not be
        set_seed(cfg["SEED"] + rank)
    params = [p for p in model.parameters() if p.requires_grad]
    from .optim import SGD
    scaling = cfg.get("LR_SCALING", os.environ.get("MX_LR_SCALING", "none"))
    if scaling not in ("none", "linear"):
        raise ValueError(f"LR_SCALING must be 'none' or 'linear', got {scaling!r}")
    lr = cfg["LR"] * (world if scaling == "linear" else 1)
    warmup = int(cfg.get("WARMUP_ITERS", 500)) if (scaling == "linear" and world > 1) else 0
    optimizer = SGD(params, lr=lr, momentum=cfg["MOMENTUM"], weight_decay=cfg["WEIGHT_DECAY"])
    sched = torch.optim.lr_scheduler.StepLR(optimizer, step_size=8, gamma=0.1)
    it_global = 0
    corrupt = RandomCorruptionGPU(p=0.5) if cfg.get("AUGMENT") else None
    history, best_ckpt, last_ckpt = out_dir / "history.jsonl", out_dir / "best.pth", out_dir / "last.pth"
    t0 = time.time()
    # cfg["TIMER"] = {"warmup": W}: bench.py --mode script's clock -- after W optimizer steps the device
    # is synchronised and t0 taken, at the end of training t1 and the number of timed steps
    timer = cfg.get("TIMER")
    n_batches = len(train_loader)

    def _start_clock():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        timer["t0"] = time.perf_counter()
        from . import _lib
        _lib.trace_marker(1)  # rocprofv3 kernel-trace delimiters (tools/prof_steps.py)
        if "loader" in timer:
            timer["wait0"] = timer["loader"].wait_s

    if timer is not None:
        if not 0 <= timer["warmup"] < n_batches * cfg["EPOCHS"]:
            raise ValueError(f"TIMER warmup {timer['warmup']} must be below the {n_batches * cfg['EPOCHS']} "
                             "training steps")
        if timer["warmup"] == 0:
            _start_clock()
    kick = getattr(train_loader, "kick", None)
    for epoch in range(1, cfg["EPOCHS"] + 1):
        if sampler is not None:
            sampler.set_epoch(epoch)
        ddp.train()
        epoch_loss = 0.0
        for i, (images, targets) in enumerate(train_loader):
            imgs, tgs = _to_device_batch(images, targets, dev)  # no-op copies for device images
            if corrupt is not None:
                imgs = [corrupt(im) for im in imgs]
            loss_dict = ddp(imgs, tgs)
            losses = sum(loss for loss in loss_dict.values())
            optimizer.zero_grad(set_to_none=True)
            losses.backward()
            if kick is not None:  # the backward is queued: stage the next batch while it runs
                kick()
            if world > 1:
                ddp.sync_gradients()
            if it_global < warmup:  # linear warm-up of the scaled LR (epoch 1 only at the default length)
                for gr in optimizer.param_groups:
                    gr["lr"] = lr * (it_global + 1) / warmup
            it_global += 1
            optimizer.step()
            epoch_loss += float(losses.item())
            if timer is not None and timer["warmup"] > 0 and it_global == timer["warmup"]:
                _start_clock()
            if rank == 0 and ((i + 1) % 100 == 0 or (i + 1) == n_batches):
                print(f"  [Epoch {epoch:03d}] batch {i + 1}/{n_batches}", flush=True)
        if timer is not None and epoch == cfg["EPOCHS"]:
            # the clock stops with the last training step; the epoch-end work (LR step, history, the
            # last.pth checkpoint: ~70 ms of state_dict copies + file write, once per epoch) is timed
            # on its own -- over a 20-step benchmark epoch it would be 3.5 ms per step
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            from . import _lib
            _lib.trace_marker(2)
            timer["t1"], timer["steps"] = time.perf_counter(), it_global - timer["warmup"]
            if "loader" in timer:
                timer["loader_wait_s"] = timer["loader"].wait_s - timer.get("wait0", 0.0)
        sched.step()
        if world > 1:
            t = torch.tensor([epoch_loss], device=dev, dtype=torch.float64)
            dist.all_reduce(t)
            epoch_loss = float(t.item())
        if rank == 0:
            _append_jsonl(history, {"epoch": epoch, "train_loss_sum": epoch_loss,
                                    "lr": float(optimizer.param_groups[0]["lr"]), "mAP50": None, "mAP50_95": None,
                                    "elapsed_sec": int(time.time() - t0)})
            print(f"[Epoch {epoch:03d}/{cfg['EPOCHS']}] loss_sum={epoch_loss:.4f}", flush=True)
            torch.save({"model": model.state_dict(), "epoch": epoch}, last_ckpt)
    if timer is not None:
        torch.cuda.synchronize()
        timer["epoch_end_s"] = time.perf_counter() - timer["t1"]
    if rank == 0:
        print("\nEvaluating on clean val set (final)...", flush=True)
    metrics = evaluate(model, val_loader, str(cfg["VAL_ANN"]), dev)
    if rank == 0:
        print(f"Final | mAP50={metrics['mAP50']:.4f} mAP50-95={metrics['mAP50_95']:.4f}", flush=True)
        torch.save({"model": model.state_dict(), "epoch": "final", "metrics": metrics}, best_ckpt)
        _append_jsonl(history, {"epoch": "final", "train_loss_sum": None,
                                "lr": float(optimizer.param_groups[0]["lr"]), "mAP50": metrics["mAP50"],
                                "mAP50_95": metrics["mAP50_95"], "elapsed_sec": int(time.time() - t0)})
        print("\nTraining done.", flush=True)
        print("Best checkpoint:", best_ckpt.resolve(), flush=True)
    return metrics


def load_frcnn_checkpoint(ckpt_path, dev):
    """eval_all.py:79-87: fasterrcnn_resnet50_fpn_v2(weights=None) + 7-class predictor + best.pth."""
    model = build_frcnn(7)
    ckpt = torch.load(ckpt_path, map_location="cpu", weights_only=True)
    model.load_state_dict(ckpt["model"])
    return model.to(dev).eval()


def eval_frcnn_variant(model, img_dir, ann_file, dev, restorer=None):
    """One test-set variant (eval_all.py:97-143). restorer: optional device U-Net applied to every
    uint8 image before detection (the fused restored-eval path of eval_restored.py)."""
    from .dataset import COCODetectionDataset, collate_fn, uint8_transform
    world, rank, _ = dist_info()
    device_jpeg = os.environ.get("MX_DEVICE_JPEG", "1") != "0"
    ds = COCODetectionDataset(img_dir, ann_file, transforms=uint8_transform, raw=device_jpeg)
    sampler = ShardSampler(len(ds), world, rank) if world > 1 else None
    loader = DataLoader(ds, batch_size=1, shuffle=False, sampler=sampler, num_workers=0, collate_fn=collate_fn,
                        pin_memory=not device_jpeg)
    if device_jpeg:
        loader = DeviceJpegLoader(loader, dev)
    if restorer is not None:
        loader = _RestoredLoader(loader, restorer, dev)
    return evaluate(model, loader, ann_file, dev, per_class=True)


class DeviceJpegLoader:
    """(file bytes, target) batches -> (uint8 HWC device images, target): the hybrid JPEG decoder
    (mx_det.jpeg, bit-identical to PIL's libjpeg-turbo decode). Files it does not handle (progressive,
    CMYK, 4:4:0) are decoded by PIL on the host, as the reference does for every file."""

    def __init__(self, loader, dev):
        self.loader, self.dev = loader, dev

    def _one(self, b):
        from . import jpeg
        try:
            return jpeg.decode(b, self.dev)
        except (jpeg.JpegUnsupported, ValueError):
            # unsupported coding, or a stream the strict parser rejects but libjpeg decodes with a
            # warning: decode on the host exactly as the reference does (PIL raises if it cannot)
            import io
            from PIL import Image
            img = np.asarray(Image.open(io.BytesIO(b.tobytes())).convert("RGB"))
            return torch.from_numpy(img.copy()).to(self.dev)

    def __iter__(self):
        for images, targets in self.loader:
            yield [self._one(b) for b in images], targets

    def __len__(self):
        return len(self.loader)


def _host_decode(b):
    """Host half of one image's decode (a prefetch thread): JPEG -> (info, pinned coefficients), or
    for files the hybrid decoder does not handle, PIL's RGB pixels (the reference's decode)."""
    from . import jpeg
    try:
        return jpeg.host_stage(b)
    except (jpeg.JpegUnsupported, ValueError):
        import io
        from PIL import Image
        return None, np.asarray(Image.open(io.BytesIO(b.tobytes())).convert("RGB")).copy()


def _pack_targets(targets, pin=True):
    """A batch's target dicts as ONE pinned byte buffer (each tensor 8-B aligned) + its layout: one
    host -> HBM copy per batch instead of one per tensor (~11 us of issue each)."""
    layout, off = [], 0
    for t in targets:
        ent = []
        for k, v in t.items():
            v = v.contiguous()
            nb = v.numel() * v.element_size()
            ent.append((k, v, off, nb))
            off += (nb + 7) & ~7
        layout.append(ent)
    if pin:
        from .conv import capture_lock
        with capture_lock:  # a pinned allocation beside an open graph capture would invalidate it
            buf = torch.empty(max(off, 8), dtype=torch.uint8, pin_memory=True)
    else:
        buf = torch.empty(max(off, 8), dtype=torch.uint8)
    for ent in layout:
        for k, v, o, nb in ent:
            if nb:
                buf[o:o + nb].copy_(v.reshape(-1).view(torch.uint8))
    return buf, [[(k, v.dtype, tuple(v.shape), o, nb) for k, v, o, nb in ent] for ent in layout]


def _unpack_targets(dbuf, layout):
    """Device views of the packed targets: same keys, dtypes and shapes as the loader's tensors."""
    return [{k: dbuf[o:o + nb].view(dt).view(shape) for k, dt, shape, o, nb in ent} for ent in layout]


class PrefetchJpegLoader:
    """The training input pipeline on the device (coco_detection_dataset.py:23 + train_frcnn_*.py's
    DataLoader): a loader of (file bytes, target) batches -> (uint8 HWC device images, device targets).
    A producer thread runs the loader (file reads, COCO target tensors), pins the targets and hands
    each image's host entropy decode to `workers` threads (the ctypes decoder releases the GIL), up to
    `depth` batches ahead; a stager thread issues each decoded batch's pinned -> HBM copies and the
    device IDCT / upsampling / colour launches (mx_det.jpeg.device_stage) on a loader stream, one
    batch ahead, so the training thread neither waits for host data work that had a step's time to
    finish nor spends the GPU-idle time after its own host syncs issuing it. Pixels are bit-identical
    to PIL's decode (tests/test_jpeg.py)."""

    def __init__(self, loader, dev, workers=4, depth=2):
        import threading
        self.loader, self.dev, self.workers, self.depth = loader, dev, int(workers), int(depth)
        self.wait_s = 0.0  # time the consuming thread spent waiting for host data (bench.py --mode script)
        self._kick = threading.Event()

    def kick(self):
        """Let the stager issue the next batch's device stage now: called by the training loop once a
        step's backward is queued (train_frcnn), so the stage's host work overlaps the GPU's backward
        instead of the GPU-idle start of the next step. Without kicks the consumer kicks when it runs
        dry (staging then happens at the step start)."""
        self._kick.set()

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        import queue
        import sys
        import threading
        from concurrent.futures import ThreadPoolExecutor
        from . import jpeg
        q = queue.Queue(maxsize=max(1, self.depth))
        stop = threading.Event()
        # the producer's Python work must not hold the GIL for a whole 5 ms switch interval while
        # the training thread waits to issue launches
        old_switch = sys.getswitchinterval()
        sys.setswitchinterval(min(old_switch, 0.0005))

        def put(item):
            while not stop.is_set():
                try:
                    q.put(item, timeout=0.1)
                    return True
                except queue.Full:
                    pass
            return False

        def produce():
            try:
                with ThreadPoolExecutor(max(1, self.workers)) as pool:
                    for images, targets in self.loader:
                        futs = [pool.submit(_host_decode, b) for b in images]
                        if not put((futs, _pack_targets(targets))):
                            return
            except BaseException as e:  # surfaced in the consuming thread
                put(e)
                return
            put(None)

        th = threading.Thread(target=produce, name="mx-prefetch", daemon=True)
        th.start()
        # device stage on a loader stream, issued by a stager thread as soon as a batch's host decode is
        # done: its coefficient / target copies and IDCT launches run beside the training step's kernels
        # and their host cost falls in the training thread's blocking syncs (loss.item(), the RoI
        # sampler's counts) instead of the GPU-idle stretch after them; the training stream waits on
        # the batch's event. One staged batch ahead (bounded HBM for staged images).
        from .conv import capture_lock
        from .conv import dedicated_stream
        ls = dedicated_stream(self.dev, "loader")
        staged = queue.Queue(maxsize=1)

        def put_staged(item):
            while not stop.is_set():
                try:
                    staged.put(item, timeout=0.1)
                    return True
                except queue.Full:
                    pass
            return False

        def stage(item):
            futs, (tbuf, layout) = item
            done = [f.result() for f in futs]
            with capture_lock, torch.cuda.device(self.dev), torch.cuda.stream(ls):
                imgs = [torch.from_numpy(host).to(self.dev) if info is None else jpeg.device_stage(info, host, self.dev)
                        for info, host in done]
                tg = _unpack_targets(tbuf.to(self.dev, non_blocking=True), layout)
                ev = torch.cuda.Event()
                ev.record(ls)
            return imgs, tg, ev

        def stager():
            try:
                while not stop.is_set():
                    try:
                        item = q.get(timeout=0.1)
                    except queue.Empty:
                        continue
                    if isinstance(item, tuple):
                        # wait for the training loop's kick (its backward is queued: the GPU is busy
                        # and the training thread about to block), or for the consumer to run dry
                        while not self._kick.wait(0.1):
                            if stop.is_set():
                                return
                        self._kick.clear()
                        item = stage(item)
                    if not put_staged(item) or item is None or isinstance(item, BaseException):
                        return
            except BaseException as e:  # surfaced in the consuming thread
                put_staged(e)

        st = threading.Thread(target=stager, name="mx-stage", daemon=True)
        st.start()
        try:
            while True:
                t0 = time.perf_counter()
                if staged.empty():
                    self.kick()
                item = staged.get()
                self.wait_s += time.perf_counter() - t0
                if item is None:
                    break
                if isinstance(item, BaseException):
                    raise item
                imgs, tg, ev = item
                main = torch.cuda.current_stream(self.dev)
                main.wait_event(ev)
                for t in imgs + [v for d in tg for v in d.values()]:
                    t.record_stream(main)
                yield imgs, tg
        finally:
            stop.set()
            sys.setswitchinterval(old_switch)


class _RestoredLoader:
    def __init__(self, loader, unet, dev):
        self.loader, self.unet, self.dev = loader, unet, dev

    def __iter__(self):
        for images, targets in self.loader:
            out = [self.unet.restore_u8(im.to(self.dev)[None])[0] for im in images]
            yield out, targets

    def __len__(self):
        return len(self.loader)
