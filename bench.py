"""Headline benchmark: images/sec of the Faster R-CNN R50-FPN v2 train step at 1333x800, bs=2/GPU.

BASELINE.json metric "images/sec FRCNN-R50-FPN train @1333x800 bs=2/GPU, 1/2/4/8 MI355X"; workload =
configs[1] (baseline train, bs=2 per GPU, HIP conv + RoIAlign + NMS ops) — the reference's training
step of scripts/train_frcnn_baseline.py:167-178 (forward + loss sum + zero_grad + backward + SGD
step + loss.item()), on synthetic VisDrone-shaped uint8 images resident in HBM (no dataset offline),
random-init weights of the same architecture, trainable_backbone_layers=3 as in the reference run.
`--augment` adds the on-GPU 50% noise/blur/low-res corruption of configs[2].

Arithmetic: the headline runs the reference's precision -- an fp32 model (train_frcnn_baseline.py:139-176,
no autocast; TF32 convs on its Ampere GPU): HipBackend("f32"), f32 activations / gradients / BN /
RoIAlign, every conv product as the bf16x3 split on MFMA (~2^-16 relative, finer than TF32's 2^-11;
tests/test_gpu_x3.py). The bf16 mode (bf16 activations and operands) is timed after it and reported
inside the same line under "bf16_variant" (--precision f32|bf16 picks one mode only). The same line
also carries "augment_variant" (configs[2]'s step with on-GPU RandomCorruption), and the metric's
"+ eval" half: "eval_variant" (eval_all.py per-image eval forward) and "eval_restored_variant"
(configs[3]: U-Net restore + eval), K images each after W warmup (--no-eval-variant skips them;
mAP@50 is parity-unpinned: no trained checkpoint ships with the reference).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

One process per GPU; gradients all-reduced over RCCL (torch.distributed "nccl") by mx_det.dp.DataParallel;
per-GPU BatchNorm statistics (no SyncBN: each GPU sees the reference's bs=2). Rank 0 prints one
JSON line. Weak scaling: per-GPU work is fixed.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "robust-object-detection_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BF16_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
# f32-equivalent peak of the bf16x3 conv path: three bf16 MFMAs per f32 product
X3_PEAK_TFLOPS = BF16_PEAK_TFLOPS / 3
HBM_PEAK_GBS = 8000.0
N_IMAGES_PER_RANK = 8


def build_model(device, trainable=3, backend=None, precision=None):
    from mx_det import frcnn
    model = frcnn.fasterrcnn_resnet50_fpn_v2(weights=None)
    model.roi_heads.box_predictor = frcnn.FastRCNNPredictor(model.roi_heads.box_predictor.cls_score.in_features, 7)
    frcnn.set_trainable_layers(model.backbone.body, trainable)
    if backend is None and precision is not None:
        from mx_det.backend import HipBackend
        backend = HipBackend(precision)
    if backend is not None:
        model.set_backend(backend)
    return model.to(device)


def make_optimizer(model):
    params = [p for p in model.parameters() if p.requires_grad]
    from mx_det.optim import SGD
    return SGD(params, lr=0.005, momentum=0.9, weight_decay=0.0005)


def train_step(model, opt, images, targets, augment=False, gen=None, as_list=False):
    if augment:
        from mx_det import ops
        B = images.shape[0]
        r = torch.rand(2 * B, generator=gen).tolist()
        codes = [0 if r[2 * i] > 0.5 else 1 + min(int(r[2 * i + 1] * 3), 2) for i in range(B)]
        images = ops.corrupt_u8(images, codes, seed=int(torch.randint(0, 2 ** 62, (1,), generator=gen)))
    if as_list:
        images = list(images)
    loss_dict = model(images, targets)
    losses = sum(loss for loss in loss_dict.values())
    opt.zero_grad(set_to_none=True)
    losses.backward()
    if hasattr(model, "sync_gradients"):  # mx_det.dp.DataParallel
        model.sync_gradients()
    opt.step()
    return float(losses.item())


def host_threads():
    """CPU threads the CPU-baseline legs run on: the host cores this job may use, whatever the launcher
    did to OMP_NUM_THREADS. torch.distributed.run sets OMP_NUM_THREADS=1 in every rank when it was unset
    (so at N>1 torch.get_num_threads() would be 1); _launch_ranks passes the parent's setting on as
    MX_HOST_THREADS. Order: MX_CPU_THREADS (explicit), MX_HOST_THREADS (the launching shell's
    OMP_NUM_THREADS), OMP_NUM_THREADS unless it is torchrun's default of 1 at N>1, else the CPUs this
    process may run on (sched_getaffinity)."""
    for k in ("MX_CPU_THREADS", "MX_HOST_THREADS"):
        v = os.environ.get(k, "")
        if v.isdigit() and int(v) > 0:
            return int(v)
    v = os.environ.get("OMP_NUM_THREADS", "")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if v.isdigit() and int(v) > 0 and not (int(v) == 1 and world > 1):
        return int(v)
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        return max(1, os.cpu_count() or 1)


class _threads:
    """torch.set_num_threads(n) for the block, restored afterwards."""

    def __init__(self, n):
        self.n = n

    def __enter__(self):
        self.old = torch.get_num_threads()
        torch.set_num_threads(self.n)
        return torch.get_num_threads()

    def __exit__(self, *a):
        torch.set_num_threads(self.old)


def cpu_baseline(gpu_model, seconds_hint=30.0):
    """The oracle CPU restatement (oracle/cpu_backend.py: torch-CPU fp32 dense ops + C torchvision ops)
    timed on this host's cores (host_threads()) for ONE train step of the same workload (bs=2, 1333x800)."""
    with _threads(host_threads()) as cores:
        return _cpu_baseline(gpu_model, seconds_hint, cores)


def _cpu_baseline(gpu_model, seconds_hint, cores):
    from oracle.cpu_backend import CpuBackend
    from mx_det.data import synth_batch
    torch.manual_seed(0)
    m = build_model("cpu", backend=CpuBackend())
    m.load_state_dict({k: v.detach().cpu() for k, v in gpu_model.state_dict().items()})
    m.train()
    opt = make_optimizer(m)
    imgs, tg = synth_batch(0, 2)
    t0 = time.perf_counter()
    n = 0
    while True:
        train_step(m, opt, imgs, tg)
        n += 1
        if time.perf_counter() - t0 > seconds_hint or n >= 2:
            break
    dt = time.perf_counter() - t0
    return {"value": 2 * n / dt, "unit": "images/sec", "cores": cores, "kind": "port",
            "sample": f"{n} train step(s) x 2 images 1333x800 on {cores} CPU threads ({dt:.1f} s)"}


TRAFFIC_FILE = os.environ.get("MX_TRAFFIC_FILE", os.path.join(ROOT, "profiles", "r06_traffic.json"))
# kernels of one op: outer list = the op's sequential kernels (summed), inner = alternative template
# instances of one kernel (launch-weighted mean)
KIND_KERNELS = {"x3_wgrad": [["mx::conv_wgrad_x3_kernel", "mx::conv_wgrad_x3w_kernel", "mx::conv_wgrad_x3d_kernel"],
                             ["mx::wgrad_reduce_kernel"]],
                "x3_fwd128": [["mx::conv_x3_buf_kernel<128, 0", "mx::conv_x3_kernel<128, 0"]],
                "x3_fwd64": [["mx::conv_x3_buf_kernel<64, 0", "mx::conv_x3_kernel<64, 0"]],
                "x3_dgrad": [["mx::conv_x3_buf_kernel<128, 1", "mx::conv_x3_buf_kernel<64, 1",
                              "mx::conv_x3_kernel<128, 1", "mx::conv_x3_kernel<64, 1"]],
                "wgrad": [["mx::conv_wgrad_buf_kernel"], ["mx::wgrad_reduce_kernel"]],
                "fwd128": [["mx::conv_igemm_buf_kernel<128, 0", "mx::conv_igemm_buf_kernel<256, 0"]],
                "dgrad": [["mx::conv_igemm_buf_kernel<128, 1", "mx::conv_igemm_buf_kernel<256, 1",
                           "mx::conv_igemm_buf_kernel<64, 1"]],
                "fwd64": [["mx::conv_igemm_buf_kernel<64, 0"]]}


# the graphed headline step's per-kernel table at this HEAD (rocprofv3 kernel trace between bench.py's
# trace markers, tools/prof_steps.py): in the step the side-stream weight gradients overlap the dgrad
# chain and run longer than when event-timed alone, so the dominant kind is chosen from it
STEP_TABLE = os.environ.get("MX_STEP_TABLE", os.path.join(ROOT, "profiles", "r06_in_step_table.txt"))  # CSV; .csv is gpurun-ignored
IN_STEP_KINDS = {"x3_wgrad": ("mx::conv_wgrad_x3", "mx::wgrad_reduce_kernel"),
                 "x3_dgrad": ("mx::conv_x3_buf_kernel<128, 1", "mx::conv_x3_buf_kernel<64, 1", "mx::conv_x3_kernel<128, 1",
                              "mx::conv_x3_kernel<64, 1"),
                 "x3_fwd": ("mx::conv_x3_buf_kernel<128, 0", "mx::conv_x3_buf_kernel<64, 0", "mx::conv_x3_kernel<128, 0",
                            "mx::conv_x3_kernel<64, 0", "mx::conv_stem_x3_kernel"),
                 "x3_split_planes": ("mx::split_planes_kernel",)}


def in_step_ms():
    """{kind: in-step kernel ms per step} from STEP_TABLE, or {} when it is absent."""
    import csv as _csv
    try:
        rows = list(_csv.DictReader(open(STEP_TABLE)))
    except OSError:
        return {}
    out = {}
    for r in rows:
        name = r["kernel"].replace("void ", "")
        for kind, pats in IN_STEP_KINDS.items():
            if name.startswith(pats):
                out[kind] = out.get(kind, 0.0) + float(r["ms_per_step"])
    return out


def pmc_traffic(kind):
    """HBM bytes per launch of the dominant op's kernels, from the committed rocprofv3 PMC pass
    (tools/pmc_traffic.sh -> profiles/r01_traffic.json: 2*FETCH_SIZE + WRITE_SIZE, gfx950-corrected);
    bench.py cannot run the profiler itself. None when the file or the kernels are absent."""
    try:
        import json as _j
        d = _j.load(open(TRAFFIC_FILE))["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    tot, hit = 0.0, False
    for alts in KIND_KERNELS.get(kind, []):
        ks = [v for k, v in d.items() if any(k.startswith(a) for a in alts)]
        if ks:
            n = sum(v["launches"] for v in ks)
            tot += sum(v["bytes_per_launch"] * v["launches"] for v in ks) / n
            hit = True
    return round(tot / 1e6, 2) if hit else None


def conv_roofline(model, opt, imgs, tg, peak=X3_PEAK_TFLOPS, step_fn=None):
    """Live HIP-event timing of every conv kernel launch in one train step (or one call of step_fn);
    the dominant kernel kind (largest total time) is reported with its algorithmic FLOPs (2 * M * N * K
    per conv, f32-equivalent for the bf16x3 path) against the peak of the arithmetic it runs (bf16
    dense / 3 for bf16x3)."""
    from mx_det import conv as mc
    t = mc.KernelTimer()
    mc.set_timer(t)
    graphs = os.environ.get("MX_GRAPHS")
    os.environ["MX_GRAPHS"] = "0"  # an eager step: every conv launch passes through the timer
    try:
        if step_fn is None:
            train_step(model, opt, imgs, tg)
        else:
            step_fn()
    finally:
        mc.set_timer(None)
        if graphs is None:
            del os.environ["MX_GRAPHS"]
        else:
            os.environ["MX_GRAPHS"] = graphs
    s = {k: v for k, v in t.summary().items() if not k.startswith("bn_")}  # conv kinds only
    # the dominant kind: the largest in-step time of the graphed step (STEP_TABLE, x3 kinds) when the
    # table exists, else the largest event-timed one
    ins = in_step_ms() if peak == X3_PEAK_TFLOPS else {}
    flops = {"x3_wgrad": s.get("x3_wgrad", {}).get("flops", 0.0), "x3_dgrad": s.get("x3_dgrad", {}).get("flops", 0.0),
             "x3_fwd": s.get("x3_fwd128", {}).get("flops", 0.0) + s.get("x3_fwd64", {}).get("flops", 0.0)}
    in_step = {k: {"ms": round(ins[k], 3), "tflops": round(flops[k] / (ins[k] * 1e-3) / 1e12, 1),
                   "frac": round(flops[k] / (ins[k] * 1e-3) / 1e12 / peak, 4)}
               for k in flops if ins.get(k) and flops[k]}
    if "x3_split_planes" in ins:
        in_step["x3_split_planes"] = {"ms": round(ins["x3_split_planes"], 3), "bound": "hbm"}
    big = max((k for k in in_step if "frac" in in_step[k]), key=lambda k: in_step[k]["ms"], default=None)
    dom = {"x3_fwd": "x3_fwd128"}.get(big, big) if big in ("x3_wgrad", "x3_dgrad", "x3_fwd") else None
    if dom not in s:
        dom = max(s, key=lambda k: s[k]["ms"])
    d = s[dom]
    achieved = d["flops"] / (d["ms"] * 1e-3) / 1e12
    traf = pmc_traffic(dom)
    allf = sum(v["flops"] for v in s.values())
    allms = sum(v["ms"] for v in s.values())
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": traf,
            "traffic_unit": "MB per launch (HBM, rocprofv3 PMC, " + os.path.relpath(TRAFFIC_FILE, ROOT) + ")",
            "kernel": {"fwd128": "conv_igemm_buf_kernel<128|256,0,*> (+ conv_splitk_reduce_kernel)",
                       "fwd64": "conv_igemm_buf_kernel<64,0,*> (+ conv_splitk_reduce_kernel)",
                       "dgrad": "conv_igemm_buf_kernel<*,1,*> (+ conv_splitk_reduce_kernel)",
                       "wgrad": "conv_wgrad_buf_kernel (+ wgrad_reduce_kernel)",
                       "x3_fwd128": "conv_x3_buf_kernel<*,0,*> (+ conv_splitk_reduce_kernel<*,float>)",
                       "x3_fwd64": "conv_x3_buf_kernel<64,0,*> (+ conv_splitk_reduce_kernel<*,float>)",
                       "x3_dgrad": "conv_x3_buf_kernel<*,1,*> (+ conv_splitk_reduce_kernel<*,float>)",
                       "x3_wgrad": "conv_wgrad_x3_kernel / _x3d / _x3w (+ wgrad_reduce_kernel)"}[dom],
            "launches_per_step": d["launches"], "avg_launch_us": round(1000 * d["ms"] / d["launches"], 2),
            "gflop_per_launch": round(d["flops"] / d["launches"] / 1e9, 3),
            # operands read once + output written once, mean over the kind's launches; traffic / this
            # is the re-read factor (L2 misses beyond the algorithmic minimum)
            "algorithmic_mb_per_launch": round(d["bytes"] / d["launches"] / 1e6, 2),
            "traffic_ratio": (round(traf / (d["bytes"] / d["launches"] / 1e6), 2) if traf else None),
            "in_step": ({"source": os.path.relpath(STEP_TABLE, ROOT), "dominant": big, "by_kind": in_step}
                        if in_step else None),
            "conv_stack": {"tflops": round(allf / (allms * 1e-3) / 1e12, 2), "gflop_per_step": round(allf / 1e9, 1),
                           "ms_per_step": round(allms, 2),
                           "by_kind": {k: {"launches": v["launches"], "ms": round(v["ms"], 3),
                                           "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 1)}
                                       for k, v in s.items()}}}


def _roi_footprint_bytes(feats, rois, scales, k_min, C, esize):
    """Distinct feature bytes MultiScaleRoIAlign must read: per level, the union over its RoIs of the
    pixel rectangles the bilinear taps can touch ([floor(start), floor(end)+1] clipped; aligned=False,
    torchvision roi_align_kernel.cpp), times C * element size. LevelMapper as torchvision poolers.py."""
    import numpy as np
    r = rois.detach().float().cpu().numpy()
    b = r[:, 1:]
    s = np.sqrt(np.maximum(b[:, 2] - b[:, 0], 0) * np.maximum(b[:, 3] - b[:, 1], 0))
    lv = np.clip(np.floor(4 + np.log2(s / 224 + 1e-30) + 1e-6), k_min, k_min + len(feats) - 1).astype(int) - k_min
    total = 0
    for l, f in enumerate(feats):
        H, W = f.shape[1], f.shape[2]
        m = np.zeros((H, W), bool)
        for x1, y1, x2, y2 in b[lv == l] * scales[l]:
            ys, ye = max(int(np.floor(y1)), 0), min(int(np.floor(max(y2, y1 + 1))) + 1, H - 1)
            xs, xe = max(int(np.floor(x1)), 0), min(int(np.floor(max(x2, x1 + 1))) + 1, W - 1)
            m[ys:ye + 1, xs:xe + 1] = True
        total += int(m.sum()) * C * esize
    return total


_SCRUB = {}


def time_cold(fn, reps=10, scrub_mb=4096):
    """Device time of fn() as it runs inside a train step: caches cold and no host gap. Before every
    rep a 4 GiB read (~0.6 ms) evicts the 4 MiB L2s and the 256 MiB Infinity Cache (the operands come
    from HBM, as in the step where other kernels run between producer and consumer) and keeps the GPU
    busy while the host enqueues fn's launches, so the HIP events bracket only fn's kernels (no Python /
    allocation time). A read, not a fill: a 4 GiB write left the caches full of dirty lines whose
    write-back then ran inside fn's window (the round-2 backward figure's 2.5x). Returns the mean in
    microseconds."""
    dev = torch.device("cuda", torch.cuda.current_device())
    buf = _SCRUB.get(dev)
    if buf is None:
        buf = _SCRUB[dev] = torch.zeros(scrub_mb * 2 ** 20 // 4, dtype=torch.float32, device=dev)
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    sink = torch.empty((), dtype=torch.float32, device=dev)
    for a, b in ev:
        torch.amax(buf, dim=0, out=sink)
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / reps * 1e3


def time_warm(fn, reps=10):
    """Device time of fn() replayed back to back (operands warm in L2 / Infinity Cache, as when the
    producer ran just before), mean in microseconds between the first and last event."""
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def _roi_set(rois, feats, scales, k_min):
    """Which RoI set hbm_ops timed: count and per-level split (LevelMapper, as the kernels do)."""
    w, h = rois[:, 3] - rois[:, 1], rois[:, 4] - rois[:, 2]
    lvl = torch.floor(4 + torch.log2(torch.sqrt((w * h).clamp_min(1e-12)) / 224) + 1e-6).clamp(k_min, k_min + len(feats) - 1)
    return {"rois": int(rois.shape[0]), "per_level": {f"P{int(k)}": int((lvl == k).sum()) for k in
                                                      range(k_min, k_min + len(feats))},
            "source": "the sampled RoIs of one eager train step right after the timed steps (same synthetic "
                      "batch cycle as the timed region)"}


def hbm_ops_roofline(model, opt, imgs, tg, reps=10):
    """RoIAlign forward / backward and the proposal NMS on the inputs of a real train step, timed with
    HIP events on their launch stream (torch's current stream) with cold caches and no host gaps
    (time_cold: the per-step kernel table's conditions), against the 8 TB/s HBM peak. Algorithmic bytes:
    RoIAlign = output K*7*7*C + distinct feature footprint (_roi_footprint_bytes); NMS = boxes (16 B),
    score (4), level (8), image (4) read + kept index (8) written per box (its masks stay in L2/LDS)."""
    from mx_det import ops
    from mx_det.backend import HipBackend
    cap = {}
    o_ra, o_nms, o_sel = HipBackend.multiscale_roi_align, HipBackend.proposal_nms, HipBackend.proposal_nms_select

    def ra(self, feats, rois, scales, k_min, output_size=(7, 7), sampling_ratio=2):
        cap["ra"] = ([f.detach() for f in feats], rois.detach().clone(), list(scales), k_min)
        return o_ra(self, feats, rois, scales, k_min, output_size, sampling_ratio)

    def pn(self, boxes, scores, lvl, group, G, L, thr, max_seg):
        cap["nms"] = (boxes.detach().clone(), scores.detach().clone(), lvl.clone(), group.clone(), G, L, thr, max_seg)
        return o_nms(self, boxes, scores, lvl, group, G, L, thr, max_seg)

    def ps(self, boxes, scores, lvl, group, G, L, thr, max_seg, post):
        cap["nms_sel"] = (boxes.detach().clone(), scores.detach().clone(), lvl.clone(), group.clone(), G, L, thr,
                          max_seg, post)
        return o_sel(self, boxes, scores, lvl, group, G, L, thr, max_seg, post)

    HipBackend.multiscale_roi_align, HipBackend.proposal_nms, HipBackend.proposal_nms_select = ra, pn, ps
    graphs = os.environ.get("MX_GRAPHS")
    os.environ["MX_GRAPHS"] = "0"  # eager: the RoI head graph would replay past the hook
    try:
        train_step(model, opt, imgs, tg)
    finally:
        HipBackend.multiscale_roi_align, HipBackend.proposal_nms, HipBackend.proposal_nms_select = o_ra, o_nms, o_sel
        if graphs is None:
            del os.environ["MX_GRAPHS"]
        else:
            os.environ["MX_GRAPHS"] = graphs
    torch.cuda.synchronize()

    def timed(fn):
        return time_cold(fn, reps)

    res = {}
    if "ra" in cap:
        feats, rois, scales, k_min = cap["ra"]
        K, C, es = rois.shape[0], feats[0].shape[3], feats[0].element_size()
        with torch.no_grad():
            us = timed(lambda: ops.multiscale_roi_align(feats, rois, scales, k_min))
            us_warm = time_warm(lambda: ops.multiscale_roi_align(feats, rois, scales, k_min), reps)
        byts = K * 49 * C * es + _roi_footprint_bytes(feats, rois, scales, k_min, C, es)
        gbs = byts / (us * 1e-6) / 1e9
        res["roi_set"] = _roi_set(rois, feats, scales, k_min)
        res["roi_align_fwd"] = {"kernel": "roi_align_fwd_v8_kernel", "rois": K, "channels": C,
                                "dtype": str(feats[0].dtype).replace("torch.", ""), "avg_launch_us": round(us, 2),
                                "warm_launch_us": round(us_warm, 2),
                                "algorithmic_mb": round(byts / 1e6, 2), "achieved": round(gbs, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                                "timing": "avg_launch_us: cold caches (4 GiB scrub before each rep), GPU time only; "
                                          "warm_launch_us: back-to-back replays (operands in L2 / Infinity Cache)"}
        # backward (deterministic gather): every f32 level-map element written once + gout read once;
        # the op's own call (the autograd node's body), timed without autograd bookkeeping
        fs = [f.clone().requires_grad_(True) for f in feats]
        out = ops.multiscale_roi_align(fs, rois, scales, k_min)
        g = torch.randn_like(out)
        det = ops.roi_align_deterministic(C)
        r_saved, lv_saved = out.grad_fn.saved_tensors
        shapes = [tuple(f.shape) for f in feats]
        us = timed(lambda: ops.multiscale_roi_align_backward(g, r_saved, lv_saved, shapes, list(scales)))
        us_warm = time_warm(lambda: ops.multiscale_roi_align_backward(g, r_saved, lv_saved, shapes, list(scales)), reps)
        maps = sum(f.numel() for f in feats) * 4
        byts = maps + g.numel() * g.element_size()
        gbs = byts / (us * 1e-6) / 1e9
        res["roi_align_bwd"] = {"kernel": "roi_bwd_gather_kernel (+ roi_bwd_prep_kernel)" if det else
                                "roi_align_bwd_kernel (atomics) + zero fill", "deterministic": det, "rois": K,
                                "channels": C, "avg_call_us": round(us, 2), "warm_call_us": round(us_warm, 2),
                                "level_map_mb": round(maps / 1e6, 2),
                                "algorithmic_mb": round(byts / 1e6, 2), "achieved": round(gbs, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)}
    if "nms_sel" in cap:  # the sort-free form on filter_proposals' presorted candidates (default)
        boxes, scores, lvl, group, G, L, thr, max_seg, post = cap["nms_sel"]
        n = boxes.shape[0]
        us = timed(lambda: ops.batched_nms_grouped_sorted(boxes, scores, lvl, group, G, L, thr, max_seg, post))
        us_general = timed(lambda: ops.batched_nms_grouped(boxes, scores, lvl, group, G, L, thr, max_seg))
        byts = n * (16 + 4 + 8 + 4 + 8)
        gbs = byts / (us * 1e-6) / 1e9
        res["proposal_nms"] = {"kernel": "mx_batched_nms_grouped_sorted (pre + mask + scan + post)", "boxes": n,
                               "images": G, "avg_call_us": round(us, 2), "general_path_us": round(us_general, 2),
                               "algorithmic_mb": round(byts / 1e6, 3),
                               "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(gbs / HBM_PEAK_GBS, 5), "bound": "latency (dependent scan)"}
    elif "nms" in cap:
        boxes, scores, lvl, group, G, L, thr, max_seg = cap["nms"]
        n = boxes.shape[0]
        us = timed(lambda: ops.batched_nms_grouped(boxes, scores, lvl, group, G, L, thr, max_seg))
        byts = n * (16 + 4 + 8 + 4 + 8)
        gbs = byts / (us * 1e-6) / 1e9
        res["proposal_nms"] = {"kernel": "mx_batched_nms_grouped (mask + scan)", "boxes": n, "images": G,
                               "avg_call_us": round(us, 2), "algorithmic_mb": round(byts / 1e6, 3),
                               "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(gbs / HBM_PEAK_GBS, 5), "bound": "latency (dependent scan)"}
    return res


def _time_precision(precision, args, world, rank, dev, imgs, tg):
    """Build the model in one arithmetic mode, run W warmup steps, time exactly K steps between
    barrier + synchronize pairs; returns (model, ddp, opt, seconds over K steps, max over ranks)."""
    torch.manual_seed(42)
    model = build_model(dev, precision=precision).train()
    ddp = model
    if dist.is_initialized():  # world > 1, or MX_BENCH_DP=1 (a one-rank nccl group)
        # DDP semantics (rank-0 init, per-GPU BN, averaged gradients) with the HIP graphs kept on:
        # gradients are all-reduced over RCCL after the backward (mx_det.dp.DataParallel)
        from mx_det.dp import DataParallel
        ddp = DataParallel(model)
    opt = make_optimizer(model)
    gen = torch.Generator().manual_seed(1234 + rank)

    as_list = os.environ.get("MX_BENCH_LIST") == "1"  # diagnostics: images as a list, as a DataLoader gives them

    def step(i):
        j = (2 * i) % N_IMAGES_PER_RANK
        return train_step(ddp, opt, imgs[j:j + 2], tg[j:j + 2], args.augment, gen, as_list)

    for i in range(args.warmup):
        step(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    from mx_det import _lib
    _lib.trace_marker(1)  # timed-region markers for the rocprofv3 kernel trace (tools/prof_steps.py)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    _lib.trace_marker(2)
    if world > 1:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    return model, ddp, opt, dt


def _barrier(world):
    if world > 1:
        torch.cuda.synchronize()
        dist.barrier()


def eval_step(model, img, unet=None):
    """One image of the reference's evaluation loop (eval_all.py:106-124, batch_size=1): model([image])
    in eval mode, the detections copied to the host; with unet, the corrupted uint8 image is first
    restored on the device (restore_testsets.py:53-79 fused in front of eval_restored.py:171-184)."""
    with torch.no_grad():
        if unet is not None:
            img = unet.restore_u8(img[None])[0]
        out = model([img])[0]
        return out["boxes"].cpu(), out["scores"].cpu(), out["labels"].cpu()


def _time_eval(precision, args, world, rank, dev, imgs, restored):
    """Eval-mode per-image throughput: W warmup images, then exactly K images timed between
    barrier + synchronize pairs (each rank evaluates its own shard, as engine.evaluate does)."""
    from mx_det.unet import RestorationUNet
    torch.manual_seed(42)
    model = build_model(dev, precision=precision).eval()
    unet = RestorationUNet(channels=(32, 64, 128, 256), precision=precision).to(dev).eval() if restored else None
    n = imgs.shape[0]
    for i in range(args.warmup):
        eval_step(model, imgs[i % n], unet)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    from mx_det import _lib
    _lib.trace_marker(1)  # timed-region markers (tools/prof_steps.py, tools/step_concurrency.py)
    t0 = time.perf_counter()
    for i in range(args.steps):
        eval_step(model, imgs[(args.warmup + i) % n], unet)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    _lib.trace_marker(2)
    if world > 1:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    return model, unet, dt


def cpu_eval_baseline(gpu_model, gpu_unet, img, seconds_hint=30.0):
    """The oracle CPU restatement (CpuBackend model + oracle/unet_ref.py U-Net) timed on one image of
    the same eval workload, from the GPU models' weights, on host_threads() threads."""
    with _threads(host_threads()) as cores:
        return _cpu_eval_baseline(gpu_model, gpu_unet, img, seconds_hint, cores)


def _cpu_eval_baseline(gpu_model, gpu_unet, img, seconds_hint, cores):
    from oracle.cpu_backend import CpuBackend
    m = build_model("cpu", backend=CpuBackend())
    m.load_state_dict({k: v.detach().cpu() for k, v in gpu_model.state_dict().items()})
    m.eval()
    u8 = img.cpu()
    ref_unet = None
    if gpu_unet is not None:
        from oracle.unet_ref import torch_reference_unet
        ref_unet = torch_reference_unet({k: v.detach().cpu() for k, v in gpu_unet.state_dict().items()},
                                        (32, 64, 128, 256))
    t0 = time.perf_counter()
    n = 0
    while True:
        with torch.no_grad():
            x = u8
            if ref_unet is not None:
                from oracle.unet_ref import restore_cpu
                x = torch.from_numpy(restore_cpu(ref_unet, u8.numpy()))
            m([x])
        n += 1
        if time.perf_counter() - t0 > seconds_hint or n >= 2:
            break
    dt = time.perf_counter() - t0
    what = "U-Net restore + " if ref_unet is not None else ""
    return {"value": n / dt, "unit": "images/sec", "cores": cores, "kind": "port",
            "sample": f"{n} image(s) 1333x800 ({what}eval forward) on {cores} CPU threads ({dt:.1f} s)"}


def eval_main(args, world, rank, dev, imgs):
    restored = args.mode == "eval_restored"
    prec = "bf16" if args.precision == "bf16" else "f32"
    model, unet, dt = _time_eval(prec, args, world, rank, dev, imgs, restored)
    images = args.steps * world
    what = "U-Net restore (fp32) + FRCNN eval" if restored else "FRCNN eval"
    rec = {"metric": f"images/sec {what} @1333x800 bs=1 (per-image)", "value": round(images / dt, 3),
           "unit": "images/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(1000 * dt / args.steps, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": DTYPE_TEXT[prec], "arithmetic": ARITH_TEXT[prec],
           "data": "synthetic VisDrone-shaped uint8 1333x800, random-init weights; detections copied to host",
           "config": {"workload": ("configs[3]: eval_restored.py:171-184 with restore_testsets.py:53-79 fused on "
                                   "the device" if restored else "eval_all.py:97-143 per-image eval forward"),
                      "global_batch": world, "per_gpu_batch": 1, "image": "1333x800",
                      "parallelism": f"shard{world}", "rpn_post_nms_top_n_test": 1000}}
    peak = {"f32": X3_PEAK_TFLOPS, "bf16": BF16_PEAK_TFLOPS}[prec]
    if rank == 0 and not args.no_roofline:
        rec["roofline"] = conv_roofline(model, None, None, None, peak,
                                        step_fn=lambda: eval_step(model, imgs[0], unet))
    if rank == 0 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_eval_baseline(model, unet, imgs[0])
    if rank == 0:
        print(json.dumps(rec), flush=True)


def unet_train_main(args, world, rank, dev):
    """train_restoration.py:199-205 step (batch 8 of 256x256 patches: device corruption, U-Net forward,
    L1 + 0.3 (1 - SSIM), backward, AdamW), patches/sec."""
    from mx_det.restoration import CombinedLoss, RestorationBatcher
    from mx_det.unet import RestorationUNet
    prec = "bf16" if args.precision == "bf16" else "f32"
    torch.manual_seed(42)
    m = RestorationUNet(channels=(32, 64, 128, 256), precision=prec).to(dev).train()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
    crit, batcher = CombinedLoss(0.3), RestorationBatcher(dev)
    from mx_det.data import synth_image
    import numpy as np
    src = torch.from_numpy(np.stack([synth_image(rank * 16 + i, 256, 256) for i in range(16)]))

    def step(i):
        clean = src[(8 * i) % 16:(8 * i) % 16 + 8]
        cor, tgt = batcher(clean)
        loss = crit(m(cor), tgt)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return float(loss.item())

    for i in range(args.warmup):
        step(i)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    rec = {"metric": "patches/sec U-Net restoration train 256x256 bs=8/GPU", "value": round(8 * args.steps * world / dt, 3),
           "unit": "patches/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(1000 * dt / args.steps, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": DTYPE_TEXT[prec], "arithmetic": ARITH_TEXT[prec],
           "data": "synthetic VisDrone-shaped uint8 patches, on-device corruption, random-init weights",
           "config": {"workload": "train_restoration.py:199-205 (AdamW, L1 + 0.3 (1 - SSIM))", "global_batch": 8 * world,
                      "per_gpu_batch": 8, "patch": "256x256", "channels": [32, 64, 128, 256],
                      "parallelism": f"replicas{world}"}}
    if rank == 0 and not args.no_roofline:
        peak = {"f32": X3_PEAK_TFLOPS, "bf16": BF16_PEAK_TFLOPS}[prec]
        rec["roofline"] = conv_roofline(m, None, None, None, peak, step_fn=lambda: step(0))
    if rank == 0:
        print(json.dumps(rec), flush=True)


def jpeg_main(args, world, rank, dev):
    """Test-set / loader image decode (coco_detection_dataset.py:23, restore_testsets.py:99): JPEG bytes
    of 1333x800 VisDrone-shaped images (q95 4:2:0, as build_corrupted_testsets writes them) -> uint8
    HWC RGB in HBM. Per image: host entropy decode (1 thread) + copy + device IDCT / upsample / colour.
    The device kernels are also timed alone with HIP events (roofline: HBM bytes = coefficients read
    2 B/coef + planes written and read + RGB written)."""
    import io
    import numpy as np
    from PIL import Image
    from mx_det import jpeg
    from mx_det.data import synth_image
    blobs = []
    for i in range(8):
        b = io.BytesIO()
        Image.fromarray(synth_image(rank * 8 + i, 800, 1333)).save(b, format="JPEG", quality=95)
        blobs.append(b.getvalue())
    for i in range(args.warmup):
        jpeg.decode(blobs[i % 8], dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        jpeg.decode(blobs[i % 8], dev)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # device stage alone
    import ctypes
    from mx_det import _lib
    info, coefs = jpeg.decode_coefs(blobs[0])
    cd = torch.from_numpy(coefs).to(dev)
    ws = torch.empty(_lib.load().mx_jpeg_workspace(ctypes.byref(info)), dtype=torch.uint8, device=dev)
    out = torch.empty((info.height, info.width, 3), dtype=torch.uint8, device=dev)
    run = lambda: _lib.call("mx_jpeg_reconstruct", cd.data_ptr(), ctypes.byref(info), ws.data_ptr(), ws.numel(),  # noqa: E731
                            out.data_ptr(), 0, _lib.stream())
    run()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(50):
        run()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 50 * 1e3
    byts = coefs.size * 2 + 2 * ws.numel() + out.numel()
    th = time.perf_counter()
    for i in range(16):
        jpeg.decode_coefs(blobs[i % 8])
    host_ms = (time.perf_counter() - th) / 16 * 1e3
    rec = {"metric": "images/sec JPEG decode 1333x800 q95 4:2:0 -> uint8 RGB in HBM", "value": round(args.steps / dt, 3),
           "unit": "images/sec", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(1000 * dt / args.steps, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u8/int16", "data": "synthetic VisDrone-shaped images encoded by PIL",
           "config": {"workload": "coco_detection_dataset.py:23 / restore_testsets.py:99 image decode",
                      "image": "1333x800", "host_entropy_ms": round(host_ms, 3)},
           "roofline": {"bound": "hbm", "achieved": round(byts / (us * 1e-6) / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(byts / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
                        "kernel": "jpeg_idct_kernel + jpeg_colour_kernel", "avg_launch_us": round(us, 2),
                        "algorithmic_mb": round(byts / 1e6, 3)}}
    if not args.no_cpu_baseline:
        tc = time.perf_counter()
        n = 0
        while time.perf_counter() - tc < 3.0:
            np.asarray(Image.open(io.BytesIO(blobs[n % 8])).convert("RGB"))
            n += 1
        rec["cpu_baseline"] = {"value": n / (time.perf_counter() - tc), "unit": "images/sec", "cores": 1,
                               "kind": "reference", "sample": f"{n} PIL (libjpeg-turbo) decodes, 1 thread"}
    print(json.dumps(rec), flush=True)


def script_main(args, world, rank, dev, imgs, tg):
    """The drop-in script's own training loop, timed: scripts.train_frcnn_augmented (engine.train_frcnn,
    train_frcnn_augmented.py:120-216 with RandomCorruption on the device) for one epoch over an on-disk
    synthetic VisDrone-COCO set of 1333x800 JPEGs (q95, written by rank 0 first): file read, host
    entropy decode prefetched on threads, device IDCT, corruption, the train step, loss.item(). The
    first W optimizer steps are warm-up; the K after them are timed (engine TIMER hook: the clock stops
    with the last step; the once-per-epoch tail -- history line, last.pth -- is reported as epoch_end_ms). For comparison
    the same process then times the bench's own augmented step on HBM-resident images."""
    import tempfile
    from pathlib import Path
    from scripts import train_frcnn_baseline as base
    from mx_det.data import write_coco_split
    from mx_det.engine import train_frcnn
    n_train = 2 * world * (args.steps + args.warmup)
    tmp = Path(tempfile.gettempdir()) / f"mx_script_bench_{os.getpid() if world == 1 else os.environ.get('MASTER_PORT', '0')}"
    t_gen = time.perf_counter()
    if rank == 0:
        write_coco_split(tmp / "coco", "train", 0, n_train)
        write_coco_split(tmp / "coco", "val", 100000, 2)
    _barrier(world)
    t_gen = time.perf_counter() - t_gen
    cfg = base.config()
    cfg.update(EPOCHS=1, AUGMENT=True, TRAIN_IMG=tmp / "coco/images/train", VAL_IMG=tmp / "coco/images/val",
               TRAIN_ANN=tmp / "coco/annotations/instances_train.json",
               VAL_ANN=tmp / "coco/annotations/instances_val.json", OUT_DIR=tmp / f"out{rank}", WEIGHTS=None,
               TRAINABLE_LAYERS=3, TIMER={"warmup": args.warmup},
               DECODE_THREADS=int(os.environ.get("MX_DECODE_THREADS", "4")),
               PRELOAD_DEVICE=os.environ.get("MX_SCRIPT_PRELOAD") == "1")
    prof_path = os.environ.get("MX_SCRIPT_PROFILE")  # host cProfile of the script loop (diagnostics)
    if prof_path and rank == 0:
        import cProfile
        import io
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        train_frcnn(cfg)
        pr.disable()
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(45)
        with open(prof_path, "w") as f:
            f.write(buf.getvalue())
    else:
        train_frcnn(cfg)
    dt = cfg["TIMER"]["t1"] - cfg["TIMER"]["t0"]
    steps = cfg["TIMER"]["steps"]
    if world > 1:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    rec = {"metric": "images/sec scripts.train_frcnn_augmented loop @1333x800 bs=2/GPU (JPEG files on disk)",
           "value": round(2 * steps * world / dt, 3), "unit": "images/sec", "n_gpus": world, "steps": steps,
           "warmup": args.warmup, "ms_per_step": round(1000 * dt / steps, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": f"synthetic VisDrone-shaped 1333x800 JPEG q95 files ({n_train} train images, written in "
                   f"{t_gen:.1f} s before the run), random-init weights",
           "config": {"workload": "configs[2] script loop: train_frcnn_augmented.py:120-216 (RandomCorruption "
                                  "p=0.5 on the device), device JPEG decode with threaded host entropy decode",
                      "global_batch": 2 * world, "per_gpu_batch": 2, "parallelism": f"dp{world}",
                      "trainable_backbone_layers": 3}}
    import shutil
    args.augment = True
    m, ddp, opt, dt2 = _time_precision("f32", args, world, rank, dev, imgs, tg)
    rec["bench_step"] = {"workload": "bench.py augmented step, images resident in HBM", "value":
                         round(2 * args.steps * world / dt2, 3), "ms_per_step": round(1000 * dt2 / args.steps, 3)}
    rec["script_over_bench_step"] = round(rec["value"] / rec["bench_step"]["value"], 4)
    if "loader_wait_s" in cfg["TIMER"]:
        rec["loader_wait_ms_per_step"] = round(1000 * cfg["TIMER"]["loader_wait_s"] / steps, 3)
    # outside the clock: the once-per-epoch tail (LR step, history line, last.pth checkpoint)
    rec["epoch_end_ms"] = round(1000 * cfg["TIMER"]["epoch_end_s"], 1)
    _barrier(world)
    if rank == 0:
        shutil.rmtree(tmp, ignore_errors=True)
        print(json.dumps(rec), flush=True)


DTYPE_TEXT = {"f32": "f32", "bf16": "bf16"}
ARITH_TEXT = {"f32": "f32 activations/gradients/BN/RoIAlign; conv products as bf16x3 MFMA (hi*hi + hi*lo + lo*hi, "
                     "f32 accumulate, ~2^-16 rel. per product vs TF32 2^-11)",
              "bf16": "bf16 activations and conv operands, f32 accumulate"}


# VisDrone-DET frame sizes (H, W) as the reference's loader yields them; GeneralizedRCNNTransform
# resizes each to min 800 / max 1333 (padded 768x1344 or 800x1088 batches)
VISDRONE_FRAMES = [(1080, 1920), (1080, 1920), (1500, 2000), (1500, 2000), (765, 1360), (1080, 1920),
                   (540, 960), (1050, 1400)]


def visdrone_main(args, world, rank, dev):
    """The configs[1] train step on the data path the reference actually runs: uint8 frames of VisDrone's
    native sizes, each resized on the device (mx_resize_normalize_pad: normalize + bilinear +
    zero-padded batch in one launch, boxes rescaled), two padded batch shapes alternating."""
    from mx_det.data import synth_image, synth_target
    imgs, tg = [], []
    for k, (H, W) in enumerate(VISDRONE_FRAMES):
        imgs.append(torch.from_numpy(synth_image(rank * 64 + k, H, W)).to(dev))
        tg.append({kk: v.to(dev) for kk, v in synth_target(rank * 64 + k, H, W).items()})
    prec = "f32" if args.precision == "both" else args.precision
    model, ddp, opt, dt = _time_precision(prec, args, world, rank, dev, imgs, tg)
    rec = {"metric": "images/sec FRCNN-R50-FPN train, VisDrone frame sizes (resize on device) bs=2/GPU",
           "value": round(2 * args.steps * world / dt, 3), "unit": "images/sec", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000 * dt / args.steps, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": DTYPE_TEXT[prec],
           "data": "synthetic uint8 frames at VisDrone sizes " + ", ".join(f"{w}x{h}" for h, w in VISDRONE_FRAMES),
           "config": {"workload": "configs[1] train step, native-size frames", "global_batch": 2 * world,
                      "per_gpu_batch": 2, "parallelism": f"dp{world}"}}
    if rank == 0:
        print(json.dumps(rec), flush=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launch_ranks(n):
    """torch.distributed.run --nproc-per-node n over 127.0.0.1 re-running this script with the same
    arguments; returns the launcher's exit code."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():  # torchrun would keep it; recorded for host_threads()
        env.setdefault("MX_HOST_THREADS", os.environ["OMP_NUM_THREADS"])
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this driver (RCCL / CUDA IPC)
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--augment", action="store_true")
    ap.add_argument("--mode", choices=("train", "eval", "eval_restored", "unet_train", "jpeg", "visdrone", "script"),
                    default="train",
                    help="train (default): the headline train step; eval: per-image eval forward "
                         "(eval_all.py); eval_restored: on-device U-Net restore + eval (eval_restored.py); "
                         "visdrone: the train step on uint8 frames of VisDrone's native sizes (resize on device); "
                         "script: scripts.train_frcnn_augmented's own loop over JPEG files on disk")
    ap.add_argument("--precision", choices=("both", "f32", "bf16"), default="both",
                    help="both (default): the f32 headline, then the bf16 variant in the same JSON line")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-augment-variant", action="store_true")
    ap.add_argument("--no-eval-variant", action="store_true", help="skip the eval / eval_restored legs of the train run")
    ap.add_argument("--no-dp-variant", action="store_true",
                    help="skip the one-rank nccl DataParallel leg of the train run (N=1 only)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` run directly: one rank per GPU needs a launcher. Start torch.distributed.run
        # as a child process BEFORE this process makes any HIP call (no exec from a GPU-initialised
        # process) and exit with its return code; the child ranks re-enter main() with WORLD_SIZE set.
        raise SystemExit(_launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU "
                         f"(torch.distributed.run --nproc-per-node {args.gpus}) or pass --gpus {world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device")
    # MX_BENCH_REHEARSE=1: all ranks on cuda:0 over gloo -- exercises the multi-rank code path on a
    # one-GPU box (not a performance measurement); the real N>1 run is one rank per GPU over RCCL
    rehearse = os.environ.get("MX_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    # MX_BENCH_DP=1 at one rank: a world-size-1 nccl group and the DataParallel wrapper, i.e. the N>1
    # code path (RCCL init with device_id, hook-issued async all-reduces beside the graph replays)
    one_rank_dp = world == 1 and os.environ.get("MX_BENCH_DP") == "1"
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or one_rank_dp:
        if rehearse:
            dist.init_process_group("gloo")
        elif one_rank_dp:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        else:
            dist.init_process_group("nccl", device_id=dev)

    from mx_det.data import synth_batch
    imgs, tg = synth_batch(rank * N_IMAGES_PER_RANK, N_IMAGES_PER_RANK, device=dev)
    if args.mode != "train":
        if args.mode == "unet_train":
            unet_train_main(args, world, rank, dev)
        elif args.mode == "jpeg":
            jpeg_main(args, world, rank, dev)
        elif args.mode == "visdrone":
            visdrone_main(args, world, rank, dev)
        elif args.mode == "script":
            script_main(args, world, rank, dev, imgs, tg)
        else:
            eval_main(args, world, rank, dev, imgs)
        if dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()
        return
    precs = ["f32", "bf16"] if args.precision == "both" else [args.precision]
    head = precs[0]
    model, ddp, opt, dt = _time_precision(head, args, world, rank, dev, imgs, tg)
    images = 2 * args.steps * world
    rec = {
        "metric": "images/sec FRCNN-R50-FPN train @1333x800 bs=2/GPU",
        "value": round(images / dt, 3),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * dt / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": DTYPE_TEXT[head],
        "arithmetic": ARITH_TEXT[head],
        "data": "synthetic VisDrone-shaped uint8 1333x800 (G~Poisson(55)), random-init weights",
        "config": {"workload": "configs[1]: FRCNN R50-FPN v2 baseline train step" + (" + 50% on-GPU corruption"
                                                                                   if args.augment else ""),
                   "global_batch": 2 * world, "per_gpu_batch": 2, "image": "1333x800 (padded 1344x800)",
                   "parallelism": f"dp{world}" + (" (nccl group, DataParallel)" if world == 1 and dist.is_initialized()
                                                   else ""), "trainable_backbone_layers": 3},
    }
    peak = {"f32": X3_PEAK_TFLOPS, "bf16": BF16_PEAK_TFLOPS}
    # the measurement legs run a train step through the data-parallel wrapper, whose gradient
    # all-reduces RCCL pairs by issue order: EVERY rank runs them (same collectives, same order) and
    # only rank 0 records; a barrier closes each leg
    if not args.no_roofline:
        rf = conv_roofline(ddp, opt, imgs[0:2], tg[0:2], peak[head])
        ho = hbm_ops_roofline(ddp, opt, imgs[0:2], tg[0:2])
        if rank == 0:
            rec["roofline"], rec["hbm_ops"] = rf, ho
        _barrier(world)
    cpu_model = model  # the CPU baseline starts from the headline model's weights
    for p in precs[1:]:
        del ddp, opt
        torch.cuda.empty_cache()
        m2, ddp, opt, dt2 = _time_precision(p, args, world, rank, dev, imgs, tg)
        var = {"dtype": DTYPE_TEXT[p], "arithmetic": ARITH_TEXT[p], "value": round(images / dt2, 3),
               "ms_per_step": round(1000 * dt2 / args.steps, 3)}
        if not args.no_roofline:
            rf = conv_roofline(ddp, opt, imgs[0:2], tg[0:2], peak[p])
            if rank == 0:
                var["roofline"] = rf
            _barrier(world)
        rec[p + "_variant"] = var
        del m2
    if not args.augment and not args.no_augment_variant:
        # configs[2]'s augmented step (train_frcnn_augmented.py:159-177: RandomCorruption(p=0.5) on the
        # device in front of the same step), headline precision, timed the same way
        del ddp, opt
        torch.cuda.empty_cache()
        args.augment = True
        try:
            m3, ddp, opt, dt3 = _time_precision(head, args, world, rank, dev, imgs, tg)
        finally:
            args.augment = False
        rec["augment_variant"] = {"workload": "configs[2] step: 50% on-GPU noise/blur/lowres (RandomCorruption) + "
                                              "the same train step", "dtype": DTYPE_TEXT[head],
                                  "value": round(images / dt3, 3), "ms_per_step": round(1000 * dt3 / args.steps, 3)}
        del m3
    if world == 1 and not dist.is_initialized() and not args.no_dp_variant:
        # configs[2]'s code path at one GPU: a one-rank nccl (RCCL) group and mx_det.dp.DataParallel --
        # segmented backward graphs, hook-issued async all-reduces, the NMS flag read -- on the headline
        # workload and precision, timed the same way; its ms/step over the headline's is the per-rank
        # overhead the N-GPU run pays on top of the exchange itself
        try:
            del ddp, opt
        except NameError:
            pass
        torch.cuda.empty_cache()
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ["MASTER_PORT"] = str(_free_port())
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        try:
            m5, ddp, opt, dt5 = _time_precision(head, args, world, rank, dev, imgs, tg)
            ddp.close()
        finally:
            dist.destroy_process_group()
        rec["dp_variant"] = {"workload": "configs[1] step through mx_det.dp.DataParallel in a one-rank nccl (RCCL) "
                                         "group (the N-GPU code path)", "dtype": DTYPE_TEXT[head],
                             "parallelism": "dp1 (nccl group, DataParallel)", "value": round(images / dt5, 3),
                             "ms_per_step": round(1000 * dt5 / args.steps, 3),
                             "ratio_to_headline": round(dt5 / dt, 4)}
        del m5, ddp, opt
    if not args.no_eval_variant:
        # the metric's "+ eval" half, in the same driver run: eval_all.py:97-143 per-image eval forward
        # and configs[3] (eval_restored.py: U-Net restore fused in front), headline precision, each rank
        # on its own images (eval is embarrassingly parallel per image), K images timed after W warmup
        for restored, key, what in ((False, "eval_variant", "eval_all.py per-image eval forward (1000 proposals)"),
                                    (True, "eval_restored_variant", "configs[3]: U-Net restore + eval forward")):
            try:
                del ddp, opt
            except NameError:
                pass
            torch.cuda.empty_cache()
            m4, u4, dt4 = _time_eval(head, args, world, rank, dev, imgs, restored)
            rec[key] = {"workload": what, "dtype": DTYPE_TEXT[head], "unit": "images/sec",
                        "value": round(args.steps * world / dt4, 3), "ms_per_image": round(1000 * dt4 / args.steps, 3),
                        "map50": "parity unpinned: no trained checkpoint ships with the reference (random-init weights)"}
            del m4, u4
    if rank == 0 and not args.no_cpu_baseline:
        # host-only, after every timed leg (the other ranks wait at the closing barrier); the same
        # one-node CPU port at any N (per-image work does not shard on the host)
        rec["cpu_baseline"] = cpu_baseline(cpu_model)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
