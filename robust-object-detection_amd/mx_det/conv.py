"""Convolution + BatchNorm + activation on libmx_det's MFMA implicit-GEMM kernels (NHWC).

Two arithmetic modes, chosen by the activation dtype:
  f32   precision-faithful (the reference's fp32/TF32 convs, train_frcnn_baseline.py:139-176): f32
        activations and gradients, every product as the bf16x3 split hi*hi + hi*lo + lo*hi on MFMA
        (mx_conv2d_*_x3; weights packed as hi/lo bf16 planes)
  bf16  bf16 activations and operands, f32 accumulation (mx_conv2d_*_ex)
Autograd functions:
  ConvAct      conv (+bias) (+act)                      - RPN head convs, predictor / FC layers
  ConvBNAct    conv -> train-mode BatchNorm2d (+residual) (+act) - ResNet-50 body, FPN, box head
The parameters keep torchvision's shapes ([Cout, Cin, kh, kw] conv weights, BatchNorm affine and
running buffers), so state_dicts load both ways; the kernels take KRSC bf16 copies
(split into hi / lo planes in f32 mode) made once per step.
"""
import contextlib
import ctypes
import gc
import os
import threading
import weakref

import torch
from torch.utils.weak import WeakIdKeyDictionary

from . import _lib
from ._lib import call

ACT_NONE, ACT_RELU, ACT_LEAKY = 0, 1, 2
MX_F32, MX_BF16 = 0, 1


def dcode(t):
    """libmx_det dtype code of an activation tensor."""
    if t.dtype == torch.float32:
        return MX_F32
    if t.dtype == torch.bfloat16:
        return MX_BF16
    raise RuntimeError(f"unsupported activation dtype {t.dtype}")


def is_x3(t):
    """f32 activations run the precision-faithful bf16x3 kernels."""
    return t.dtype == torch.float32


def _s():
    return _lib.stream()


class KernelTimer:
    """Optional live timing of the conv kernels with HIP events on the launch stream (bench.py's
    roofline). Records (kind, algorithmic FLOPs, start/end events) per launch."""

    def __init__(self):
        self.rec = []

    def start(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def stop(self, kind, flops, e0, tag="", byts=0.0):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.rec.append((kind, float(flops), e0, e1, tag, float(byts)))

    def summary(self, by_tag=False):
        """{kind: {launches, flops, ms, bytes}}; by_tag: keyed by (kind, shape tag) instead. bytes =
        algorithmic HBM bytes of the convs (operands read once, output written once)."""
        torch.cuda.synchronize()
        out = {}
        for kind, fl, a, b, tag, by in self.rec:
            d = out.setdefault((kind, tag) if by_tag else kind, {"launches": 0, "flops": 0.0, "ms": 0.0, "bytes": 0.0})
            d["launches"] += 1
            d["flops"] += fl
            d["ms"] += a.elapsed_time(b)
            d["bytes"] += by
        return out


def _tag(N, H, W, C, K, R, S, stride):
    return f"{N}x{H}x{W}x{C}->{K} {R}x{S}/{stride[0]}"


_timer = None


def set_timer(t):
    global _timer
    _timer = t


def _p(t):
    return t.data_ptr() if t is not None else None


def out_hw(H, W, R, S, stride, pad):
    return (H + 2 * pad[0] - R) // stride[0] + 1, (W + 2 * pad[1] - S) // stride[1] + 1


def shape(x_nhwc, K, R, S, stride, pad):
    N, H, W, C = x_nhwc.shape
    Ho, Wo = out_hw(H, W, R, S, stride, pad)
    return _lib.ConvShape(N, H, W, C, K, R, S, Ho, Wo, stride[0], stride[1], pad[0], pad[1])


def weight_krsc(w, cin_pad=None):
    """[K,C,R,S] f32 parameter -> [K,R,S,C'] bf16 (C' = cin_pad, zero channels appended)."""
    k = w.detach().permute(0, 2, 3, 1)
    if cin_pad is not None and cin_pad != k.shape[3]:
        k = torch.nn.functional.pad(k, (0, cin_pad - k.shape[3]))
    return k.to(torch.bfloat16).contiguous()


# ---- per-shape launch configuration (the reference trains with cudnn.benchmark=True) -------------
# Small layers (layer3/4, small FPN levels, box head) sit between latency chains (fewer, longer
# blocks) and split-K partial traffic (more blocks): the best block tile / split cap / wgrad block
# target differs per shape. The first eager launch of a shape times each candidate with HIP events
# on the launch stream (outputs are pure functions of the inputs, so re-running is harmless) and
# the winner is reused (and baked into the captured graphs). MX_CONV_TUNE=0: library defaults.
# fwd / dgrad: (block tile BMTxBN override, split-K cap, buffer-kernel LDS ring depth); 0 = auto
_FD_CANDS = ((0, 0, 0, 0), (0, 0, 1, 0), (0, 0, 2, 0), (64, 64, 0, 0), (64, 64, 1, 0), (128, 128, 1, 0),
             (0, 0, 1, 4), (0, 0, 0, 4), (128, 128, 1, 4))
_WG_CANDS = ((3, 0), (3, 512), (3, 1024), (3, 384), (2, 0), (0, 0))  # (wgrad kernel variant, block target)
# bf16x3 kernels (block tile x split-K cap x ring alternative (3): 128x128 at 3 stages / 1 block per CU,
# 256x128 at 2 stages, ...; wgrad block target)
_FD_CANDS_X3 = ((0, 0, 0, 0), (0, 0, 1, 0), (0, 0, 2, 0), (64, 128, 0, 0), (128, 128, 1, 0), (64, 64, 0, 0),
                (64, 128, 1, 0), (256, 128, 0, 0), (0, 0, 0, 3), (0, 0, 0, 4), (128, 128, 0, 0),
                (0, 0, 0, 5), (64, 64, 0, 5))
if __import__("os").environ.get("MX_X3_ALTW", "1") == "0":  # A/B switch for the newest candidate
    _FD_CANDS_X3 = tuple(c for c in _FD_CANDS_X3 if c[3] != 5)
# wgrad variant 7: LDS-DMA on pre-split hi / lo planes (19 % faster kernel on the P2 3x3, but the split
# pass costs ~70 us there: wins only on the largest shapes)
_WG_CANDS_X3 = ((3, 0), (3, 256), (3, 768), (3, 1024), (4, 0), (4, 512), (5, 0), (5, 512), (7, 0))
if __import__("os").environ.get("MX_X3_DMAW", "1") == "0":  # A/B switch for the newest candidate
    _WG_CANDS_X3 = tuple(c for c in _WG_CANDS_X3 if c[0] != 7)
_tune_cache = {}


def _tune_on():
    import os
    return os.environ.get("MX_CONV_TUNE", "1") != "0"


def _apply_fd(cfg):
    call("mx_conv_set_tile", cfg[0], cfg[1])
    call("mx_conv_set_max_splits", cfg[2])
    call("mx_conv_set_stages", cfg[3])


def _apply_wg(c):
    call("mx_conv_set_wgrad_variant", int(c[0]))
    call("mx_conv_set_wgrad_target", int(c[1]))


_FD_DEFAULT, _WG_DEFAULT = (0, 0, 0, 0), (3, 0)  # the library's own settings (restored after each launch)


_spin = []  # spin-kernel cycles per ms on this device (measured once)


def _gpu_time(run, reps=3):
    """GPU time (ms) of `reps` back-to-back launches of `run`: they are queued behind a ~0.3-ms spin
    kernel, so host launch cost does not gap them (small layers launch faster than Python issues)."""
    def ev():
        return torch.cuda.Event(enable_timing=True)
    if not _spin:
        a, b = ev(), ev()
        a.record()
        torch.cuda._sleep(1 << 20)
        b.record()
        b.synchronize()
        _spin.append((1 << 20) / max(a.elapsed_time(b), 1e-3))
    run()  # warm (first-touch allocations, instruction cache)
    e0, e1 = ev(), ev()
    torch.cuda._sleep(int(0.3 * _spin[0]))
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1)


def _tuned(key, cands, apply, run, default):
    """Launch `run` under the cached best candidate for `key` (timing the candidates at first use).
    MX_CONV_TUNE=0 leaves the library's launch settings untouched (defaults or mx_conv_set_*)."""
    if not _tune_on():
        return run()
    cfg = _tune_cache.get(key)
    if cfg is None:
        if _timer is not None or torch.cuda.is_current_stream_capturing():
            cfg = cands[0]
        else:
            # two interleaved rounds, each candidate's faster one kept: a single timing per candidate
            # let clock / cache noise pick different winners from run to run
            ts = [float("inf")] * len(cands)
            for _ in range(2):
                for i, c in enumerate(cands):
                    apply(c)
                    ts[i] = min(ts[i], _gpu_time(run))
            best = None
            for t, c in zip(ts, cands):
                if best is None or t < 0.97 * best[0]:  # prefer the earlier (default) within 3 %
                    best = (t, c)
            cfg = best[1]
            _tune_cache[key] = cfg
    apply(cfg)
    try:
        return run()
    finally:
        apply(default)


def conv_fwd(x, wk, stride, pad, bias=None, residual=None, act=ACT_NONE, out_dtype=None, stats=False, cin=None,
             xp=None):
    """x NHWC, wk KRSC bf16 -> y NHWC; optional BN stat partials. bf16 x: wk [K,R,S,C], output
    out_dtype (default bf16). f32 x (bf16x3): wk [2,K,R,S,C] hi / lo planes, output and residual f32.
    cin: the weight's real input channels (<= C); a 7x7 conv to 64 channels of a <= 4-channel input
    (the ResNet stem) runs mx_conv2d_stem_x3 (MX_STEM_KERNEL=0: the generic x3 kernels). xp: x's
    split_planes (f32 x, C % 32 == 0): mx_conv2d_fwd_x3p reads them instead of splitting x."""
    x3 = is_x3(x)
    assert wk.dtype == torch.bfloat16 and x.is_contiguous() and wk.is_contiguous()
    if x3:
        assert wk.dim() == 5 and wk.shape[0] == 2, wk.shape
        K, R, S, C = wk.shape[1:]
        out_dtype = torch.float32
    else:
        assert x.dtype == torch.bfloat16 and wk.dim() == 4
        K, R, S, C = wk.shape
        out_dtype = out_dtype or torch.bfloat16
    assert x.shape[3] == C, (x.shape, wk.shape)
    sh = shape(x, K, R, S, stride, pad)
    y = torch.empty((sh.N, sh.Ho, sh.Wo, K), dtype=out_dtype, device=x.device)
    st = None
    if stats:
        mb = _lib.load().mx_conv_mblocks(ctypes.byref(sh))
        st = torch.empty((2, mb, K), dtype=torch.float32, device=x.device)
    if residual is not None:
        residual = residual.contiguous()
        assert residual.dtype == (torch.float32 if x3 else torch.bfloat16), residual.dtype
    t0 = _timer.start() if _timer else None
    if (x3 and cin is not None and cin <= 4 and K == 64 and R == 7 and S == 7 and residual is None
            and act in (ACT_NONE, ACT_RELU) and os.environ.get("MX_STEM_KERNEL", "1") != "0"):
        call("mx_conv2d_stem_x3", ctypes.byref(sh), _p(x), _p(wk), _p(bias), int(act), _p(y), _p(st), _s())
        if _timer:
            _timer.stop("x3_fwd64", 2.0 * sh.N * sh.Ho * sh.Wo * K * R * S * cin, t0,
                        _tag(sh.N, sh.H, sh.W, C, K, R, S, stride),
                        x.numel() * x.element_size() + wk.numel() * 2 + y.numel() * y.element_size())
        return (y, st) if stats else y

    def run():
        if x3:
            wsb = _lib.load().mx_conv_workspace_x3(ctypes.byref(sh), 0)
            ws = torch.empty(wsb, dtype=torch.uint8, device=x.device) if wsb else None
            call("mx_conv2d_fwd_x3p" if xp is not None else "mx_conv2d_fwd_x3", ctypes.byref(sh),
                 _p(xp if xp is not None else x), _p(wk), _p(bias), _p(residual), int(act), _p(y), _p(st),
                 _p(ws), wsb, _s())
            return
        wsb = _lib.load().mx_conv_workspace(ctypes.byref(sh), 0)
        ws = torch.empty(wsb, dtype=torch.uint8, device=x.device) if wsb else None
        call("mx_conv2d_fwd_ex", ctypes.byref(sh), _p(x), _p(wk), _p(bias), _p(residual), int(act), _p(y),
             1 if out_dtype == torch.bfloat16 else 0, _p(st), _p(ws), wsb, _s())

    key = ("fwd", x.dtype, sh.N, sh.H, sh.W, C, K, R, S, tuple(stride), tuple(pad), residual is not None, out_dtype,
           xp is not None)
    _tuned(key, _FD_CANDS_X3 if x3 else _FD_CANDS, _apply_fd, run, _FD_DEFAULT)
    if _timer:
        kind = ("x3_" if x3 else "") + ("fwd128" if K > 64 else "fwd64")
        _timer.stop(kind, 2.0 * sh.N * sh.Ho * sh.Wo * K * R * S * C, t0, _tag(sh.N, sh.H, sh.W, C, K, R, S, stride),
                    x.numel() * x.element_size() + wk.numel() * 2 + y.numel() * y.element_size())
    return (y, st) if stats else y


def pack_weight(w, cin_pad=None, stride=(1, 1), pad=(0, 0), kpad=None, krsc=True, dgrad=False, split=False):
    """f32 [K,C,R,S] device parameter -> (wk, wt) in one kernel (mx_conv_pack_weight):
    wk [K,R,S,Cpad] bf16 (fwd operand) and wt, the dgrad operand (taps grouped by stride-parity
    class, output channels zero-padded to kpad); either can be skipped. split: bf16x3 operands,
    wk [2,K,R,S,Cpad] and wt [2 * Cpad*R*S*kpad] as hi / lo planes."""
    w = w.detach()
    if w.dtype != torch.float32 or not w.is_contiguous():
        w = w.float().contiguous()
    K, C, R, S = w.shape
    cp = cin_pad or C
    kp = kpad or K
    np_ = 2 if split else 1
    sh = _lib.ConvShape(1, 1, 1, cp, kp, R, S, 1, 1, stride[0], stride[1], pad[0], pad[1])
    wk = None
    if krsc:
        wk = torch.empty(((2,) if split else ()) + (K, R, S, cp), dtype=torch.bfloat16, device=w.device)
    wt = torch.empty(np_ * cp * R * S * kp, dtype=torch.bfloat16, device=w.device) if dgrad else None
    call("mx_conv_pack_weight", ctypes.byref(sh), _p(w), C, K, _p(wk), _p(wt), int(split), _s())
    return wk, wt


def _ceil8(n):
    return (n + 7) // 8 * 8


class PackDesc(ctypes.Structure):
    _fields_ = [("w", ctypes.c_void_p), ("wk", ctypes.c_void_p), ("wt", ctypes.c_void_p), ("Cin", ctypes.c_int64),
                ("Kout", ctypes.c_int64), ("Cpad", ctypes.c_int64), ("Kpad", ctypes.c_int64), ("R", ctypes.c_int32),
                ("S", ctypes.c_int32), ("stride_h", ctypes.c_int32), ("stride_w", ctypes.c_int32),
                ("pad_h", ctypes.c_int32), ("pad_w", ctypes.c_int32), ("flags", ctypes.c_int32)]


class _Entry:
    __slots__ = ("w", "cp", "kp", "stride", "pad", "wk", "wt", "version", "dense", "split")


class WeightPacker:
    """Per-step bf16 conv operands of a whole model, packed in ONE launch (mx_conv_pack_batched).

    Weights are registered once (f32 parameter or a view of one, its padded channel counts, stride,
    pad, whether the dgrad layout is needed, bf16x3 hi/lo planes or not); `refresh()` repacks
    exactly the entries whose version
    counter moved since they were packed (optimizer step, load_state_dict) -- frozen layers are
    packed once. ConvAct / ConvBNAct take their operands from here when registered and fall back
    to a per-call pack_weight otherwise. Buffers are rewritten in place on the stream, so a
    backward must run before the next refresh that changes its weights (the train loop's order)."""

    def __init__(self):
        self.entries = {}
        self.order = []
        self._plan = None
        self._plan_key = None
        self._descs = None

    @staticmethod
    def key(w, cp, kp, stride, pad, split=False):
        return (w.data_ptr(), tuple(w.shape), cp, kp, tuple(stride), tuple(pad), bool(split))

    def register(self, w, stride, pad, dgrad, dense=False, split=False):
        """dense: the conv covers its whole input (output 1x1, e.g. FC6 as a 7x7 conv on the RoI tile);
        its dgrad operand is laid out for the 1x1-GEMM form. split: bf16x3 hi / lo planes."""
        K, C, R, S = w.shape
        cp, kp = _ceil8(C), _ceil8(K)
        k = self.key(w, cp, kp, stride, pad, split)
        if k in self.entries:
            return
        e = _Entry()
        # detached alias (same storage and version counter): a registered VIEW of a parameter (FC6 /
        # FC7) must not keep its autograd node -- and the parameter's AccumulateGrad node, bound to
        # the stream it was created on -- alive across steps and graph captures
        e.w, e.cp, e.kp, e.stride, e.pad, e.dense = w.detach(), cp, kp, tuple(stride), tuple(pad), bool(dense)
        e.split = bool(split)
        np_ = 2 if split else 1
        e.wk = torch.empty(((2,) if split else ()) + (K, R, S, cp), dtype=torch.bfloat16, device=w.device)
        e.wt = torch.empty(np_ * cp * R * S * kp, dtype=torch.bfloat16, device=w.device) if dgrad else None
        e.version = None
        self.entries[k] = e
        self.order.append(k)
        self._elist = None  # (rebuilt by refresh)

    @staticmethod
    def desc(e):
        K, C, R, S = e.w.shape
        return PackDesc(e.w.data_ptr(), e.wk.data_ptr(), e.wt.data_ptr() if e.wt is not None else None,
                        C, K, e.cp, e.kp, R, S, e.stride[0], e.stride[1], e.pad[0], e.pad[1],
                        (1 if e.dense else 0) | (2 if e.split else 0))

    def fusable(self, params):
        """Per parameter: the entry whose packing mx_sgd_pack_step can fold into the parameter's SGD
        update (the parameter's only entry, covering all of it, <= 49 taps), else None."""
        by_ptr = {}
        for k in self.order:
            e = self.entries[k]
            by_ptr.setdefault(e.w.data_ptr(), []).append(e)
        out = []
        for p in params:
            es = by_ptr.get(p.data_ptr(), ())
            e = es[0] if len(es) == 1 else None
            if e is not None and not (e.w.numel() == p.numel() and e.w.is_contiguous() and p.is_contiguous()
                                      and e.w.shape[2] * e.w.shape[3] <= 49):
                e = None
            out.append(e)
        return out

    @staticmethod
    def mark_packed(entries):
        """The optimizer wrote these entries' operands along with the update (mx_sgd_pack_step)."""
        for e in entries:
            if e is not None:
                e.version = e.w._version

    def refresh(self):
        el = self.__dict__.get("_elist")
        if el is None:  # (key, entry) in registration order; the per-step check below runs right after
            el = self._elist = [(k, self.entries[k]) for k in self.order]  # loss.item(): GPU idle time
        dirty = [k for k, e in el if e.version != e.w._version]
        if not dirty:
            return
        upload = tuple(dirty) != self._plan_key
        if upload:
            descs = (PackDesc * len(dirty))()
            for i, k in enumerate(dirty):
                descs[i] = self.desc(self.entries[k])
            nb = _lib.load().mx_conv_pack_plan_bytes(len(dirty))
            self._plan = torch.empty(nb, dtype=torch.uint8, device=self.entries[dirty[0]].w.device)
            self._descs = descs
            self._plan_key = tuple(dirty)
        call("mx_conv_pack_batched", ctypes.cast(self._descs, ctypes.c_void_p), len(dirty), _p(self._plan),
             self._plan.numel(), int(upload), _s())
        for k in dirty:
            e = self.entries[k]
            e.version = e.w._version

    def lookup(self, w, cp, kp, stride, pad, dgrad, dense=False, split=False):
        e = self.entries.get(self.key(w, cp, kp, stride, pad, split))
        if e is None or e.version != w._version or (dgrad and (e.wt is None or e.dense != dense)):
            return None
        return e.wk, e.wt


_packer = None


def set_packer(p):
    global _packer
    _packer = p


def get_packer():
    return _packer


_nograd_ops = WeakIdKeyDictionary()  # weight tensor -> {layout: (version, (wk, wt))}, no-grad use only


def operands(w, cin_pad, stride, pad, kpad, dgrad, dense=False, split=False):
    """(wk, wt) for a conv weight: from the model's WeightPacker when registered and current, else
    packed now (one launch; the dense dgrad layout by a transpose of wk). An unregistered weight used
    without autograd (eval: the heads' concatenated cls + box weights, cached by their modules) keeps
    its operands while the tensor object and its version counter stay the same; never inside a graph
    capture (a replay must repack what the captured step recomputes)."""
    if _packer is not None:
        r = _packer.lookup(w, cin_pad, kpad, stride, pad, dgrad, dense, split)
        if r is not None:
            return r
    if (not torch.is_grad_enabled() and not w.requires_grad and w.is_cuda
            and os.environ.get("MX_EVAL_OPCACHE", "1") != "0" and not torch.cuda.is_current_stream_capturing()):
        per = _nograd_ops.get(w)
        if per is None:
            per = _nograd_ops[w] = {}
        lk = (cin_pad, kpad, tuple(stride), tuple(pad), bool(dgrad), bool(dense), bool(split))
        e = per.get(lk)
        if e is None or e[0] != w._version:
            e = per[lk] = (w._version, _operands_now(w, cin_pad, stride, pad, kpad, dgrad, dense, split))
        return e[1]
    return _operands_now(w, cin_pad, stride, pad, kpad, dgrad, dense, split)


def _operands_now(w, cin_pad, stride, pad, kpad, dgrad, dense, split):
    if dense and dgrad:
        wk, _ = pack_weight(w, cin_pad, stride, pad, split=split)
        K = w.shape[0]
        planes = wk.view(2 if split else 1, K, -1)
        wt = torch.nn.functional.pad(planes.transpose(1, 2), (0, kpad - K)).contiguous().view(-1)
        return wk, wt
    return pack_weight(w, cin_pad, stride, pad, kpad=kpad, dgrad=dgrad, split=split)


def split_planes(t):
    """f32 tensor -> its bf16x3 planes [2, *shape] (hi, lo: the split the x3 kernels make in registers;
    mx_split_planes). The x3p conv entries read them by LDS-DMA (no split VALU); bitwise the same."""
    t = t.contiguous()
    pl = torch.empty((2,) + tuple(t.shape), dtype=torch.bfloat16, device=t.device)
    call("mx_split_planes", _p(t), t.numel(), _p(pl), _s())
    return pl


def planes_for(n_elems, chans, krs):
    """Whether a conv operand of n_elems f32 values is split into planes once (split_planes) for the
    x3p kernels: its channel count a multiple of 32 (the buffer kernel's K-tile), and enough MFMA work
    per element to pay the split pass (8 B of HBM traffic per element): MX_X3_PLANES=0 turns it off,
    MX_X3_PLANES_KRS (default 1152: a 3x3 conv to 128 channels) is the minimum output channels x taps
    of the conv reading it, MX_X3_PLANES_MIN (default 4M) the minimum element count."""
    if os.environ.get("MX_X3_PLANES", "1") == "0" or chans % 32:
        return False
    return (krs >= int(os.environ.get("MX_X3_PLANES_KRS", "1152"))
            and n_elems >= int(os.environ.get("MX_X3_PLANES_MIN", str(4 << 20))))


def _x_planes(x, K, R, S, dense, wgrad):
    """x's split_planes when the conv's forward (and its wgrad) should read planes, else None: the
    planes its producer wrote beside it (`x._mx_planes`, ConvBNAct with planes_krs), or -- only when
    the weight takes a gradient (the wgrad gains most: per-shape timings) -- one split pass."""
    if not is_x3(x) or dense or R * S > 64 or not planes_for(x.numel(), x.shape[3], K * R * S):
        return None
    pl = getattr(x, "_mx_planes", None)
    if pl is not None and pl.shape[1:] == x.shape:
        return pl
    return split_planes(x) if wgrad else None


def _dy_planes_wanted(n_elems, chans, x3, C, R, S, dense):
    """Whether a conv's dy (n_elems values, chans channels) is read as planes by its dgrad (and, with x's
    planes, its wgrad)."""
    return x3 and not dense and R * S <= 64 and planes_for(n_elems, chans, C * R * S)


def _dy_planes(dy, C, R, S, dense):
    """dy's split_planes for the dgrad (and, with x's planes, the wgrad), or None."""
    if not _dy_planes_wanted(dy.numel(), dy.shape[-1], is_x3(dy), C, R, S, dense):
        return None
    return split_planes(dy)


def _is_dense(x_shape, R, S, stride, pad):
    """A conv whose single output pixel sees the whole input (valid RxS conv on an RxS map)."""
    return (x_shape[1], x_shape[2]) == (R, S) and tuple(pad) == (0, 0) and R * S > 1


def conv_dgrad(dy, wt, x_shape, R, S, stride, pad, residual=None, bnb=None, dyp=None):
    """dy NHWC [N,Ho,Wo,K] (K = the wt's padded output channels), wt from pack_weight(dgrad=True)
    -> dx NHWC [N,H,W,C] of dy's dtype (+ residual, a tensor of dx's shape and dtype added in the
    epilogue, at every pixel once under either stride). f32 dy: bf16x3 kernels on the split wt; dyp: dy's
    split_planes (K % 32 == 0), read by mx_conv2d_dgrad_x3p instead of splitting dy."""
    N, H, W, C = x_shape
    K = dy.shape[3]
    x3 = is_x3(dy)
    assert wt.numel() == (2 if x3 else 1) * C * R * S * K, (wt.numel(), C, R, S, K)
    Ho, Wo = out_hw(H, W, R, S, stride, pad)
    sh = _lib.ConvShape(N, H, W, C, K, R, S, Ho, Wo, stride[0], stride[1], pad[0], pad[1])
    dx = torch.empty((N, H, W, C), dtype=dy.dtype, device=dy.device)
    dyc = dy.contiguous()
    t0 = _timer.start() if _timer else None
    if residual is not None:
        assert residual.dtype == dy.dtype and residual.shape == dx.shape and residual.is_contiguous()
    part, mb = None, (N * H * W + 63) // 64
    if bnb is not None:  # dx is the gradient of a train-mode BN output: its backward partials too
        part = torch.empty((2, mb, C), dtype=torch.float32, device=dy.device)

    def run():
        if x3:
            wsb = _lib.load().mx_conv_workspace_x3(ctypes.byref(sh), 1)
            ws = torch.empty(wsb, dtype=torch.uint8, device=dy.device) if wsb else None
            b = bnb if part is not None else None
            call("mx_conv2d_dgrad_x3p" if dyp is not None else "mx_conv2d_dgrad_x3", ctypes.byref(sh),
                 _p(dyp if dyp is not None else dyc), _p(wt), _p(residual), _p(dx),
                 _p(b.y) if b else None, _p(b.z) if b else None, _p(b.mean) if b else None,
                 _p(b.invstd) if b else None, int(b.act) if b else 0, _p(part), mb, _p(ws), wsb, _s())
            return
        wsb = _lib.load().mx_conv_workspace(ctypes.byref(sh), 1)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dy.device) if wsb else None
        if part is not None:
            call("mx_conv2d_dgrad_bnb", ctypes.byref(sh), _p(dyc), _p(wt), _p(residual), _p(dx), _p(bnb.y),
                 _p(bnb.z), _p(bnb.mean), _p(bnb.invstd), int(bnb.act), _p(part), mb, _p(ws), wsb, _s())
        else:
            call("mx_conv2d_dgrad_ex", ctypes.byref(sh), _p(dyc), _p(wt), _p(residual), _p(dx), _p(ws), wsb, _s())

    key = ("dgrad", dy.dtype, N, H, W, C, K, R, S, tuple(stride), tuple(pad), residual is not None, part is not None,
           dyp is not None)
    _tuned(key, _FD_CANDS_X3 if x3 else _FD_CANDS, _apply_fd, run, _FD_DEFAULT)
    if part is not None:
        bnb.part = part
    if _timer:
        _timer.stop(("x3_" if x3 else "") + "dgrad", 2.0 * N * Ho * Wo * K * R * S * C, t0,
                    _tag(N, H, W, C, K, R, S, stride),
                    dy.numel() * dy.element_size() + wt.numel() * 2 + dx.numel() * dx.element_size())
    return dx


# ---- weight gradients on a side stream ----------------------------------------------------------
# In the backward pass every conv's wgrad is independent of the dgrad chain that the next layers
# wait for, so it runs on a second HIP stream: small-grid layers (layer3/4, small FPN levels) then
# share the chip with the next layers' BN-backward and dgrad instead of running back to back. The
# main stream joins the side stream at the end of the backward pass (an autograd engine callback);
# the operands stay referenced until then. Single-process only: DDP's reducer reads each gradient
# from its AccumulateGrad hook on the main stream, so multi-rank runs keep wgrad in order.
_pending = []
_pending_task = [None]  # the autograd graph task whose end-of-backward callback joins _pending
# The side-stream wgrad's dw reaches AccumulateGrad from the side stream; the backward's end-of-pass
# callback (_join_side) makes the main stream wait for it, so torch's "AccumulateGrad node's stream does
# not match" warning (printed once per process, then the engine's own stream wait) is expected here.
if hasattr(torch.autograd.graph, "set_warn_on_accumulate_grad_stream_mismatch"):
    torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
_dp = False


def set_data_parallel(flag):
    """mx_det.dp.DataParallel (gradients averaged after the backward, not from AccumulateGrad hooks)
    keeps the side stream legal in multi-rank runs."""
    global _dp
    _dp = bool(flag)


class _Uses:
    """Forward uses of one weight by the autograd graphs still waiting for their backward."""
    __slots__ = ("n", "__weakref__")

    def __init__(self):
        self.n = 0


_uses = weakref.WeakValueDictionary()


def _count_use(w):
    """Count a forward use of weight w; a view (FC6's 4-D view of the Linear weight) counts against
    its base parameter, so two views of one parameter in one graph are two uses of it (grad_dest)."""
    if not w.is_leaf and w._base is not None:
        w = w._base
    c = _uses.get(id(w))
    if c is None:
        c = _uses[id(w)] = _Uses()
    c.n += 1
    return c


def side_wgrad_enabled(ctx):
    """Only the gradient of a leaf weight used ONCE in the graph, whose .grad is None, qualifies:
    AccumulateGrad then adopts the tensor without a kernel, so nothing on the main stream reads it
    before the join. A weight shared by several calls (the RPN head over the FPN levels) has its
    gradients summed in autograd's input buffer on the main stream, and an existing .grad is added
    to: both would read dw too early. The use count is dropped by the backward that reads it."""
    import os
    uses, ctx.uses = ctx.uses, None
    if os.environ.get("MX_SIDE_WGRAD", "1") == "0" or _timer is not None:
        return False
    w = ctx.wref()
    if w is None or not w.is_leaf or w.grad is not None or uses is None or uses.n != 1:
        return False
    import torch.distributed as dist
    return _dp or not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1)


# parameter -> (flat bucket, offset): the gradient slots of mx_det.dp.DataParallel (set there, dropped
# by its close()); weak keys, so nothing here keeps a parameter or pickles a bucket with it
grad_slots = WeakIdKeyDictionary()


def grad_dest(ctx):
    """The data-parallel bucket slot (mx_det.dp.DataParallel: `grad_slots[parameter]`) of this conv's
    weight gradient, as a fresh view for the wgrad kernel to write into -- or None. AccumulateGrad
    adopts the returned tensor as `.grad` (autograd holds its only reference), so the gradient is born in
    the all-reduce buffer. Only a weight used ONCE in the graph whose `.grad` is None qualifies (a shared
    weight's calls would all write the same slot before autograd sums them); a view of a parameter (FC6's
    [1024, 256, 7, 7] over the Linear weight) maps to its base's slot, and its uses are counted on the
    base (_count_use), so two views of one parameter disqualify both. Call before side_wgrad_enabled
    (which consumes ctx.uses)."""
    uses = ctx.uses
    if uses is None or uses.n != 1:
        return None
    w = ctx.wref()
    if w is None:
        return None
    p = w if w.is_leaf else w._base
    slot = grad_slots.get(p) if p is not None else None
    if slot is None or not p.is_leaf or p.grad is not None or not w.is_contiguous() or w.numel() != p.numel():
        return None
    flat, off = slot
    return flat.narrow(0, off, p.numel()).view(w.shape)


def wgrad_stream(device):
    """The side stream of the weight gradients. (One per issuing stream measured neutral, r05d.)"""
    return dedicated_stream(device, "wgrad")


def _wgrad_plan(ctx, dy, x, K, R, S, stride, pad, kout=None, cin=None, dyp=None, xp=None):
    """A conv backward's weight gradient, decided before its dgrad is launched: (job or its arguments,
    side, fork event) for _wgrad_run after the dgrad, or None when the weight needs no gradient.

    Side-stream wgrads and the HIP graph executor (profiles r05b-r05f): a captured backward graph is
    cut into in-order node lists along first dependents; each list runs on one hardware queue, and a
    wait between lists costs ~10 us of idle GPU. MX_WGRAD_FORK selects where a side wgrad forks:
      "early" (default) -- from an event recorded here, before the dgrad (the wgrad is prepared first:
                 every allocation and copy on the current stream). The dgrad stays the first dependent,
                 so the dgrad chain -- the backward's critical path -- keeps one queue;
      "late"  -- after its dgrad: the wgrad is the dgrad's first dependent and the chain starts a new
                 list at every conv (A/B 91.0 vs 94.2 img/s for early, r05c). Grouping several wgrads
                 behind one fork measured slower still (90.3 at 3 per fork, 69 at 6: r05f), removed."""
    if not ctx.needs_input_grad[1]:
        return None
    dst = grad_dest(ctx)
    side = side_wgrad_enabled(ctx)
    if side and os.environ.get("MX_WGRAD_FORK", "early") != "late":
        job = wgrad_prepare(dy, x, K, R, S, stride, pad, kout, cin, dst, dyp, xp)
        fork = torch.cuda.Event()
        fork.record()
        return job, side, fork
    return (dy, x, K, R, S, stride, pad, kout, cin, dst, dyp, xp), side, None


def _wgrad_run(plan):
    job, side, fork = plan
    if not isinstance(job, _WgradJob):
        job = wgrad_prepare(*job)
    return wgrad_launch(job, side, fork)


def _join_side():
    cur = torch.cuda.current_stream()
    for ev, _keep in _pending:
        cur.wait_event(ev)
    _pending.clear()


class _WgradJob:
    """A weight gradient's launch prepared ahead of time (wgrad_prepare): shape, operands, output and
    split workspace allocated and the tuner's pick applied, so the launch itself allocates nothing."""
    __slots__ = ("sh", "x3", "entry", "dw", "dyc", "x", "ws", "wsb", "cfg", "kout", "cin", "K", "R", "S", "stride",
                 "t0", "C", "nbytes")


_WG_CANDS_X3P = ((3, 0), (3, 256), (3, 768), (3, 1024))  # the pre-split kernel: block targets only


def wgrad_prepare(dy, x, K, R, S, stride, pad, kout=None, cin=None, out=None, dyp=None, xp=None):
    """Everything of conv_wgrad before the launch: on the current stream (allocations, dy.contiguous(),
    the tuner's first trial of the shape). A side-stream launch forked BEFORE the dgrad (_wgrad_plan)
    needs these done first: a workspace allocated after the dgrad could reuse the dgrad's just-freed
    split-K slab while the dgrad's reduce still reads it. dyp / xp: both operands' split_planes
    (mx_conv2d_wgrad_x3p, the LDS-DMA kernel) -- used only when both are given."""
    j = _WgradJob()
    sh = j.sh = shape(x, K, R, S, stride, pad)
    j.kout = kout = kout or K
    j.C = x.shape[3]
    j.cin = cin = cin or x.shape[3]
    j.K, j.R, j.S, j.stride = K, R, S, stride
    j.x3 = x3 = is_x3(x)
    j.nbytes = dy.numel() * dy.element_size() + x.numel() * x.element_size()
    assert dy.dtype == x.dtype, (dy.dtype, x.dtype)
    pl = x3 and dyp is not None and xp is not None
    wsfn = "mx_conv_workspace_x3p" if pl else "mx_conv_workspace_x3" if x3 else "mx_conv_workspace"
    j.entry = entry = "mx_conv2d_wgrad_x3p" if pl else "mx_conv2d_wgrad_x3" if x3 else "mx_conv2d_wgrad_ex"
    if pl:
        dy, x = dyp, xp  # the operands the launch reads
    if out is not None:
        assert out.shape == (kout, cin, R, S) and out.dtype == torch.float32 and out.is_contiguous(), out.shape
        dw = out
    else:
        dw = torch.empty((kout, cin, R, S), dtype=torch.float32, device=x.device)
    j.dw = dw
    j.x = x
    j.dyc = dyc = dy.contiguous()
    j.t0 = _timer.start() if _timer else None
    key = ("wgrad", x.dtype, sh.N, sh.H, sh.W, j.C, K, R, S, tuple(stride), tuple(pad), pl)
    if key not in _tune_cache and _tune_on() and _timer is None and not torch.cuda.is_current_stream_capturing():
        def trial():  # timed on the current stream; the real launch may go to the side stream
            wsb_ = getattr(_lib.load(), wsfn)(ctypes.byref(sh), 2)
            ws_ = torch.empty(wsb_, dtype=torch.uint8, device=x.device) if wsb_ else None
            call(entry, ctypes.byref(sh), _p(dyc), _p(x), _p(dw), kout, cin, 1, _p(ws_), wsb_, _s())
        _tuned(key, _WG_CANDS_X3P if pl else _WG_CANDS_X3 if x3 else _WG_CANDS, _apply_wg, trial, _WG_DEFAULT)
    j.cfg = _tune_cache.get(key, _WG_DEFAULT) if _tune_on() else None
    if j.cfg is not None:
        _apply_wg(j.cfg)
    j.wsb = getattr(_lib.load(), wsfn)(ctypes.byref(sh), 2)
    j.ws = torch.empty(j.wsb, dtype=torch.uint8, device=x.device) if j.wsb else None
    if j.cfg is not None:
        _apply_wg(_WG_DEFAULT)
    return j


def wgrad_launch(j, side=False, fork=None):
    """Launch a prepared weight gradient (wgrad_prepare) on the current stream, or with side=True on
    the side stream, after `fork` (an event recorded on the current stream) or, without one, after
    everything issued so far on the current stream. Returns dW."""
    stream = _s()
    if side:
        st = wgrad_stream(j.x.device)
        if fork is not None:  # recorded by _wgrad_plan before the dgrad
            st.wait_event(fork)
        else:
            st.wait_stream(torch.cuda.current_stream())
        stream = st.cuda_stream
    if j.cfg is not None:
        _apply_wg(j.cfg)
    call(j.entry, ctypes.byref(j.sh), _p(j.dyc), _p(j.x), _p(j.dw), j.kout, j.cin, 1, _p(j.ws), j.wsb, stream)
    if j.cfg is not None:
        _apply_wg(_WG_DEFAULT)
    if side:
        ev = torch.cuda.Event()
        ev.record(st)
        task = torch._C._current_graph_task_id()
        if not _pending or _pending_task[0] != task:
            # first side wgrad of this backward (a backward that raised never ran its callback: its
            # events stay listed and are joined by this one's)
            _pending_task[0] = task
            torch.autograd.Variable._execution_engine.queue_callback(_join_side)
        # dw itself is NOT held: AccumulateGrad adopts the tensor only while autograd holds the sole
        # reference (an extra one makes it clone dw on the main stream, before the side kernel ran)
        _pending.append((ev, (j.dyc, j.x, j.ws)))
    dw, sh, C, K, R, S, stride, t0 = j.dw, j.sh, j.C, j.K, j.R, j.S, j.stride, j.t0
    x3 = j.x3
    j.dw = None
    if _timer:
        _timer.stop(("x3_" if x3 else "") + "wgrad", 2.0 * sh.N * sh.Ho * sh.Wo * K * R * S * C, t0,
                    _tag(sh.N, sh.H, sh.W, C, K, R, S, stride), j.nbytes + dw.numel() * 4)
    return dw


def conv_wgrad(dy, x, K, R, S, stride, pad, kout=None, cin=None, side=False, out=None):
    """dy NHWC [N,Ho,Wo,K], x NHWC (both bf16, or both f32 -> bf16x3 kernels) -> dW f32
    [kout, cin, R, S] (torch weight layout; the zero-padded channels K > kout, C > cin are dropped).
    side=True (inside a backward pass only): launched on the side stream, joined at the end of the
    backward. out: a preallocated f32 [kout, cin, R, S] destination (grad_dest)."""
    return wgrad_launch(wgrad_prepare(dy, x, K, R, S, stride, pad, kout, cin, out), side)


def act_bias_bwd(gy, y, act, K8, need_db, g_dtype=torch.bfloat16, planes=False):
    """(g, db): g = gy * act'(y) as g_dtype [..., K8] (zero-padded columns; the dgrad/wgrad operand:
    bf16, or f32 for the bf16x3 path), db = sum of g over all but the last dim (f32, or None) --
    one launch (mx_act_bias_bwd). planes=True (f32): (g, db, g's bf16x3 planes) from the same launch
    (mx_act_bias_bwd_p)."""
    K = gy.shape[-1]
    gy = gy.contiguous()
    M = gy.numel() // K
    assert gy.dtype in (torch.bfloat16, torch.float32) and y.dtype == gy.dtype and y.shape == gy.shape
    g = torch.empty(gy.shape[:-1] + (K8,), dtype=g_dtype, device=gy.device)
    db = torch.empty(K, dtype=torch.float32, device=gy.device) if need_db else None
    ws = None
    if need_db:
        ws = bn_scratch(_lib.load().mx_act_bias_bwd_workspace(M, K), gy.device)
    if planes:
        assert gy.dtype == torch.float32 and g_dtype == torch.float32 and M > 0
        gp = torch.empty((2,) + tuple(g.shape), dtype=torch.bfloat16, device=gy.device)
        call("mx_act_bias_bwd_p", _p(gy), _p(y.contiguous()) if act else None, M, K, K8, int(act), _p(g), _p(db),
             _p(ws), ws.numel() if ws is not None else 0, _p(gp), _s())
        return g, db, gp
    call("mx_act_bias_bwd", _p(gy), _p(y.contiguous()) if act else None, dcode(gy), M, K, K8, int(act), _p(g),
         dcode(g), _p(db), _p(ws), ws.numel() if ws is not None else 0, _s())
    return g, db


class GradSlot:
    """Root-gradient absorption inside a captured backward graph: a graph output whose gradient arrives
    in a static buffer (frcnn._Graphs' static_gout) and whose only in-graph consumer can add it itself
    -- a stride-1 conv in its dgrad epilogue (ConvAct), the RPN canvas unpack -- is left out of the
    backward roots; the consumer reads `buf` (set after the forward capture) instead of autograd adding
    the two gradients in a separate pass. `taken` is set when the consumer claims the slot at forward
    time (frcnn._absorb_roots keeps an unclaimed output as an ordinary backward root), `stream` is the
    stream the slot was opened on: the consumer must run there (its backward then reads `buf` in stream
    order; a consumer on another stream would read it outside autograd's cross-stream edges)."""
    __slots__ = ("buf", "taken", "stream")

    def __init__(self):
        self.buf, self.taken, self.stream = None, False, None

    def claim(self):
        self.taken = True
        return self


_absorb = {}
_absorb_on = False


class absorb_mode:
    """Context of a graph capture's forward: modules that can take a root gradient into an in-graph
    consumer create GradSlots (RPNHead.raw)."""

    def __enter__(self):
        global _absorb_on
        self.prev, _absorb_on = _absorb_on, True
        return self

    def __exit__(self, *a):
        global _absorb_on
        _absorb_on = self.prev
        _absorb.clear()
        _chains.clear()


def absorbing():
    return _absorb_on


class GradChain:
    """A tensor read by several convs inside a captured graph (a backbone stage output: the next
    stage's first conv and downsample, and the FPN lateral conv): their backwards run in a fixed
    order; each adds the running sum of the earlier ones' input gradients in its own dgrad epilogue
    (conv_dgrad residual) and hands it on; the last returns the total to autograd, the others None --
    no separate accumulation passes. Consumers join at forward time (n counts them), so a consumer
    that does not see the chain simply returns its gradient to autograd as usual.
    Every consumer must run on ONE stream (recorded at the first join): the running sum passes between
    their backwards outside autograd's edges, so autograd would insert no cross-stream wait for it (the
    downsample-branch side-stream attempt of round 3 crashed the backward capture exactly so); a join
    from another stream raises at forward time."""
    __slots__ = ("n", "seen", "acc", "stream")

    def __init__(self):
        self.n, self.seen, self.acc, self.stream = 0, 0, None, None

    def last(self):
        return self.seen + 1 >= self.n

    def hand(self, dx):
        self.seen += 1
        if self.seen >= self.n:
            self.seen, self.acc = 0, None
            return dx
        self.acc = dx
        return None


_chains = {}


def chain_over(t):
    """Inside a graph capture (absorb_mode): the convs consuming `t` from here on accumulate its
    gradient through one GradChain (MX_GRAD_CHAIN=0: autograd sums them, for A/B checks)."""
    if os.environ.get("MX_GRAD_CHAIN", "1") == "0":
        return
    _chains[id(t)] = (weakref.ref(t), GradChain())


def _cur_stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream if t.is_cuda else None


def _chain_join(t):
    e = _chains.get(id(t))
    if e is None or e[0]() is not t:
        return None
    ch = e[1]
    st = _cur_stream(t)
    if ch.n == 0:
        ch.stream = st
    elif st != ch.stream:
        raise RuntimeError("GradChain: a consumer of a chained tensor runs on a different stream than the "
                           "chain's first consumer; the running gradient sum would cross streams outside "
                           "autograd's edges. Run every consumer of the tensor on one stream.")
    ch.n += 1
    return ch


def _chain_res(chain, res):
    """A dgrad's residual with the chain's running sum added."""
    if chain is None or chain.acc is None:
        return res
    return chain.acc if res is None else res + chain.acc


def absorb_into(t, slot):
    """The next ConvAct consuming tensor `t` (on this stream) adds slot.buf to its input gradient."""
    slot.stream = _cur_stream(t)
    _absorb[id(t)] = (weakref.ref(t), slot)


def _absorb_take(t):
    e = _absorb.pop(id(t), None)
    if e is None or e[0]() is not t:
        return None
    if _cur_stream(t) != e[1].stream:
        raise RuntimeError("GradSlot: the consumer of an absorbed graph output runs on a different stream "
                           "than the slot was opened on; run it on the producer's stream")
    return e[1].claim()


def conv_act_nograd(x, w, b, stride, pad, act, out_dtype):
    """ConvAct's forward without autograd (eval, torch.no_grad): no saved tensors, no dgrad operand, and
    no split of x into planes for a weight gradient nobody takes (planes x's producer wrote are still
    read); bitwise the same y."""
    K = w.shape[0]
    dense = _is_dense(x.shape, w.shape[2], w.shape[3], stride, pad)
    wk, _ = operands(w, x.shape[3], stride, pad, _ceil8(K), False, dense, split=is_x3(x))
    xp = _x_planes(x, K, w.shape[2], w.shape[3], dense, False)
    return conv_fwd(x, wk, stride, pad, bias=b.detach() if b is not None else None, act=act, out_dtype=out_dtype,
                    xp=xp)


class ConvAct(torch.autograd.Function):
    """y = act(conv(x, w) + b). x NHWC (bf16, or f32: bf16x3); w [K,C,R,S] f32 parameter; b f32 [K]
    or None."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, act, out_dtype):
        K = w.shape[0]
        need_dx = ctx.needs_input_grad[0]
        dense = _is_dense(x.shape, w.shape[2], w.shape[3], stride, pad)
        # narrow heads (RPN cls+box 15, predictor 35): the dgrad operand is zero-padded to K8
        wk, wt = operands(w, x.shape[3], stride, pad, _ceil8(K), need_dx, dense, split=is_x3(x))
        xp = _x_planes(x, K, w.shape[2], w.shape[3], dense, ctx.needs_input_grad[1])
        y = conv_fwd(x, wk, stride, pad, bias=b.detach() if b is not None else None, act=act, out_dtype=out_dtype,
                     xp=xp)
        ctx.save_for_backward(x, y, wt if need_dx else None, xp)
        ctx.cfg = (stride, pad, act, w.shape, b is not None)
        ctx.wref, ctx.uses = weakref.ref(w), _count_use(w)
        ctx.slot = _absorb_take(x) if _absorb else None
        ctx.chain = _chain_join(x) if _chains and need_dx else None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y, wt, xp = ctx.saved_tensors
        stride, pad, act, wshape, has_b = ctx.cfg
        K, _, R, S = wshape
        dx = dw = db = None
        K8 = (K + 7) // 8 * 8
        dense = _is_dense(x.shape, R, S, stride, pad)
        need_db = has_b and ctx.needs_input_grad[2]
        if _dy_planes_wanted(gy.numel() // K * K8, K8, is_x3(x), x.shape[3], R, S, dense) and gy.numel():
            # the backward head writes dy's planes beside it (no split pass over the gradient)
            gk, db, gp = act_bias_bwd(gy, y, act, K8, need_db, g_dtype=x.dtype, planes=True)
        else:
            gk, db = act_bias_bwd(gy, y, act, K8, need_db, g_dtype=x.dtype)
            gp = None
        wg = _wgrad_plan(ctx, gk, x, K8, R, S, stride, pad, kout=K, cin=wshape[1], dyp=gp, xp=xp)  # before the dgrad
        if ctx.needs_input_grad[0]:
            if _is_dense(x.shape, R, S, stride, pad):  # 1x1-GEMM form: dX[N, R*S*C] = dY[N, K8] wt
                N, H, W, C = x.shape
                dx = conv_dgrad(gk.view(N, 1, 1, K8), wt, (N, 1, 1, H * W * C), 1, 1, (1, 1), (0, 0)).view(N, H, W, C)
                if ctx.chain is not None and ctx.chain.acc is not None:
                    dx = dx + ctx.chain.acc
                if ctx.slot is not None and ctx.slot.buf is not None:  # claimed slot: its gradient too
                    dx = dx + ctx.slot.buf
            else:
                extra = ctx.slot.buf if ctx.slot is not None else None
                if extra is not None and not (extra.dtype == gk.dtype and extra.shape == x.shape and
                                              extra.is_contiguous()):
                    raise RuntimeError("absorbed gradient needs an input-shaped buffer of the gradient's dtype")
                dx = conv_dgrad(gk, wt, x.shape, R, S, stride, pad, residual=_chain_res(ctx.chain, extra), dyp=gp)
            if ctx.chain is not None:
                dx = ctx.chain.hand(dx)
        if wg is not None:
            dw = _wgrad_run(wg)
        return dx, dw, db, None, None, None, None


_scratch = {}
# held for the duration of every graph capture (frcnn._Graphs / _SegGraphs) and by other threads that
# issue device work (engine.PrefetchJpegLoader's stager): HIP's global capture mode rejects stream /
# allocation calls made from any thread while a capture is open
capture_lock = threading.RLock()


@contextlib.contextmanager
def capture_guard():
    """Around every graph capture: capture_lock, and Python's cyclic GC paused -- a collection inside
    the capture could destroy an earlier step's graph or free its tensors mid-capture."""
    with capture_lock:
        was = gc.isenabled()
        gc.disable()
        try:
            yield
        finally:
            if was:
                gc.enable()


def capture_stream(device):
    """The stream graph captures (frcnn._Graphs / _SegGraphs) warm up AND capture on, one per device:
    the warm-up allocates this stream's reduction scratch (bn_scratch) outside any capture, so no
    workspace is ever allocated from a graph's private pool."""
    return dedicated_stream(device, "capture")


_dedicated = {}


def dedicated_stream(device, name, high_priority=False):
    """The framework's side stream `name` on `device`: a HIP stream of its own (mx_stream_create),
    created once. torch.cuda.Stream() hands out a round-robin pool of 32 streams per device, so a
    process that creates more (a model per test, a loader per epoch) silently aliases two of them --
    measured: a graph capture crashed in hipStreamEndCapture once a newer pool stream aliased the
    capture stream's neighbours. Dedicated streams never alias each other or a pool stream."""
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _dedicated.get((idx, name))
    if s is None:
        h = ctypes.c_void_p()
        call("mx_stream_create_high_priority" if high_priority else "mx_stream_create", idx, ctypes.addressof(h))
        s = _dedicated[(idx, name)] = torch.cuda.ExternalStream(h.value, device=torch.device("cuda", idx))
    return s


_scratch_kept = []


def bn_scratch(nbytes, device):
    """Persistent per-(device, stream) workspace of the one-launch reductions (BN, bias gradients, RPN
    loss): zero-filled when allocated; its leading arrival counters are left zero by every launch, so
    it is reused by every call on that stream (they are stream-ordered). Per stream: launches on two
    streams may overlap and must not share counters. A grown workspace keeps the old one alive (a
    captured graph may still address it)."""
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    t = _scratch.get(key)
    if t is None or t.numel() < nbytes:
        if torch.cuda.is_current_stream_capturing():
            # allocated inside a capture it would come from that graph's private pool and be shared
            # with every later graph on the stream: captures warm up on their capture stream first
            # (capture_stream), so every workspace exists before the capture begins
            raise RuntimeError("bn_scratch: first use of a stream inside a graph capture (warm the capture "
                               "up on conv.capture_stream(device) first)")
        if t is not None:
            _scratch_kept.append(t)
        t = torch.zeros(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
        _scratch[key] = t
    return t


def bn_train_finalize(st, K, M, gamma, beta, eps, momentum, rmean, rvar):
    """Train-mode BatchNorm from the conv's statistics partials st [2, mb, K]: batch mean / invstd, the
    apply's per-channel scale / shift, and the running-stat update in place (mx_bn_finalize_ex)."""
    mean = torch.empty(K, dtype=torch.float32, device=st.device)
    invstd, scale, shift = torch.empty_like(mean), torch.empty_like(mean), torch.empty_like(mean)
    fws = bn_scratch(_lib.load().mx_bn_finalize_workspace(st.shape[1], K), st.device)
    call("mx_bn_finalize_ex", _p(st), st.shape[1], K, M, _p(gamma.detach()), _p(beta.detach()), float(eps),
         float(momentum), _p(rmean), _p(rvar), _p(mean), _p(invstd), _p(scale), _p(shift), _p(fws), fws.numel(), _s())
    return mean, invstd, scale, shift


def conv_bn_act_maxpool(x, conv, bn, act, k, st, pd):
    """Forward-only conv -> train-mode BatchNorm -> act -> max pool, for a block no gradient flows
    through (the frozen ResNet stem: conv1 / bn1 parameters frozen, image input): the conv writes the
    BN statistics partials (mx_conv2d_stem_x3 for the 7x7 stem), and the BN apply runs inside the pool
    (mx_bn_act_maxpool), so the full-resolution activation is written once (the conv output) and
    never re-written. Same running-stat update and result as conv_bn + maxpool."""
    assert is_x3(x) and bn.training
    if bn.num_batches_tracked is not None and id(bn) not in _nbt_batched:
        bn.num_batches_tracked.add_(1)
    w = conv.weight
    wk, _ = operands(w, x.shape[3], conv.stride, conv.padding, _ceil8(w.shape[0]), False, split=True)
    z, stt = conv_fwd(x.contiguous(), wk, conv.stride, conv.padding, stats=True, cin=w.shape[1])
    N, H, W, K = z.shape
    _, _, scale, shift = bn_train_finalize(stt, K, N * H * W, bn.weight, bn.bias, bn.eps, bn.momentum,
                                           bn.running_mean, bn.running_var)
    Ho, Wo = (H + 2 * pd - k) // st + 1, (W + 2 * pd - k) // st + 1
    y = torch.empty((N, Ho, Wo, K), dtype=torch.float32, device=z.device)
    call("mx_bn_act_maxpool", _p(z), N, H, W, K, _p(scale), _p(shift), int(act), k, st, pd, _p(y), _s())
    return y


class ConvBNAct(torch.autograd.Function):
    """y = act(BN_train(conv(x, w)) (+ residual)). Updates running stats in place."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, residual, rmean, rvar, stride, pad, act, eps, momentum, link=None,
                bnb_own=None, bnb_feed=None, planes_krs=0):
        need_dx = ctx.needs_input_grad[0]
        ctx.link, ctx.role = link if link is not None else (None, None)
        ctx.bnb_own, ctx.bnb_feed = bnb_own, bnb_feed
        wk, wt = operands(w, x.shape[3], stride, pad, _ceil8(w.shape[0]), need_dx, split=is_x3(x))
        xp = _x_planes(x, w.shape[0], w.shape[2], w.shape[3], False, ctx.needs_input_grad[1])
        z, st = conv_fwd(x, wk, stride, pad, stats=True, cin=w.shape[1], xp=xp)
        K = w.shape[0]
        M = z.numel() // K
        mean, invstd, scale, shift = bn_train_finalize(st, K, M, gamma, beta, eps, momentum, rmean, rvar)
        y = torch.empty_like(z)
        res = residual.contiguous() if residual is not None else None
        t0 = _timer.start() if _timer else None
        # planes_krs: the output channels x taps of the conv this output feeds (frcnn marks the producers
        # of the P2 / box-head 3x3 inputs): when that conv will read pre-split planes, write them here
        if planes_krs and is_x3(z) and planes_for(M * K, K, planes_krs):
            yp = torch.empty((2,) + tuple(z.shape), dtype=torch.bfloat16, device=z.device)
            call("mx_bn_apply_p", _p(z), M, K, _p(scale), _p(shift), _p(res), int(act), _p(y), _p(yp), _s())
            y._mx_planes = yp
        else:
            call("mx_bn_apply", _p(z), dcode(z), M, K, _p(scale), _p(shift), _p(res), int(act), _p(y), dcode(y),
                 _s())
        if _timer:  # bn kinds record algorithmic HBM bytes instead of FLOPs
            _timer.stop("bn_apply", M * K * z.element_size() * (2 + (1 if res is not None else 0)), t0, f"{M}x{K}")
        ctx.save_for_backward(x, wt if need_dx else None, z, y, mean, invstd, gamma, xp)
        ctx.cfg = (stride, pad, act, w.shape, residual is not None)
        if bnb_own is not None:  # the next conv's dgrad will produce this BN's backward partials
            bnb_own.y, bnb_own.z, bnb_own.mean, bnb_own.invstd, bnb_own.act = y, z, mean, invstd, act
        ctx.wref, ctx.uses = weakref.ref(w), _count_use(w)
        ctx.chain = _chain_join(x) if _chains and need_dx else None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, wt, z, y, mean, invstd, gamma, xp = ctx.saved_tensors
        stride, pad, act, wshape, has_res = ctx.cfg
        K, _, R, S = wshape
        M = z.numel() // K
        gy = gy.to(z.dtype).contiguous()
        sums = torch.empty((2, K), dtype=torch.float32, device=z.device)
        coef = torch.empty((3, K), dtype=torch.float32, device=z.device)
        own = ctx.bnb_own
        if own is not None and own.part is not None:  # partials from the next conv's dgrad epilogue
            part, own.part = own.part, None
            mb = part.shape[1]
            ws = bn_scratch(_lib.load().mx_bn_finalize_workspace(mb, K), z.device)
            call("mx_bn_bwd_finalize", _p(part), mb, K, M, _p(mean), _p(invstd), _p(gamma.detach()), _p(sums),
                 _p(coef), _p(ws), ws.numel(), _s())
        else:
            wsb = _lib.load().mx_bn_bwd_workspace(M, K)
            ws = bn_scratch(wsb, z.device)
            t0 = _timer.start() if _timer else None
            call("mx_bn_bwd_reduce_ex", _p(gy), _p(y), _p(z), dcode(z), M, K, int(act), _p(mean), _p(invstd),
                 _p(gamma.detach()), _p(ws), ws.numel(), _p(sums), _p(coef), _s())
            if _timer:
                _timer.stop("bn_bwd_reduce", M * K * z.element_size() * (3 if act else 2), t0, f"{M}x{K}")
        dz = torch.empty_like(z)
        dres = torch.empty_like(z) if has_res else None
        t0 = _timer.start() if _timer else None
        # dz feeds this conv's dgrad and wgrad: as pre-split planes too when they read them (_dy_planes)
        dzp = None
        if is_x3(z) and R * S <= 64 and planes_for(z.numel(), K, x.shape[3] * R * S):
            dzp = torch.empty((2,) + tuple(z.shape), dtype=torch.bfloat16, device=z.device)
            call("mx_bn_bwd_apply_p", _p(gy), _p(y), _p(z), M, K, int(act), _p(coef), _p(dz), _p(dres), _p(dzp), _s())
        else:
            call("mx_bn_bwd_apply_ex", _p(gy), _p(y), _p(z), dcode(z), M, K, int(act), _p(coef), _p(dz), _p(dres),
                 _s())
        if _timer:
            _timer.stop("bn_bwd_apply", M * K * z.element_size() * (4 + (1 if has_res else 0)), t0, f"{M}x{K}")
        dx = dw = None
        wg = _wgrad_plan(ctx, dz, x, K, R, S, stride, pad, cin=wshape[1], dyp=dzp, xp=xp)  # before the dgrad
        link = ctx.link
        if ctx.role == "sink" and dres is not None:
            link.dres, dres = dres, None  # handed to the block's first conv: added in its dgrad epilogue
        if ctx.needs_input_grad[0]:
            res = None
            if ctx.role == "src":
                res, link.dres = link.dres, None
            feed = ctx.bnb_feed
            chain = ctx.chain
            # BN-backward partials from this epilogue only when it produces the input's whole gradient
            bnb = feed if (feed is not None and feed.y is not None and tuple(stride) == (1, 1)
                           and feed.y.shape == x.shape and (chain is None or chain.last())) else None
            dx = conv_dgrad(dz, wt, x.shape, R, S, stride, pad, residual=_chain_res(chain, res), bnb=bnb, dyp=dzp)
            if chain is not None:
                dx = chain.hand(dx)
        if wg is not None:
            dw = _wgrad_run(wg)
        dgamma = sums[1] if ctx.needs_input_grad[2] else None
        dbeta = sums[0] if ctx.needs_input_grad[3] else None
        return dx, dw, dgamma, dbeta, dres, None, None, None, None, None, None, None, None, None, None, None


class Conv2d(torch.nn.Module):
    """nn.Conv2d-compatible parameters (state_dict keys weight/bias), NHWC activations. out_dtype None:
    the activation dtype of the input (bf16 or f32)."""

    def __init__(self, cin, cout, k, stride=1, padding=0, bias=True, act=ACT_NONE, out_dtype=None):
        super().__init__()
        k = (k, k) if isinstance(k, int) else tuple(k)
        self.stride = (stride, stride) if isinstance(stride, int) else tuple(stride)
        self.padding = (padding, padding) if isinstance(padding, int) else tuple(padding)
        self.weight = torch.nn.Parameter(torch.empty(cout, cin, *k))
        self.bias = torch.nn.Parameter(torch.zeros(cout)) if bias else None
        self.act = act
        self.out_dtype = out_dtype
        torch.nn.init.kaiming_uniform_(self.weight, a=5 ** 0.5)

    def forward(self, x, be):
        return be.conv(x, self.weight, self.bias, self.stride, self.padding, self.act, self.out_dtype)


class BatchNorm2d(torch.nn.Module):
    """nn.BatchNorm2d-compatible parameters/buffers (weight, bias, running_mean, running_var,
    num_batches_tracked); the arithmetic runs inside ConvBN."""

    def __init__(self, c, eps=1e-5, momentum=0.1):
        super().__init__()
        self.eps, self.momentum = eps, momentum
        self.weight = torch.nn.Parameter(torch.ones(c))
        self.bias = torch.nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))


_nbt_batched = set()


_nbt_cache = [None, None, None]  # (modules, their counters, their ids) of the last call


def count_batches(bns):
    """num_batches_tracked += 1 for every module in `bns` in one foreach launch (called once per
    training forward by the model); conv_bn then skips its own per-layer increment for them. The
    counter list and id set are reused while the same modules (and counters) come back: this runs
    right after the previous step's loss.item(), so its host time is GPU idle."""
    global _nbt_batched
    c = _nbt_cache
    if (c[0] is None or len(c[0]) != len(bns) or any(a is not b for a, b in zip(c[0], bns))
            or any(x is not b.num_batches_tracked for x, b in zip(c[1][0], c[1][1]))):
        mods = [b for b in bns if b.num_batches_tracked is not None]
        c[0], c[1], c[2] = list(bns), ([b.num_batches_tracked for b in mods], mods), {id(b) for b in bns}
    if c[1][0]:
        torch._foreach_add_(c[1][0], 1)
    _nbt_batched = c[2]


class ResLink:
    """Residual-gradient hand-off inside a ResNet bottleneck without downsample: the block input x
    feeds conv1 and is the identity added after bn3, so autograd would add conv1's dgrad and the
    identity gradient in a separate pass. The last conv ("sink") keeps its residual gradient here
    instead of returning it, and the first conv ("src", whose backward always runs later: it is
    upstream of the sink) adds it in its dgrad epilogue."""

    def __init__(self):
        self.dres = None

    def bind(self, role):
        return (self, role)


class BNBLink:
    """BN-backward hand-off between a ConvBNAct (the owner, whose BN output y feeds exactly one conv)
    and that next conv (the feeder): the feeder's dgrad IS the owner's incoming gradient, so its
    epilogue also emits the owner's BN-backward column partials (mx_conv2d_dgrad_bnb) and the
    owner's backward finishes them with one small launch (mx_bn_bwd_finalize) instead of a full
    bn_bwd_reduce pass over (dy, y, z). Feeder backward always runs first (it is downstream)."""

    def __init__(self):
        self.y = self.z = self.mean = self.invstd = self.part = None
        self.act = 0


def conv_bn(x, conv, bn, act, residual=None, link=None, bnb_own=None, bnb_feed=None):
    """Conv2d(bias=False) + BatchNorm2d (+ residual) + activation as one fused unit. Train mode:
    batch statistics + running-stat update (nn.BatchNorm2d semantics); eval: BN folded into the conv."""
    if bn.training:
        if bn.num_batches_tracked is not None and id(bn) not in _nbt_batched:
            bn.num_batches_tracked.add_(1)
        return ConvBNAct.apply(x, conv.weight, bn.weight, bn.bias, residual, bn.running_mean, bn.running_var,
                               conv.stride, conv.padding, act, bn.eps, bn.momentum, link, bnb_own, bnb_feed,
                               getattr(conv, "planes_krs", 0))
    return eval_conv_bn(x, conv, bn, act, residual)


class ConvNormAct(torch.nn.Sequential):
    """torchvision Conv2dNormActivation layout: child "0" = Conv2d, child "1" = BatchNorm2d (or a
    parameter-free activation when norm is None), so state_dict keys match (e.g. fpn.inner_blocks.0.0.weight,
    rpn.head.conv.0.0.bias)."""

    def __init__(self, cin, cout, k, stride=1, padding=None, norm=True, act=ACT_RELU):
        padding = (k - 1) // 2 if padding is None else padding
        conv = Conv2d(cin, cout, k, stride, padding, bias=not norm, act=ACT_NONE if norm else act)
        if norm:
            super().__init__(conv, BatchNorm2d(cout))
        else:
            super().__init__(conv, torch.nn.ReLU() if act == ACT_RELU else torch.nn.Identity())
        self.norm, self.act_code = norm, act

    def forward(self, x, be, residual=None, bnb_own=None, bnb_feed=None):
        if self.norm:
            if bnb_own is None and bnb_feed is None:
                return be.conv_bn(x, self[0], self[1], self.act_code, residual)
            return be.conv_bn(x, self[0], self[1], self.act_code, residual, bnb_own=bnb_own, bnb_feed=bnb_feed)
        c = self[0]
        return be.conv(x, c.weight, c.bias, c.stride, c.padding, c.act, c.out_dtype)


def fold_bn(conv, bn):
    """Eval-mode BatchNorm folded into the conv: w' = w*gamma/sqrt(var+eps), b' = beta - mean*scale."""
    scale = bn.weight.detach() / torch.sqrt(bn.running_var + bn.eps)
    w = conv.weight.detach() * scale.view(-1, 1, 1, 1)
    b = bn.bias.detach() - bn.running_mean * scale
    if conv.bias is not None:
        b = b + conv.bias.detach() * scale
    return w, b.float().contiguous()


def cached_operand(owner, key, tensors, make):
    """make()'s value, kept in owner.__dict__ while every tensor of `tensors` keeps its storage and version
    counter: eval-mode BN folding + packing ran ~5 torch ops and a pack launch per conv per image. A
    BatchNorm's running statistics are written in place by the HIP kernels without a version bump, so the
    folding callers list the module's num_batches_tracked, which every training forward bumps (torch
    in-place add); without it (track_running_stats=False) nothing is cached."""
    if any(t is None for t in tensors) or os.environ.get("MX_EVAL_OPCACHE", "1") == "0":
        return make()
    sig = tuple((t.data_ptr(), t._version) for t in tensors)
    cache = owner.__dict__.setdefault("_mx_opcache", {})
    e = cache.get(key)
    if e is None or e[0] != sig:
        e = cache[key] = (sig, make())
    return e[1]


def _fold_tensors(conv, bn):
    ts = [conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.num_batches_tracked]
    return ts + ([conv.bias] if conv.bias is not None else [])


def eval_conv_bn(x, conv, bn, act, residual=None):
    def make():
        w, b = fold_bn(conv, bn)
        return pack_weight(w, x.shape[3], conv.stride, conv.padding, split=is_x3(x))[0], b
    wk, b = cached_operand(conv, ("fold", id(bn), x.shape[3], is_x3(x)), _fold_tensors(conv, bn), make)
    return conv_fwd(x.contiguous(), wk, conv.stride, conv.padding, bias=b, residual=residual, act=act,
                    cin=conv.weight.shape[1])
