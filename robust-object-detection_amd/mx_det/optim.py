"""SGD on libmx_det's multi-tensor kernel (mx_sgd_step): torch.optim.SGD's API and update rule.

The reference trains with torch.optim.SGD(params, lr=0.005, momentum=0.9, weight_decay=5e-4) and
StepLR(8, 0.1) (scripts/train_frcnn_baseline.py:149-153, step at :176). This class is a drop-in
(same constructor, param_groups, state_dict with per-parameter 'momentum_buffer', works with
torch.optim.lr_scheduler) whose step() is ONE launch per 64 parameters for f32 CUDA parameters
instead of torch's foreach path (three multi_tensor_apply launches plus host-side grouping).
Parameters that are not f32 CUDA tensors (e.g. a CPU model) take torch's own implementation.
"""
import ctypes
import os

import torch
from torch.autograd.graph import increment_version

from . import _lib


# MX_SGD_PACK=0: keep the update and the conv operand repack as two launches (sgd_kernel, then
# WeightPacker.refresh's pack_batched_kernel before the next forward)
_SGD_PACK = int(os.environ.get("MX_SGD_PACK", "1"))


def mc_PackDesc():
    from .conv import PackDesc
    return PackDesc


class _SgdParam(ctypes.Structure):  # mx_sgd_param
    _fields_ = [("p", ctypes.c_void_p), ("buf", ctypes.c_void_p), ("n", ctypes.c_int64), ("first", ctypes.c_int32),
                ("pack", ctypes.c_int32)]


class SGD(torch.optim.SGD):
    def __init__(self, params, lr=1e-3, momentum=0, dampening=0, weight_decay=0, nesterov=False, **kw):
        super().__init__(params, lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                         nesterov=nesterov, **kw)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        fast = self.__dict__.setdefault("_fast", {})
        for group in self.param_groups:
            if self._pack_step(group):
                continue
            if self._fast_step(group, fast):
                continue
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            if (group.get("maximize") or group["momentum"] == 0 or
                    any(not p.is_cuda or p.dtype != torch.float32 or p.grad.is_sparse or
                        not p.is_contiguous() or not p.grad.is_contiguous() for p in ps)):
                self._torch_step(group, ps)
                continue
            n = len(ps)
            bufs, first = [], (ctypes.c_uint8 * n)()
            for i, p in enumerate(ps):
                st = self.state[p]
                b = st.get("momentum_buffer")
                if b is None:
                    b = st["momentum_buffer"] = torch.empty_like(p, memory_format=torch.contiguous_format)
                    first[i] = 1
                bufs.append(b)
            P = (ctypes.c_void_p * n)(*[p.data_ptr() for p in ps])
            G = (ctypes.c_void_p * n)(*[p.grad.data_ptr() for p in ps])
            B = (ctypes.c_void_p * n)(*[b.data_ptr() for b in bufs])
            N = (ctypes.c_int64 * n)(*[p.numel() for p in ps])
            _lib.call("mx_sgd_step", P, G, B, N, first, n, float(group["lr"]), float(group["momentum"]),
                      float(group["dampening"]), float(group["weight_decay"]), int(group["nesterov"]),
                      _lib.stream())
            # the kernel wrote through raw pointers: bump the version counters as an in-place torch op
            # would (autograd checks, and the conv WeightPacker repacks by version)
            increment_version(ps)
            increment_version(bufs)
            if len(ps) == len(group["params"]):  # all present: cache the static arrays for _fast_step
                self.__dict__.setdefault("_fast", {})[id(group)] = (
                    group["params"], n, P, B, N, (ctypes.c_uint8 * n)(), bufs, [p.data_ptr() for p in ps],
                    [b.data_ptr() for b in bufs])
        return loss

    def _pack_step(self, group):
        """Conv weights registered with the current WeightPacker (mx_det.conv.get_packer) get their
        bf16 operands written by the update itself (mx_sgd_pack_step: one launch for the whole group,
        no separate repack of the new weights before the next forward). Returns False to take the
        other paths (no packer, nothing to fold, or a case the multi-tensor kernel does not cover).
        Steady state (same parameters, buffers and packer): only the gradients' pointers are gathered
        on the host; the device plan is rebuilt when anything else changes."""
        from . import conv as mc
        pk = mc.get_packer()
        if pk is None or _SGD_PACK == 0:
            return False
        ps = group["params"]
        cache = self.__dict__.setdefault("_pk", {})
        c = cache.get(id(group))
        if c is not None and c["ps"] is ps and c["packer"] is pk and c["ready"]:
            grads = [p.grad for p in ps]
            if any(g is None for g in grads):
                return False
            # the plan holds the parameters' and momentum buffers' addresses: still theirs? (per-parameter
            # state dicts cached by identity: no tensor hashing on this host-critical path -- the GPU
            # idles while the optimizer is issued after the backward's last graph launch returns;
            # load_state_dict replaces self.state, which drops this cache)
            if c.get("state") is not self.state or c.get("sdicts") is None:
                c["state"], c["sdicts"] = self.state, [self.state[p] for p in ps]
            if ([p.data_ptr() for p in ps] != c["pptr"] or
                    any(d.get("momentum_buffer") is not b for d, b in zip(c["sdicts"], c["bufs"]))):
                c = None
        if c is None or c["ps"] is not ps or c["packer"] is not pk or not c["ready"]:
            if (not ps or group.get("maximize") or group["momentum"] == 0 or
                    any(p.grad is None or not p.is_cuda or p.dtype != torch.float32 or p.grad.is_sparse or
                        not p.is_contiguous() for p in ps)):
                return False
            c = self._pack_plan(group, pk)
            if c is None:
                return False
            cache[id(group)] = c
            grads = [p.grad for p in ps]
        gptr = [g.data_ptr() for g in grads]
        if gptr != c["gkey"]:
            if any(not g.is_contiguous() or g.dtype != torch.float32 or g.is_sparse or not g.is_cuda for g in grads):
                return False
            c["gdev"] = torch.tensor(gptr, dtype=torch.int64).pin_memory().to(ps[0].device, non_blocking=True)
            c["gkey"] = gptr
        _lib.call("mx_sgd_pack_step", c["plan"].data_ptr(), c["gdev"].data_ptr(), len(ps), c["blocks"], c["lds"],
                  float(group["lr"]), float(group["momentum"]), float(group["dampening"]),
                  float(group["weight_decay"]), int(group["nesterov"]), _lib.stream())
        increment_version(ps)
        increment_version(c["bufs"])
        pk.mark_packed(c["entries"])
        if not c["ready"]:  # first momentum step done: the next plan has every first flag clear
            c["ready"] = all(not f for f in c["first"])
            if not c["ready"]:
                cache.pop(id(group), None)
        return True

    def _pack_plan(self, group, pk):
        ps = group["params"]
        entries = pk.fusable(ps)
        if not any(e is not None for e in entries):
            return None
        n = len(ps)
        # new momentum buffers stay local until the plan is built: a failed build must not leave
        # uninitialised buffers in self.state (a retried step / state_dict would read them as momentum)
        first, bufs, fresh = [], [], {}
        for p in ps:
            b = self.state[p].get("momentum_buffer") if p in self.state else None
            if b is None:
                b = fresh[p] = torch.empty_like(p, memory_format=torch.contiguous_format)
                first.append(1)
            else:
                first.append(0)
            bufs.append(b)
        packs = [e for e in entries if e is not None]
        descs = (mc_PackDesc() * len(packs))(*[pk.desc(e) for e in packs])
        prm = (_SgdParam * n)()
        j = 0
        for i, (p, b, e) in enumerate(zip(ps, bufs, entries)):
            prm[i] = _SgdParam(p.data_ptr(), b.data_ptr(), p.numel(), first[i], j if e is not None else -1)
            j += e is not None
        lib = _lib.load()
        nb = lib.mx_sgd_pack_plan_bytes(n)
        host = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
        blocks, lds = ctypes.c_int64(0), ctypes.c_size_t(0)
        _lib.call("mx_sgd_pack_build", prm, n, descs, host.data_ptr(), nb, ctypes.byref(blocks), ctypes.byref(lds))
        for p, b in fresh.items():
            self.state[p]["momentum_buffer"] = b
        return {"ps": ps, "packer": pk, "pptr": [p.data_ptr() for p in ps], "entries": entries, "bufs": bufs,
                "first": first, "ready": not any(first), "plan": host.to(ps[0].device, non_blocking=True),
                "blocks": blocks.value, "lds": lds.value, "gkey": None}

    def _fast_step(self, group, fast):
        """Steady state: every parameter of the group has a grad and a momentum buffer, and the
        parameter list is unchanged -> reuse the cached pointer arrays; only the grads' pointers
        (new tensors each step) are gathered. Returns False to take the general path."""
        ps = group["params"]
        c = fast.get(id(group))
        if c is None or c[0] is not ps or c[1] != len(ps):
            fast.pop(id(group), None)
            return False
        # parameters and momentum buffers still the cached storage (p.data =, load_state_dict, ...)
        st = self.state
        bufs = [st[p].get("momentum_buffer") if p in st else None for p in ps]
        if (any(b is None for b in bufs) or [p.data_ptr() for p in ps] != c[7]
                or [b.data_ptr() for b in bufs] != c[8]):
            fast.pop(id(group), None)
            return False
        grads = [p.grad for p in ps]
        if any(g is None or not g.is_contiguous() for g in grads):
            return False
        n = len(ps)
        G = (ctypes.c_void_p * n)(*[g.data_ptr() for g in grads])
        _lib.call("mx_sgd_step", c[2], G, c[3], c[4], c[5], n, float(group["lr"]), float(group["momentum"]),
                  float(group["dampening"]), float(group["weight_decay"]), int(group["nesterov"]), _lib.stream())
        increment_version(ps)
        increment_version(c[6])
        return True

    def _torch_step(self, group, ps):
        for p in ps:
            d = p.grad
            if group["weight_decay"]:
                d = d.add(p, alpha=group["weight_decay"])
            if group["momentum"]:
                st = self.state[p]
                b = st.get("momentum_buffer")
                if b is None:
                    b = st["momentum_buffer"] = d.clone().detach()
                else:
                    b.mul_(group["momentum"]).add_(d, alpha=1 - group["dampening"])
                d = d.add(b, alpha=group["momentum"]) if group["nesterov"] else b
            p.add_(d, alpha=-group["lr"] if not group.get("maximize") else group["lr"])
