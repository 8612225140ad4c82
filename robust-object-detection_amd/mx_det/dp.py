"""Data-parallel training over RCCL that keeps the HIP-graph replays.

torch DistributedDataParallel launches its bucket all-reduces from AccumulateGrad hooks; the
replayed trunk / RoI-head backward graphs write their parameters' gradients directly and bypass
those hooks, so under DDP the model had to run eagerly (24 ms instead of 18 ms per step on one
MI355X). `DataParallel` gives the same semantics as the DDP configuration the reference-style
scripts use (DistributedDataParallel(broadcast_buffers=False)):
  * identical start: parameters and buffers broadcast from rank 0;
  * per-GPU BatchNorm statistics (buffers are never synchronised afterwards);
  * gradients averaged over ranks before the optimizer step
while the graphs stay on. The exchange overlaps the backward: the RoI head's gradients are
all-reduced as soon as its backward graph has replayed, and under this wrapper the trunk's backward
is captured as a chain of per-segment graphs (frcnn._SegGraphs: FPN + RPN head, layer4, layer3,
layer2) whose hand-off hook starts each segment's all-reduce (one flat bucket per segment, 5-60 MB)
on RCCL's stream while the later segments' graphs run; `sync_gradients()` then only waits, scales
and scatters back.

Rank consistency: RCCL pairs collectives by issue order, and whether a unit replays a graph (and so
fires a hook) is decided per rank from local shapes (e.g. a rank whose sampled RoI count differs runs
its RoI head eagerly). The hooks therefore only mark a group ready; collectives are always issued in
one canonical order [roi_heads, fpn+rpn_head, layer4, layer3, layer2, stem+layer1, buckets]. A hook
for a later group first issues every earlier group not yet started (their gradients are final: the
backward produces them before the later group's), so each rank issues the same sizes in the same
order whichever of its units replayed graphs. Anything not started by a hook (eager trunk, other parameters) is reduced there
in ~`bucket_mb` buckets. Over xGMI a ring all-reduce of the 172 MB of f32 gradients costs
~2·(N-1)/N·172 MB / bus bandwidth; with the overlap only the last segment's (layer2, 5 MB) is
exposed.

Persistent buckets: every group (and every remaining bucket) owns ONE flat f32 gradient buffer for
the wrapper's lifetime, and each trainable parameter a fixed slot in it (`conv.grad_slots`, a weak
id-keyed map owned by this wrapper and cleared by `close()`; nothing is stored on the parameter). The conv
weight gradients -- all but ~1 % of the 43M trainable values -- are written by their wgrad kernels
straight into their slot (conv.grad_dest: the conv backward hands AccumulateGrad a view of the slot,
which it adopts as `.grad`; inside the captured backward graphs the slot is the graph's own gradient
buffer), so the all-reduce runs on the gradients in place: no flatten copy in, no unflatten copy out.
A gradient that arrives elsewhere (BatchNorm affine, biases, the RPN head's weights summed over five
levels, a parameter unused on this rank) is copied into its slot (one multi-tensor launch per group)
and the parameter's `.grad` becomes the slot view. Over RCCL the average is `ReduceOp.AVG` (ncclAvg:
no separate 1/N pass); gloo has no AVG, so it sums and scales. In a one-rank group the average is the
sum (RCCL's in-place one-rank sum moves no data, where its AVG rewrites every bucket: ~0.3 ms per
step), unless one_rank_sum=False.

Failing together: a rank whose proposal NMS reports a failure (RegionProposalNetwork.check_nms,
num_keep < 0) must not raise alone -- the other ranks would block in the next all-reduce until the
RCCL timeout. Under this wrapper the RPN records the failure instead (`_mx_defer_nms_error`); the
first all-reduce of every step carries one extra float, this rank's failure flag, and
`sync_gradients()` reads the reduced flag (a wait on that first collective only, long finished by
then) and raises on every rank before the optimizer step, with the local message where there is one.
"""
import torch
import torch.distributed as dist


def _slot_view(flat, off, p):
    return flat.narrow(0, off, p.numel()).view(p.shape)


def _in_slot(g, ptr):
    """True when gradient g already IS its parameter's slot, the one starting at address `ptr` of a
    persistent flat bucket. Only conv.grad_dest hands out tensors at a slot address, and always the
    dense slot view of the parameter's shape, so the address alone decides (the check runs per
    parameter in the backward hooks and at sync: it must stay ~1 us, not a chain of tensor queries)."""
    return g is not None and g.data_ptr() == ptr


class DataParallel:
    def __init__(self, model, bucket_mb=64, group=None, one_rank_sum=True):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group)
        with torch.no_grad():
            for t in list(model.parameters()) + list(model.buffers()):
                dist.broadcast(t.data, 0, group=group)
        self.params = [p for p in model.parameters() if p.requires_grad]
        self._work = {}  # key -> (work, key) started from a graph hand-off hook
        # the RoI head's gradients are complete as soon as its backward graph has replayed, before
        # the trunk's (most of the step's backward): their all-reduce starts right then and overlaps
        # the trunk backward (hook fired by frcnn._Graphs; without it they join the normal buckets)
        rh = getattr(model, "roi_heads", None)
        early = {id(p) for p in rh.parameters() if p.requires_grad} if rh is not None else set()
        self.early = [p for p in self.params if id(p) in early]
        if self.early:
            rh.__dict__["_mx_grads_ready"] = self._early_reduce
        # trunk segments (frcnn._SegGraphs keys): started from the segmented backward graphs' hook
        self.segments = {}
        if hasattr(model, "backbone") and hasattr(model, "rpn"):
            body = model.backbone.body
            seg = {"fpn+rpn_head": list(model.backbone.fpn.parameters()) + list(model.rpn.head.parameters()),
                   "layer4": list(body.layer4.parameters()), "layer3": list(body.layer3.parameters()),
                   "layer2": list(body.layer2.parameters()),
                   "stem+layer1": list(body.conv1.parameters()) + list(body.bn1.parameters()) +
                   list(body.layer1.parameters())}
            self.segments = {k: [p for p in v if p.requires_grad] for k, v in seg.items()}
            self.segments = {k: v for k, v in self.segments.items() if v}
            model.__dict__["_mx_seg_ready"] = self._segment_reduce
        seen = early | {id(p) for v in self.segments.values() for p in v}
        rest = [p for p in self.params if id(p) not in seen]
        # the canonical issue order of the hook-startable groups (backward order)
        self.groups = ([("roi_heads", self.early)] if self.early else []) + list(self.segments.items())
        self.issued, self.last_issued = [], []  # keys in issue order: this step's, the last synced step's
        # buckets in reverse registration order (the backward produces the later layers' first)
        self.buckets, cur, size = [], [], 0
        for p in reversed(rest):
            cur.append(p)
            size += p.numel() * 4
            if size >= bucket_mb * 2 ** 20:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self.bucket_mb = bucket_mb
        # persistent flat buffer per group / bucket, a fixed slot per parameter (module docstring); the
        # first collective of the step (canonical order) carries the NMS failure flag after its slots
        from . import conv as _conv
        self._slots = _conv.grad_slots
        units = self.groups + [(("bucket", i), b) for i, b in enumerate(self.buckets)]
        self.flag_key = units[0][0] if units else None
        self.flats = {}
        for key, ps in units:
            if any(p.dtype != torch.float32 for p in ps) or len({p.device for p in ps}) != 1:
                raise RuntimeError("DataParallel: trainable parameters must be f32 on one device per group")
            n = sum(p.numel() for p in ps)
            flat = torch.zeros(n + (key == self.flag_key), dtype=torch.float32, device=ps[0].device)
            slots, off = [], 0
            for p in ps:
                self._slots[p] = (flat, off)
                slots.append((p, off, flat.data_ptr() + 4 * off))
                off += p.numel()
            self.flats[key] = (flat, slots)
        self._adopt = {}  # key -> [(p, off)] whose .grad becomes its slot view at sync (not in slot at _start)
        self._flag_host = None
        self.rpn = getattr(model, "rpn", None)
        if self.rpn is not None:
            self.rpn.__dict__["_mx_defer_nms_error"] = True
        self.op, self.scale = dist.ReduceOp.SUM, 1.0 / self.world
        if dist.get_backend(group) == "nccl":  # RCCL: ncclAvg, the 1/N folded into the reduction
            self.op, self.scale = dist.ReduceOp.AVG, None
        if self.world == 1 and one_rank_sum:  # one rank's average is its sum: in place, RCCL moves no data
            self.op, self.scale = dist.ReduceOp.SUM, None
        self.copied = 0  # gradients copied into their slot in the last synced step (diagnostics)
        self._copied = 0
        for m in model.modules():  # graphs and side-stream wgrad stay enabled under this wrapper
            m.__dict__["_mx_dp"] = True
        _conv.set_data_parallel(True)

    def close(self):
        """Drop this wrapper's gradient slots (conv.grad_slots) and hooks; `.grad`s keep their views."""
        for flat, slots in self.flats.values():
            for p, _, _ in slots:
                cur = self._slots.get(p)
                if cur is not None and cur[0] is flat:
                    del self._slots[p]
        for m, k in ((getattr(self.model, "roi_heads", None), "_mx_grads_ready"), (self.model, "_mx_seg_ready"),
                     (self.rpn, "_mx_defer_nms_error")):
            if m is not None:
                m.__dict__.pop(k, None)

    def __call__(self, *args, **kwargs):
        return self.model(*args, **kwargs)

    def train(self, mode=True):
        self.model.train(mode)
        return self

    def eval(self):
        self.model.eval()
        return self

    @torch.no_grad()
    def _start(self, key):
        """Gather group `key`'s gradients into its flat buffer (only those not already written into
        their slot) and start its all-reduce."""
        flat, slots = self.flats[key]
        src, dst, zero, adopt = [], [], [], []
        for p, off, ptr in slots:
            g = p.grad
            if g is None:
                zero.append(_slot_view(flat, off, p))
                adopt.append((p, off))
            elif not _in_slot(g, ptr):
                src.append(g)
                dst.append(_slot_view(flat, off, p))
                adopt.append((p, off))
        self._adopt[key] = adopt
        if zero:
            torch._foreach_zero_(zero)
        if src:
            torch._foreach_copy_(dst, src)
        self._copied += len(src)
        if key == self.flag_key:  # this rank's proposal-NMS failure flag rides in the first collective
            flat[-1].fill_(1.0 if self.rpn is not None and self.rpn.__dict__.get("_nms_error") else 0.0)
        return dist.all_reduce(flat, op=self.op, group=self.group, async_op=True), key

    def _issue_through(self, key):
        """Start, in canonical order, every group up to and including `key` not yet started."""
        if key not in dict(self.groups):
            return
        for k, _ in self.groups:
            if k not in self._work:
                self._work[k] = self._start(k)
                self.issued.append(k)
            if k == key:
                return

    def _early_reduce(self):
        """frcnn._Graphs hand-off of the RoI head (first in canonical order)."""
        self._issue_through("roi_heads")

    def _segment_reduce(self, key, params):
        """frcnn._SegGraphs hand-off: `params`' gradients are final for this backward, and so are those
        of every group before `key` in canonical order."""
        self._issue_through(key)

    @torch.no_grad()
    def sync_gradients(self):
        """Average the trainable gradients over all ranks (call after backward, before step). A
        parameter without a gradient on this rank contributes zeros (and gets the average).
        Every rank issues the all-reduces in the same canonical order (module docstring), whichever
        of them its hooks started. Afterwards every trainable `.grad` is its bucket slot."""
        if self.groups:
            self._issue_through(self.groups[-1][0])  # whatever no hook started, in canonical order
        started = self._work
        self._work = {}
        pending = [started[k] for k, _ in self.groups]
        for i in range(len(self.buckets)):
            pending.append(self._start(("bucket", i)))
            self.issued.append("bucket")
        for work, key in pending:
            work.wait()
            flat, _ = self.flats[key]
            if self.scale is not None:
                flat.mul_(self.scale)
        # the host work after the last collective is issued stays short (the GPU drains meanwhile): the
        # flag read waits on the first collective only; only gradients _start found outside their slot
        # are re-pointed
        if pending:
            self._check_flag(*pending[0])
        for _, key in pending:
            flat, _ = self.flats[key]
            for p, off in self._adopt.pop(key, ()):
                p.grad = _slot_view(flat, off, p)
        self.last_issued, self.issued = self.issued, []
        self.copied, self._copied = self._copied, 0

    def _check_flag(self, work, key):
        """Read the reduced NMS failure flag of the step's first collective (module docstring) and
        raise on every rank if any rank failed. The read waits for that collective only (on a stream
        of its own), not for the rest of the backward."""
        flat, _ = self.flats[key]
        local = self.rpn.__dict__.pop("_nms_error", None) if self.rpn is not None else None
        if flat.is_cuda:
            if self._flag_host is None:
                self._flag_host = torch.zeros((), dtype=torch.float32, pin_memory=True)
                from . import conv as _conv
                # high priority: on a stream sharing a hardware queue with the backward the 4-B copy
                # waited for the whole trunk backward (~4.6 ms of host block, tools/dp_host_timeline.py)
                self._flag_stream = _conv.dedicated_stream(flat.device, "dp_flag", high_priority=True)
            with torch.cuda.stream(self._flag_stream):
                work.wait()
                self._flag_host.copy_(flat[-1], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
            ev.synchronize()
            bad = float(self._flag_host)
        else:
            work.wait()
            bad = float(flat[-1])
        if bad != 0.0:
            raise RuntimeError("DataParallel: the proposal NMS failed on at least one rank this step; no rank "
                               "applies it" + (f" (this rank: {local})" if local else ""))
