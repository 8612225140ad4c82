"""Data-parallel training over RCCL that keeps the HIP-graph replays.

torch DistributedDataParallel launches its bucket all-reduces from AccumulateGrad hooks; the
replayed trunk / RoI-head backward graphs write their parameters' gradients directly and bypass
those hooks, so under DDP the model had to run eagerly (24 ms instead of 18 ms per step on one
MI355X). `DataParallel` gives the same semantics as the DDP configuration the reference-style
scripts use (DistributedDataParallel(broadcast_buffers=False)):
  * identical start: parameters and buffers broadcast from rank 0;
  * per-GPU BatchNorm statistics (buffers are never synchronised afterwards);
  * gradients averaged over ranks before the optimizer step
while the graphs stay on: after `loss.backward()` the trainable gradients are averaged by a few
large flat all-reduces (one per ~`bucket_mb` of gradients, issued back to back on RCCL's stream,
then scaled and scattered back with one multi-tensor copy each). The exchange is not overlapped
with the backward (the trunk's gradients all appear when its graph finishes); over xGMI a ring
all-reduce of the 172 MB of f32 gradients costs ~2·(N-1)/N·172 MB / bus bandwidth.
"""
import torch
import torch.distributed as dist
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

from . import conv as _conv


class DataParallel:
    def __init__(self, model, bucket_mb=64, group=None):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group)
        with torch.no_grad():
            for t in list(model.parameters()) + list(model.buffers()):
                dist.broadcast(t.data, 0, group=group)
        self.params = [p for p in model.parameters() if p.requires_grad]
        # the RoI head's gradients are complete as soon as its backward graph has replayed, before
        # the trunk's (most of the step's backward): their all-reduce starts right then and overlaps
        # the trunk backward (hook fired by frcnn._Graphs; without it they join the normal buckets)
        rh = getattr(model, "roi_heads", None)
        early = {id(p) for p in rh.parameters() if p.requires_grad} if rh is not None else set()
        self.early = [p for p in self.params if id(p) in early]
        self._early_work = None
        if self.early:
            rh.__dict__["_mx_grads_ready"] = self._early_reduce
        rest = [p for p in self.params if id(p) not in early]
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
        for m in model.modules():  # graphs and side-stream wgrad stay enabled under this wrapper
            m.__dict__["_mx_dp"] = True
        _conv.set_data_parallel(True)

    def __call__(self, *args, **kwargs):
        return self.model(*args, **kwargs)

    def train(self, mode=True):
        self.model.train(mode)
        return self

    def eval(self):
        self.model.eval()
        return self

    @torch.no_grad()
    def _start(self, params):
        grads = []
        for p in params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            grads.append(p.grad)
        flat = _flatten_dense_tensors(grads)
        return dist.all_reduce(flat, group=self.group, async_op=True), flat, grads

    def _early_reduce(self):
        if self._early_work is None:
            self._early_work = self._start(self.early)

    @torch.no_grad()
    def sync_gradients(self):
        """Average the trainable gradients over all ranks (call after backward, before step). A
        parameter without a gradient on this rank contributes zeros (and gets the average)."""
        pending = []
        if self.early:
            pending.append(self._early_work if self._early_work is not None else self._start(self.early))
            self._early_work = None
        for b in self.buckets:
            pending.append(self._start(b))
        for work, flat, grads in pending:
            work.wait()
            flat.mul_(1.0 / self.world)
            torch._foreach_copy_(grads, _unflatten_dense_tensors(flat, grads))
