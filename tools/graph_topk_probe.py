"""Probe: torch.topk over RPN-sized rows captured in a HIP graph and replayed on fresh inputs, against
eager (the per-level top-k the proposal chain used before mx_level_topk). Prints per-replay equality."""
import torch

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
levels = [201600, 50400, 12600, 3150, 819]
x = torch.randn(2, sum(levels), device=dev, generator=g)


def chain(v):
    outs, o = [], 0
    for n in levels:
        outs.append(v[:, o:o + n].topk(min(2000, n), dim=1)[1] + o)
        o += n
    return torch.cat(outs, 1)


side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(2):
        chain(x)
torch.cuda.current_stream().wait_stream(side)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    out = chain(x)
for i in range(3):
    x.copy_(torch.randn(2, sum(levels), device=dev, generator=g))
    graph.replay()
    ref = chain(x)
    torch.cuda.synchronize()
    print(f"replay {i}: equal indices {torch.equal(out, ref)}; equal as sets "
          f"{torch.equal(out.sort(1)[0], ref.sort(1)[0])}", flush=True)
