"""Probe: HIP graph capture with streams forked and joined repeatedly (the level lanes).
mode 'pre' / 'in': lane streams created before / inside the capture, one parent;
'nest': P parents (the main stream + P-1 side streams forked from it, as the posterior net
and past decoder are), each forking its own nl lanes per level."""
import sys
import torch
mode = sys.argv[1]
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 3
levels = int(sys.argv[3]) if len(sys.argv) > 3 else 50
npar = int(sys.argv[4]) if len(sys.argv) > 4 else 1
with_lanes = [int(v) for v in sys.argv[5].split(",")] if len(sys.argv) > 5 else list(range(npar))
dev = torch.device("cuda", 0)
xs = [torch.ones(1 << 16, device=dev) for _ in range((nl + 1) * npar)]
lanes = {}
def lane(p, k):
    s = lanes.get((p, k))
    if s is None:
        s = lanes[(p, k)] = torch.cuda.Stream(device=dev)
    return s
if mode != "in":
    for p in range(npar):
        for k in range(0 if p else 1, nl + 1):
            lane(p, k)
def level(p, cur):
    base = p * (nl + 1)
    if p not in with_lanes:
        xs[base].add_(1.0)
        return
    for k in range(1, nl + 1):
        lane(p, k).wait_stream(cur)
    xs[base].add_(1.0)
    for k in range(1, nl + 1):
        with torch.cuda.stream(lane(p, k)):
            xs[base + k].add_(float(k))
    for k in range(1, nl + 1):
        cur.wait_stream(lane(p, k))
def step():
    main = torch.cuda.current_stream()
    pars = [main] + [lane(p, 0) for p in range(1, npar)]
    for p in range(1, npar):
        pars[p].wait_stream(main)
    for lv in range(levels):
        for p in range(npar):
            with torch.cuda.stream(pars[p]):
                level(p, pars[p])
    for p in range(1, npar):
        main.wait_stream(pars[p])
g = torch.cuda.CUDAGraph()
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    step()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
print("eager ok", flush=True)
with torch.cuda.graph(g):
    step()
print("captured", mode, nl, levels, npar, flush=True)
g.replay(); torch.cuda.synchronize()
print("replayed", float(xs[1][0]), flush=True)
