"""Probe: does the NCCL flight recorder show when the watchdog retires eager works?
World-1 RCCL group; a few async all-reduces; synchronize; dump the FR at intervals."""
import os, pickle, time, sys
os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
os.environ.setdefault("TORCH_NCCL_TRACE_BUFFER_SIZE", "2000")
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29731")
import torch, torch.distributed as dist
import torch._C._distributed_c10d as c10d
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1)
pg = dist.group.WORLD
print("pg name", pg.group_name, "seq", pg._get_backend(torch.device("cuda"))._get_sequence_number_for_group(), flush=True)
x = torch.ones(1 << 20, device="cuda")
ws = [dist.all_reduce(x, async_op=True) for _ in range(5)]
for w in ws:
    w.wait()
torch.cuda.synchronize()
del ws
def dump():
    d = pickle.loads(c10d._dump_nccl_trace(True, False, False))
    return d
d = dump()
print("top keys", sorted(d.keys()), flush=True)
ents = d.get("entries", [])
print("n entries", len(ents), flush=True)
if ents:
    print("entry keys", sorted(ents[0].keys()), flush=True)
    print({k: ents[0][k] for k in ents[0] if k not in ("frames", "input_sizes", "output_sizes")}, flush=True)
t0 = time.time()
for k in range(12):
    d = dump()
    ents = d.get("entries", [])
    print(f"t={time.time()-t0:.3f}s retired={[e.get('retired') for e in ents]} state={[e.get('state') for e in ents]}", flush=True)
    time.sleep(0.02)
# capture one all-reduce, then see the captured entry
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, capture_error_mode="thread_local"):
    dist.all_reduce(x)
print("seq after capture", pg._get_backend(torch.device("cuda"))._get_sequence_number_for_group(), flush=True)
g.replay(); torch.cuda.synchronize()
time.sleep(0.3)
d = dump()
ents = d.get("entries", [])
print("after capture:", [(e.get('record_id'), e.get('collective_seq_id'), e.get('retired'), e.get('state'), e.get('process_group')) for e in ents], flush=True)
dist.destroy_process_group()
print("done", flush=True)
