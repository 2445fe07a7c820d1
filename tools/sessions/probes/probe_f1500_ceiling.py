import json, os, sys
import numpy as np, torch
ROOT = "/root/repo" if os.path.exists("/root/repo") else os.getcwd()
sys.path.insert(0, ROOT)
from tulips_amd import csum
import bench
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream()
timer = bench.Timer(torch, stream)
NB, SEG, NSEG = 16, 1500, 65536
bb = NSEG * SEG
arena = torch.empty(NB * bb + 256, dtype=torch.uint8, device=dev)
csum.fill_splitmix(arena, NB * bb)
out = torch.empty(NB * NSEG, dtype=torch.uint16, device=dev)
sink = torch.zeros(1024, dtype=torch.int32, device=dev)
def fr(i, st):
    b = i % NB
    csum.lib.tulips_csum_stream_read(arena.data_ptr() + b * bb, bb, sink.data_ptr(), 0, st)
def ff(i, st):
    b = i % NB
    csum.lib.tulips_csum_batch_fixed(arena.data_ptr() + b * bb, SEG, SEG, None, None, None, out.data_ptr() + b * NSEG * 2, NSEG, 0, st)
row = {}
for name, fn in (("stream_read_98MB", fr), ("F1500", ff)):
    for i in range(NB): fn(i, stream.cuda_stream)
    ts = float(np.median([timer(fn, 64) for _ in range(3)]))
    tp = float(np.median([timer(fn, 64, branches=4) for _ in range(3)]))
    row[name] = [round(ts * 1e6, 2), round(tp * 1e6, 2), round(bb / ts / 8e12, 4), round(bb / tp / 8e12, 4)]
print(json.dumps(row))
