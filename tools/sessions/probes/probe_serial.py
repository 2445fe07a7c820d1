import sys, os
sys.path.insert(0, "/root/repo")
import torch, numpy as np
import bench
from tulips_amd import csum
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream()
NB, SEG, NSEG = 16, 1500, 65536
bb = NSEG * SEG
arena = torch.empty(NB * bb + 256, dtype=torch.uint8, device=dev)
csum.fill_splitmix(arena, NB * bb)
outs = torch.empty(NB * NSEG, dtype=torch.uint16, device=dev)
fixed = csum.lib.tulips_csum_batch_fixed
def f(i, s):
    b = i % NB
    fixed(arena.data_ptr() + b * bb, SEG, SEG, None, None, None, outs.data_ptr() + b * NSEG * 2, NSEG, 0, s)
T = bench.Timer(torch, st)
for rep in range(2):
    for reps, br in ((512, 1), (1024, 1), (64, 1), (512, 4), (512, 1)):
        t = T(f, reps, branches=br)
        print(rep, reps, br, round(t * 1e6, 3), flush=True)
