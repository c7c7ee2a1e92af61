"""Node list (type, kernel, deps) of the pipelined C3 step graph, to read which nodes the decoder
branch's first kernels wait for (GPU box):
    python tools/probe/pipe_graph.py [C3] > gpurun_out/pipe_graph.txt"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import graph_nodes  # noqa: E402
from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer  # noqa: E402

cfgname = sys.argv[1] if len(sys.argv) > 1 else "C3"
cfg = bench.CONFIGS[cfgname]
dev = torch.device("cuda:0")
kept = []
base = torch.cuda.CUDAGraph


class Kept(base):
    def __new__(cls, keep_graph=False):
        g = base.__new__(cls, True)
        kept.append(g)
        return g

    def __init__(self, keep_graph=False):
        super().__init__(True)


torch.cuda.CUDAGraph = Kept
enc, dec = bench.build(cfg, dev)
tr = TeacherForcedTrainer(enc, dec, lstm=cfg["decoder"] == "lstm", graph=True, pipeline=True)
for i in range(3):
    b = bench.synthetic_batch(cfg["batch"], 0, i, dev)
    tr.step(*b)
torch.cuda.synchronize()
for gi, g in enumerate(kept):
    print(f"=== graph {gi}")
    for line in graph_nodes.describe(g.raw_cuda_graph()):
        print(line)
