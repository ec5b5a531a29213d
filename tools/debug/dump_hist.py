"""Dump the device histogram of the bench stream (first N bytes, seed 42) to a
.npy file under gpurun_out/ (for host-side table experiments at full scale).
usage: python tools/debug/dump_hist.py BYTES zipf|uniform OUT"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from huffman_amd.pipeline import StreamCodec

n = int(sys.argv[1])
kind = 0 if sys.argv[2] == "uniform" else 1
c = StreamCodec(0)
x = torch.empty(n, dtype=torch.uint8, device="cuda")
c.dev.generate(x.data_ptr(), n, offset=0, kind=kind, alpha=1.1, seed=42)
c.histogram(x)
np.save(sys.argv[3], c.hist.cpu().numpy().view(np.uint64))
