"""Debug helper: GPU guided filter vs the oracle on one configuration; prints where they differ.
Usage: python tools/dbg_gf.py NZ NY NX CZ CY CX EPS R [seed]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import zarrs_tools_amd as zt
from oracle import oracle as O

a = sys.argv[1:]
shape = tuple(int(x) for x in a[0:3])
chunk = tuple(int(x) for x in a[3:6])
eps, r = float(a[6]), int(a[7])
seed = int(a[8]) if len(a) > 8 else 0
rng = np.random.default_rng(seed)
v = (rng.random(shape, dtype=np.float32) * 300).astype(np.float32)
ref = O.guided_filter_apply(v, chunk, eps, r, nthreads=8)
x = torch.from_numpy(v).cuda()
y = torch.empty_like(x)
zt.GuidedFilter(eps, r).apply(zt.DeviceArray(x, chunk), zt.DeviceArray(y, chunk))
torch.cuda.synchronize()
out = y.cpu().numpy()
err = np.abs(out.astype(np.float64) - ref) / np.maximum(1.0, np.abs(ref))
bad = err > 1e-5
print("shape", shape, "chunk", chunk, "eps", eps, "r", r, "max err", err.max(), "bad", bad.sum(),
      "of", bad.size)
if bad.any():
    idx = np.argwhere(bad)
    for ax, name in enumerate("zyx"):
        vals, cnt = np.unique(idx[:, ax], return_counts=True)
        print(f"  bad {name}:", dict(zip(vals.tolist()[:40], cnt.tolist()[:40])))
    for p in idx[:8]:
        p = tuple(p)
        print("  ", p, "gpu", out[p], "ref", ref[p], "v", v[p])
