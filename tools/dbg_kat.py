import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import zarrs_tools_amd as zt
from oracle import oracle as O
v = np.array([[i + j for j in range(4)] for i in range(4)], dtype=np.float32)
x = torch.from_numpy(v).cuda()
g = zt.GuidedFilter(1.0, 2)
whole = g.apply_ndarray(x)
torch.cuda.synchronize()
print("whole\n", whole.cpu().numpy())
for sub in [((0, 0), (2, 2)), ((0, 2), (2, 2)), ((2, 0), (2, 2)), ((2, 2), (2, 2))]:
    r = g.apply_ndarray(x, zt.ArraySubset(*sub))
    torch.cuda.synchronize()
    print(sub, "\n", r.cpu().numpy())
blk = x[0:4, 2:4]
r = g.apply_ndarray(blk)
torch.cuda.synchronize()
print("view block cols 2:4 (stride", blk.stride(), ")\n", r.cpu().numpy())
print("oracle", O.guided_filter_apply_ndarray(v[:, 2:4].copy(), 1.0, 2))
