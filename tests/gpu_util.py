"""Helpers shared by the -m gpu tests: host<->device transfer of any Zarr element type."""
import numpy as np

from oracle import oracle as O


def to_dev(a: np.ndarray, dtype: str):
    import torch
    from zarrs_tools_amd import torch_dtype
    a = np.ascontiguousarray(a, dtype=O.NP_STORAGE[dtype])
    if a.size == 0:
        return torch.empty(a.shape, dtype=torch_dtype(dtype), device="cuda")
    flat = torch.from_numpy(a.reshape(-1).view(np.uint8).copy()).cuda()
    return flat.view(torch_dtype(dtype)).reshape(a.shape)


def from_dev(t, dtype: str) -> np.ndarray:
    import torch
    shape = tuple(t.shape)
    if t.numel() == 0:
        return np.zeros(shape, dtype=O.NP_STORAGE[dtype])
    b = t.contiguous().reshape(-1).view(torch.uint8).cpu().numpy()
    return b.view(O.NP_STORAGE[dtype]).reshape(shape)


def rel_err(out: np.ndarray, ref: np.ndarray) -> float:
    out = out.astype(np.float64)
    ref = ref.astype(np.float64)
    if out.size == 0:
        return 0.0
    return float(np.max(np.abs(out - ref) / np.maximum(1.0, np.abs(ref))))


# Float tolerance (stated in DESIGN.md §5): |gpu - ref| <= 1e-5 * max(1, |ref|). The GPU sums
# box windows in f32 (fixed tree order); the reference in f64 through summed-area tables.
FLOAT_TOL = 1e-5
