"""``zarrs_ome`` for the accelerated path: an OME-Zarr (v0.5) multiscale group from a Zarr V3
array, every level computed by the HIP downsample kernel over the store.

    python -m zarrs_tools_amd.zarrs_ome INPUT OUTPUT [FACTOR,...] [--max-levels N] [--discrete]
        [--gaussian-sigma S,...] [--gaussian-kernel-half-size H,...] [--device D]
        [--chunk-limit N] [--name NAME]

Follows src/bin/zarrs_ome.rs (0.7.2): level 0 is a copy of the input (:341-366, no reencoding);
level i is the downsample of level i-1 read back from the output (:515-738) with the output chunk
shape min(input chunk, output shape) (:549-559); the loop stops when every axis has factor 1 or
extent 1 (:731-737); each level adds a multiscales dataset with scale = the cumulative factor and
translation (scale - 1) / 2 (:716-726). Mean downsampling, the mode with --discrete (ties by
the smallest value: the documented deviation), or with --gaussian-sigma a Gaussian
of each level's input before the mean (apply_chunk_continuous_gaussian, :236-271; kernel half
size default ceil(3 sigma), :494-502; ignored with --discrete, :638-646). The multiscales
"type" is "mode", "average" or "gaussian" (:468-475); axes are named by the array's dimension
names, else by index (:431-449).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import shutil
import sys
import time

import numpy as np

from . import _abi
from . import store as S


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="zarrs_ome")
    ap.add_argument("input")
    ap.add_argument("output")
    ap.add_argument("factor", nargs="?", default=None,
                    type=lambda s: [int(x) for x in s.split(",")])
    ap.add_argument("--max-levels", type=int, default=10)
    ap.add_argument("--discrete", action="store_true")
    ap.add_argument("--gaussian-sigma", default=None,
                    type=lambda s: [float(x) for x in s.split(",")])
    ap.add_argument("--gaussian-kernel-half-size", default=None,
                    type=lambda s: [int(x) for x in s.split(",")])
    ap.add_argument("--name", default=None)
    ap.add_argument("--exists", choices=["erase", "exit"], default="erase")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--chunk-limit", type=int, default=0)
    return ap


def level_scale(scale, in_shape, out_shape):
    """relative_scale *= (input / output) as f32 per axis (zarrs_ome.rs:570-578)."""
    f32 = np.float32
    return [float(f32(f32(s) * f32(int(i) // int(o)))) for s, i, o in
            zip(scale, in_shape, out_shape)]


def level_translation(scale):
    """(s - 1.0) * 0.5 in f32 (zarrs_ome.rs:721-723)."""
    f32 = np.float32
    return [float(f32(f32(f32(s) - f32(1.0)) * f32(0.5))) for s in scale]


def run(input_path, output_path, factor=None, max_levels: int = 10, discrete: bool = False,
        name=None, exists: str = "erase", device: int = 0, nthreads: int = 0,
        gaussian_sigma=None, gaussian_kernel_half_size=None, log=print) -> dict:
    t0 = time.perf_counter()
    info = S.open_array(input_path)
    nd = info.ndim
    factor = [2] * nd if factor is None else [int(f) for f in factor]
    if len(factor) != nd:
        raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                     "downsample factor must match the array rank")
    gauss = None
    if gaussian_sigma is not None and not discrete:
        sigma = [float(s) for s in gaussian_sigma]
        half = ([int(h) for h in gaussian_kernel_half_size] if gaussian_kernel_half_size
                else [int(math.ceil(s * 3.0)) for s in sigma])
        if len(sigma) != nd or len(half) != nd:
            raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                         "gaussian sigma / kernel half size must match the rank")
        gauss = (sigma, half)
    if os.path.exists(output_path):
        if exists == "exit":
            raise _abi.FilterError(_abi.ERR_OTHER, f"output {output_path} already exists")
        shutil.rmtree(output_path)
    os.makedirs(output_path)
    shutil.copytree(input_path, os.path.join(output_path, "0"))
    log(f"0: copy {input_path} -> {output_path}/0 ({info.data_type} {list(info.shape)})")
    scale = [1.0] * nd
    datasets = [{"path": "0", "coordinateTransformations": [
        {"type": "scale", "scale": list(scale)}]}]
    shape = list(info.shape)
    stats = []
    for i in range(1, max_levels + 1):
        src, dst = os.path.join(output_path, str(i - 1)), os.path.join(output_path, str(i))
        if gauss is not None:
            st = S.downsample_gaussian(src, dst, factor, gauss[0], gauss[1], device=device,
                                       nthreads=nthreads)
        else:
            st = S.downsample(src, dst, factor, discrete=discrete, device=device,
                              nthreads=nthreads)
        stats.append(st)
        out = S.open_array(dst)
        # zarrs_ome.rs:570-578: the real factor is input_shape / output_shape (integer division),
        # accumulated into an f32 scale; translation (s - 1) * 0.5 in f32 (:716-723)
        scale = level_scale(scale, shape, out.shape)
        datasets.append({"path": str(i), "coordinateTransformations": [
            {"type": "scale", "scale": list(scale)},
            {"type": "translation", "translation": level_translation(scale)}]})
        log(f"{i}: {list(shape)} -> {list(out.shape)} in {st['wall_s']:.2f}s")
        shape = list(out.shape)
        if all(f == 1 or s == 1 for f, s in zip(factor, shape)):
            break
    names = info.dimension_names if getattr(info, "dimension_names", None) else None
    axes = [{"name": (names[k] if names and names[k] is not None else str(k))}
            for k in range(nd)]
    group = {"zarr_format": 3, "node_type": "group", "attributes": {"ome": {
        "version": "0.5",
        "multiscales": [{"name": name or os.path.basename(os.path.normpath(input_path)),
                         "axes": axes, "datasets": datasets,
                         "type": "mode" if discrete else ("average" if gauss is None
                                                          else "gaussian"),
                         "metadata": {"description": "Created with zarrs_tools_amd zarrs_ome",
                                      "kwargs": {"factor": factor, "discrete": discrete,
                                                 "gaussian_sigma": None if gauss is None
                                                 else gauss[0]}}}]}}}
    with open(os.path.join(output_path, "zarr.json"), "w") as f:
        json.dump(group, f, indent=2)
    log(f"Output {output_path} in {time.perf_counter() - t0:.2f}s")
    return {"levels": len(stats), "stats": stats}


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    try:
        run(a.input, a.output, a.factor, a.max_levels, a.discrete, a.name, a.exists, a.device,
            a.chunk_limit, a.gaussian_sigma, a.gaussian_kernel_half_size)
    except _abi.FilterError as e:
        print(f"Error: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
