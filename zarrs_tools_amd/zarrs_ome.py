"""``zarrs_ome`` for the accelerated path: an OME-Zarr (v0.5) multiscale group from a Zarr V3
array, every level computed by the HIP downsample kernel over the store.

    python -m zarrs_tools_amd.zarrs_ome INPUT OUTPUT [FACTOR,...] [--max-levels N] [--discrete]
        [--gaussian-sigma S,...] [--gaussian-kernel-half-size H,...] [--physical-size P,...]
        [--physical-units U,...] [--name NAME] [--group-attributes JSON]
        [--exists erase|exit|overwrite] [--ome-zarr-version 0.5] [reencoding args]
        [--device D] [--chunk-limit N]

Follows src/bin/zarrs_ome.rs (0.7.2):
* the output group gets --group-attributes (:317-323); --exists erase / exit / overwrite (:326-339);
* level 0 is a copy of the input, or with any reencoding argument (ZarrReencodingArgs,
  lib.rs:274-377) the input reencoded into the new encoding (:341-366);
* array 0's attributes move to the group, without "_zarrs" (:368-377);
* level i is the downsample of level i-1 (:515-738): read back from the output store as the
  reference does, or — when level 0 and its pyramid fit 80 % of the free device memory
  (`--no-device-resident` turns it off) — computed from the previous level kept in HBM, level 0
  read once and every level written once (the same kernels, so the same bits). Its encoding is the
  input's with zarrs_ome's per-level shapes (:528-560): a sharded input gets the shard shape
  min(shard, output) and the inner chunk min(inner chunk, output); otherwise the chunk shape
  min(chunk, output), which get_array_builder_reencode applies only to sharded outputs
  (lib.rs:623-646), so an unsharded level keeps the input's chunk grid. The loop stops when every
  axis has factor 1 or extent 1 (:731-737);
* each level adds a dataset with the cumulative f32 scale of input/output shape ratios and
  translation (scale - 1) / 2 (:570-578, :716-726);
* axes are named by the array's dimension names, else by index, typed by --physical-units (space,
  time, "channel", or a custom unit, :379-446); --physical-size is the multiscale's
  coordinateTransformations (:448-452); the multiscales "type" is "mode", "average" or "gaussian"
  (:468-475).
Mean downsampling, the mode with --discrete (ties by the smallest value: the documented deviation,
DESIGN.md §2), or with --gaussian-sigma a Gaussian of each level's input before the mean
(apply_chunk_continuous_gaussian, :236-271; kernel half size default ceil(3 sigma), :494-502;
ignored with --discrete, :638-646).
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
from .zarrs_filter import (REENCODE_KEYS, _add_reencode_args, _device_ok, encoding_of,
                           read_to_device, write_from_device)

VERSION = "zarrs_tools_amd 0.2 (MI355X)"

# OME-NGFF 0.5 units (ome_zarr_metadata 0.2.3 AxisUnit: Space | Time | Custom)
SPACE_UNITS = {
    "angstrom", "attometer", "centimeter", "decimeter", "exameter", "femtometer", "foot",
    "gigameter", "hectometer", "inch", "kilometer", "megameter", "meter", "micrometer", "mile",
    "millimeter", "nanometer", "parsec", "petameter", "picometer", "terameter", "yard",
    "yoctometer", "yottameter", "zeptometer", "zettameter"}
TIME_UNITS = {
    "attosecond", "centisecond", "day", "decisecond", "exasecond", "femtosecond", "gigasecond",
    "hectosecond", "hour", "kilosecond", "megasecond", "microsecond", "millisecond", "minute",
    "nanosecond", "petasecond", "picosecond", "second", "terasecond", "yoctosecond",
    "yottasecond", "zeptosecond", "zettasecond"}


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="zarrs_ome")
    ap.add_argument("input")
    ap.add_argument("output")
    ap.add_argument("factor", nargs="?", default=None,
                    type=lambda s: [int(x) for x in s.split(",")])
    ap.add_argument("--ome-zarr-version", default="0.5", choices=["0.5"])
    ap.add_argument("--max-levels", type=int, default=10)
    ap.add_argument("--physical-size", default=None,
                    type=lambda s: [float(x) for x in s.split(",")])
    ap.add_argument("--physical-units", default=None, type=lambda s: s.split(","))
    ap.add_argument("--discrete", action="store_true")
    ap.add_argument("--gaussian-sigma", default=None,
                    type=lambda s: [float(x) for x in s.split(",")])
    ap.add_argument("--gaussian-kernel-half-size", default=None,
                    type=lambda s: [int(x) for x in s.split(",")])
    ap.add_argument("--name", default=None)
    ap.add_argument("--group-attributes", default=None)
    ap.add_argument("--exists", choices=["erase", "exit", "overwrite"], default="erase")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--no-device-resident", action="store_true",
                    help="read every level back from the store (the reference's loop)")
    _add_reencode_args(ap)  # adds --chunk-limit too
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


def level_encoding(info: "S.ArrayInfo", out_shape) -> dict:
    """zarrs_ome.rs:528-560: the per-level chunk (and shard) shape of level i from level i-1."""
    if info.chunk_shape != info.inner_chunk_shape:  # sharded input
        return {"shard_shape": [min(c, s) for c, s in zip(info.chunk_shape, out_shape)],
                "chunk_shape": [min(g, s) for g, s in zip(info.inner_chunk_shape, out_shape)]}
    return {"chunk_shape": [min(c, s) for c, s in zip(info.chunk_shape, out_shape)]}


def axis_of(name: str, unit):
    """units_to_axis (zarrs_ome.rs:390-432)."""
    if unit is None:
        return {"name": name}
    if unit in SPACE_UNITS:
        return {"name": name, "type": "space", "unit": unit}
    if unit in TIME_UNITS:
        return {"name": name, "type": "time", "unit": unit}
    if unit == "channel":
        return {"name": name, "type": "channel"}
    return {"name": name, "unit": unit}


def _reencode_level0(src, dst, encoding, nthreads, log):
    """Reencode::apply for level 0: the input's data in the new encoding, chunk row by chunk row
    (host copy through the store codecs)."""
    S.create_output_like(src, dst, encoding.get("data_type"), encoding)
    out = S.open_array(dst)
    info = S.open_array(src)
    cz = out.chunk_shape[0]
    for z0 in range(0, info.shape[0], cz):
        n = min(cz, info.shape[0] - z0)
        block = S.read_array(src, [z0] + [0] * (info.ndim - 1), [n] + list(info.shape[1:]),
                             nthreads=nthreads)
        if out.data_type != info.data_type:
            raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                         "zarrs_ome level 0: --data-type is not supported")
        S.write_array(dst, block, [z0] + [0] * (info.ndim - 1), nthreads=nthreads)
    log(f"0: reencode {src} -> {dst} ({out.data_type} {list(out.shape)})")


def _device_pyramid_fits(info, gauss, device: int, frac: float = 0.8) -> bool:
    """Level 0 + the pyramid (< 1/7 of level 0 for 2x factors, bounded by level 0 here) + the
    f32 Gaussian of the largest level, against `frac` of the free device memory."""
    import torch
    n = int(np.prod(info.shape))
    need = 2 * n * S.NUMPY[info.data_type]().itemsize + (4 * n if gauss is not None else 0)
    free, _ = torch.cuda.mem_get_info(device)
    return need <= frac * free


def run(input_path, output_path, factor=None, max_levels: int = 10, discrete: bool = False,
        name=None, exists: str = "erase", device: int = 0, nthreads: int = 0,
        gaussian_sigma=None, gaussian_kernel_half_size=None, physical_size=None,
        physical_units=None, group_attributes=None, reencoding=None, log=print,
        device_resident: bool = True) -> dict:
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
    for what, v in (("physical size", physical_size), ("physical units", physical_units)):
        if v is not None and len(v) != nd:
            raise _abi.InvalidParameters(_abi.ERR_INVALID_PARAMETERS,
                                         f"{what} must have one entry per axis")
    group_attrs = {}
    if group_attributes:
        group_attrs.update(json.loads(group_attributes) if isinstance(group_attributes, str)
                           else group_attributes)
    if os.path.exists(output_path):
        if exists == "exit":
            raise _abi.FilterError(_abi.ERR_OTHER, "Output exists, exiting")
        if exists == "erase":
            shutil.rmtree(output_path)
    os.makedirs(output_path, exist_ok=True)
    lvl0 = os.path.join(output_path, "0")
    if reencoding:
        _reencode_level0(input_path, lvl0, reencoding, nthreads, log)
    else:
        if os.path.exists(lvl0):
            shutil.rmtree(lvl0)
        shutil.copytree(input_path, lvl0)
        log(f"0: copy {input_path} -> {lvl0} ({info.data_type} {list(info.shape)})")
    # move array 0's attributes to the group (zarrs_ome.rs:368-377)
    meta0_path = os.path.join(lvl0, "zarr.json")
    with open(meta0_path) as f:
        meta0 = json.load(f)
    moved = dict(meta0.get("attributes") or {})
    moved.pop("_zarrs", None)
    group_attrs.update(moved)
    meta0["attributes"] = {}
    with open(meta0_path, "w") as f:
        json.dump(meta0, f, indent=2)
    dim_names = meta0.get("dimension_names")

    scale = [1.0] * nd
    datasets = [{"path": "0", "coordinateTransformations": [
        {"type": "scale", "scale": list(scale)}]}]
    shape = list(S.open_array(lvl0).shape)
    stats = []
    lvl0_info = S.open_array(lvl0)
    on_device = (device_resident and _device_ok(device)
                 and _device_pyramid_fits(lvl0_info, gauss, device))
    cur = None  # the previous level in HBM (device-resident pyramid)
    if on_device:
        from . import filter as F
        ctx = F.default_context(device)
        t1 = time.perf_counter()
        cur = read_to_device(lvl0, device, nthreads)
        log(f"   level 0 -> device in {time.perf_counter() - t1:.2f}s")
    for i in range(1, max_levels + 1):
        src, dst = os.path.join(output_path, str(i - 1)), os.path.join(output_path, str(i))
        src_info = S.open_array(src)
        out_shape = [max(s // f, 1) for s, f in zip(shape, factor)]  # downsample.rs:162-168
        enc = level_encoding(src_info, out_shape)
        if on_device:
            # the level from the previous one in HBM: (Gaussian, f32) then the downsample, the
            # same kernels as the store path's per-row calls (chunked == whole array)
            t1 = time.perf_counter()
            S.create_output(src, dst, None, out_shape, enc)
            v = cur
            if gauss is not None:
                v = F.Gaussian(gauss[0], gauss[1]).apply_ndarray(v, dtype_out="float32", ctx=ctx)
            ds = F.Downsample(factor, discrete=discrete)
            nxt = ds._apply(v, src_info.data_type, discrete, ctx)
            nxt = nxt.reshape(out_shape)
            ctx.synchronize()
            t_k = time.perf_counter() - t1
            t2 = time.perf_counter()
            write_from_device(dst, nxt, nthreads)
            st = {"wall_s": time.perf_counter() - t1, "decode_s": 0.0,
                  "encode_s": time.perf_counter() - t2, "h2d_s": 0.0, "kernel_s": t_k,
                  "d2h_s": 0.0, "voxels": int(nxt.numel()), "device_resident": True}
            cur = nxt
        elif gauss is not None:
            st = S.downsample_gaussian(src, dst, factor, gauss[0], gauss[1], device=device,
                                       nthreads=nthreads, encoding=enc)
        else:
            st = S.downsample(src, dst, factor, discrete=discrete, device=device,
                              nthreads=nthreads, encoding=enc)
        stats.append(st)
        out = S.open_array(dst)
        scale = level_scale(scale, shape, out.shape)
        datasets.append({"path": str(i), "coordinateTransformations": [
            {"type": "scale", "scale": list(scale)},
            {"type": "translation", "translation": level_translation(scale)}]})
        log(f"{i}: {list(shape)} -> {list(out.shape)} in {st['wall_s']:.2f}s")
        shape = list(out.shape)
        if all(f == 1 or s == 1 for f, s in zip(factor, shape)):
            break
    units = physical_units or [None] * nd
    axes = [axis_of(dim_names[k] if dim_names and dim_names[k] is not None else str(k),
                    units[k]) for k in range(nd)]
    ms = {}
    if name is not None:
        ms["name"] = name
    ms["axes"] = axes
    ms["datasets"] = datasets
    if physical_size is not None:
        ms["coordinateTransformations"] = [{"type": "scale",
                                            "scale": [float(x) for x in physical_size]}]
    ms["type"] = "mode" if discrete else ("average" if gauss is None else "gaussian")
    ms["metadata"] = {"description": "Created with zarrs_ome", "repository": "zarrs_tools_amd",
                      "version": VERSION}
    group_attrs["ome"] = {"version": "0.5", "multiscales": [ms]}
    group = {"zarr_format": 3, "node_type": "group", "attributes": group_attrs}
    with open(os.path.join(output_path, "zarr.json"), "w") as f:
        json.dump(group, f, indent=2)
    log(f"Output {output_path} in {time.perf_counter() - t0:.2f}s")
    return {"levels": len(stats), "stats": stats}


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    enc = encoding_of({k: getattr(a, k, None) for k in REENCODE_KEYS})
    try:
        run(a.input, a.output, a.factor, a.max_levels, a.discrete, a.name, a.exists, a.device,
            a.filter_chunk_limit or 0, a.gaussian_sigma, a.gaussian_kernel_half_size,
            a.physical_size, a.physical_units, a.group_attributes, enc,
            device_resident=not a.no_device_resident)
    except _abi.FilterError as e:
        print(f"Error: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
