#!/usr/bin/env python3
"""End-to-end zarrs_ome (store -> OME-Zarr group) on a synthetic u16 volume: level 0 copied, levels
1..L by the HIP downsample, (a) device-resident (level 0 read once, every level written once) and
(b) the reference's loop (each level read back from the store). Prints one JSON line. Warm page
cache. A sample of every level is checked bit-exactly against the oracle downsample of the same
block (test infrastructure, never timed)."""
import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--chunk", type=int, default=256)
    ap.add_argument("--levels", type=int, default=5)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    ap.add_argument("--gpus", type=int, nargs="*", default=[],
                    help="also run zarrs_ome --gpus N for each N, every process on device 0 "
                         "(a one-GPU rehearsal of the octant split)")
    ap.add_argument("--cli", action="store_true",
                    help="also time each mode as a fresh `python -m zarrs_tools_amd.zarrs_ome` "
                         "process (interpreter start-up and imports included, as a user sees it)")
    a = ap.parse_args()
    import numpy as np
    from oracle import oracle as O
    from zarrs_tools_amd import store as S
    from zarrs_tools_amd import zarrs_ome as ZO
    work = os.path.join(a.dir, f"zt_ome_{os.getpid()}")
    os.makedirs(work, exist_ok=True)
    try:
        pin = os.path.join(work, "in.zarr")
        shape = (a.size,) * 3
        S.create_array(pin, "uint16", shape, (a.chunk,) * 3)
        S.write_synth(pin, S.SYNTH_U16, nthreads=a.threads)
        res = {"metric": "zarrs_ome 2x mean pyramid end-to-end (store -> OME-Zarr, warm page "
                         "cache)", "config": {"shape": shape, "chunk": [a.chunk] * 3,
                                               "dtype": "uint16", "levels": a.levels,
                                               "host_threads": a.threads}}
        modes = [("device_resident", True, 1), ("store_loop", False, 1)]
        modes += [(f"octants_{g}_procs_one_gpu", True, g) for g in a.gpus]
        # parity reference: a corner block of every level by the oracle chain (never timed)
        blk = min(64, a.size)
        refs, ref = [], S.read_array(pin, (0, 0, 0), (blk,) * 3)
        for lvl in range(1, a.levels + 1):
            ref = O.downsample(ref, "uint16", (2, 2, 2), "uint16")
            refs.append(ref)
            if min(ref.shape) <= 1:
                break
        ok = True
        for mode, dev, g in modes:
            out = os.path.join(work, mode)
            t0 = time.perf_counter()
            kw = {"gpus": g, "gpu_devices": [0] * g} if g > 1 else {}
            r = ZO.run(pin, out, max_levels=a.levels, nthreads=a.threads, log=lambda *x: None,
                       device_resident=dev, **kw)
            wall = time.perf_counter() - t0
            res[mode] = {"wall_s": round(wall, 3), "levels": r["levels"],
                         "input_gvox_per_s": round(a.size ** 3 / wall / 1e9, 3),
                         "level_s": [round(st["wall_s"], 3) for st in r["stats"]],
                         "phases": r.get("phases", {})}
            oct_st = [st for st in r["stats"] if "per_rank" in st]
            if oct_st:  # the octant workers' own phases (box read, device pyramid, writes)
                res[mode]["octant_ranks"] = [
                    {k: (round(v, 3) if isinstance(v, float) else v) for k, v in pr.items()}
                    for pr in oct_st[0]["per_rank"]]
            for lvl, want in enumerate(refs[:r["levels"]], start=1):
                got = S.read_array(os.path.join(out, str(lvl)), (0, 0, 0), want.shape)
                ok = ok and bool(np.array_equal(got, want))
            shutil.rmtree(out, ignore_errors=True)  # (disk: one output at a time)
            if a.cli:
                import subprocess
                cmd = [sys.executable, "-m", "zarrs_tools_amd.zarrs_ome", pin, out,
                       "--max-levels", str(a.levels)]
                if not dev:
                    cmd.append("--no-device-resident")
                if g > 1:
                    cmd += ["--gpus", str(g), "--gpu-devices", ",".join(["0"] * g)]
                t0 = time.perf_counter()
                subprocess.run(cmd, check=True, cwd=ROOT, stdout=subprocess.DEVNULL)
                res[mode]["cli_wall_s"] = round(time.perf_counter() - t0, 3)
                got = S.read_array(os.path.join(out, "1"), (0, 0, 0), refs[0].shape)
                ok = ok and bool(np.array_equal(got, refs[0]))
                shutil.rmtree(out, ignore_errors=True)
        res["parity"] = {"bit_exact_corner_blocks": ok}
        print(json.dumps(res), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
