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
        for mode, dev in (("device_resident", True), ("store_loop", False)):
            out = os.path.join(work, mode)
            t0 = time.perf_counter()
            r = ZO.run(pin, out, max_levels=a.levels, nthreads=a.threads, log=lambda *x: None,
                       device_resident=dev)
            wall = time.perf_counter() - t0
            res[mode] = {"wall_s": round(wall, 3), "levels": r["levels"],
                         "input_gvox_per_s": round(a.size ** 3 / wall / 1e9, 3),
                         "level_s": [round(st["wall_s"], 3) for st in r["stats"]]}
        # parity: a corner block of every level vs the oracle chain on the same block
        blk = min(64, a.size)
        ref = S.read_array(pin, (0, 0, 0), (blk,) * 3)
        ok = True
        for lvl in range(1, res["device_resident"]["levels"] + 1):
            ref = O.downsample(ref, "uint16", (2, 2, 2), "uint16")
            n = ref.shape
            for mode in ("device_resident", "store_loop"):
                got = S.read_array(os.path.join(work, mode, str(lvl)), (0, 0, 0), n)
                ok = ok and bool(np.array_equal(got, ref))
            if min(n) <= 1:
                break
        res["parity"] = {"bit_exact_corner_blocks": ok}
        print(json.dumps(res), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
