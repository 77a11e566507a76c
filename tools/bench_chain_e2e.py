#!/usr/bin/env python3
"""End-to-end run-config chain (zarrs_filter.rs:338-381): guided_filter -> $t -> gaussian -> $u ->
downsample, store -> store on a synthetic f32 volume, (a) device-resident (the chain input read
once, the output written once) and (b) step by step through temporary stores (the reference's
loop). Prints one JSON line; the two outputs are compared bit for bit."""
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
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    a = ap.parse_args()
    import numpy as np
    from zarrs_tools_amd import store as S
    from zarrs_tools_amd import zarrs_filter as ZF
    work = os.path.join(a.dir, f"zt_chain_{os.getpid()}")
    os.makedirs(work, exist_ok=True)
    try:
        pin = os.path.join(work, "in.zarr")
        shape = (a.size,) * 3
        S.create_array(pin, "float32", shape, (a.chunk,) * 3)
        S.write_synth(pin, S.SYNTH_STEP_NOISE_F32, nthreads=a.threads)

        def steps(out):
            return [{"filter": "guided_filter", "input": pin, "output": "$t", "epsilon": 2500.0,
                     "radius": 2},
                    {"filter": "gaussian", "input": "$t", "output": "$u",
                     "sigma": [1.0, 1.0, 1.0], "kernel_half_size": [3, 3, 3]},
                    {"filter": "downsample", "input": "$u", "output": out, "stride": [2, 2, 2]}]
        res = {"metric": "zarrs_filter run-config chain end-to-end (guided r=2 -> gaussian -> "
                         "downsample 2x, warm page cache)",
               "config": {"shape": shape, "chunk": [a.chunk] * 3, "dtype": "float32",
                          "host_threads": a.threads}}
        outs = {}
        for mode, chain in (("device_chain", True), ("store_steps", False)):
            outs[mode] = os.path.join(work, mode + ".zarr")
            t0 = time.perf_counter()
            st = ZF.run(steps(outs[mode]), tmp=work, chunk_limit=a.threads,
                        log=lambda *x: None, device_chain=chain)
            wall = time.perf_counter() - t0
            res[mode] = {"wall_s": round(wall, 3),
                         "input_gib_per_s": round(a.size ** 3 * 4 / 2 ** 30 / wall, 3),
                         "device_resident": [bool(s.get("device_resident")) for s in st],
                         "step_s": [round(s["wall_s"], 3) for s in st]}
        res["bit_identical"] = bool(np.array_equal(S.read_array(outs["device_chain"]),
                                                   S.read_array(outs["store_steps"])))
        print(json.dumps(res), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
