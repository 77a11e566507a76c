#!/usr/bin/env python3
"""End-to-end (store -> store) guided filter rate: a Zarr V3 store on host storage in, a Zarr V3
store out, chunk decode -> H2D -> HIP kernel -> D2H -> chunk encode pipelined (zt_store_guided_
filter). Prints one JSON line. The input store is written first (not timed) and is therefore in
the host page cache: the rate is "warm page cache" (no drop_caches without root).

A sample of the output (the first chunk row) is checked against the oracle (test
infrastructure, never timed): planes [0, c) of the output depend only on input planes [0, c+2r),
so the oracle run on that block gives the reference's values for them.
"""
import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cpu_store_baseline(pin, pout, shape, chunk, eps, radius, threads, nchunks):
    """The reference's CPU path store -> store on a sample of output chunks (GuidedFilter::apply,
    guided_filter.rs:260-316): per chunk, in a pool of host threads, read the chunk plus its 2r
    halo from the input store (decode), run the C restatement of apply_ndarray (oracle/, faithful
    incl. the dead SAT), and write the chunk to the output store (encode). Test infrastructure:
    the oracle is the baseline here, never the measured product."""
    import itertools
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    from oracle import oracle as O
    from zarrs_tools_amd import store as S
    S.create_output_like(pin, pout)
    grid = [-(-n // c) for n, c in zip(shape, chunk)]
    coords = list(itertools.islice(itertools.product(*[range(g) for g in grid]), nchunks))
    h = 2 * radius

    def one(cc):
        o0 = [c * k for c, k in zip(cc, chunk)]
        on = [min(k, n - s) for k, n, s in zip(chunk, shape, o0)]
        i0 = [max(0, s - h) for s in o0]
        i1 = [min(n, s + e + h) for s, e, n in zip(o0, on, shape)]
        block = S.read_array(pin, i0, [b - a for a, b in zip(i0, i1)], nthreads=1)
        out = O.guided_filter_apply_ndarray(block, eps, radius, faithful=True)
        sub = tuple(slice(s - a, s - a + e) for s, a, e in zip(o0, i0, on))
        S.write_array(pout, np.ascontiguousarray(out[sub]), o0, nthreads=1)
        return int(np.prod(on))

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        vox = sum(ex.map(one, coords))
    secs = time.perf_counter() - t0
    return {"value": round(vox * 4 / 2 ** 30 / secs, 4), "unit": "GiB/s", "cores": threads,
            "kind": "port", "secs": round(secs, 2),
            "sample": f"{len(coords)} output chunks of {'x'.join(map(str, chunk))} (first in C "
                      f"order), store read of chunk + 2r halo, oracle apply_ndarray (faithful), "
                      f"store write; {threads} host threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--nz", type=int, default=0, help="z extent (default: --size)")
    ap.add_argument("--chunk", type=int, default=256)
    ap.add_argument("--radius", type=int, default=2)
    ap.add_argument("--eps", type=float, default=2500.0)
    ap.add_argument("--codec", default="bytes", choices=["bytes", "gzip", "zstd"])
    ap.add_argument("--level", type=int, default=1)
    ap.add_argument("--shard-inner", type=int, default=0, help="sharded store, inner chunk edge")
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--t", type=int, default=0,
                    help="4-D time series (config T): T timepoints of nz x size x size")
    ap.add_argument("--t-chunk", type=int, default=4, help="chunk extent along t (4-D)")
    ap.add_argument("--procs", type=int, default=1,
                    help="zarrs_filter --gpus N's store split (4-D: (t, z) blocks) over N "
                         "processes, all on device 0 here (a one-GPU rehearsal)")
    ap.add_argument("--cpu-chunks", type=int, default=0,
                    help="also time the CPU store -> store baseline on this many output chunks")
    a = ap.parse_args()

    from zarrs_tools_amd import store as S
    work = os.path.join(a.dir, f"zt_e2e_{os.getpid()}")
    os.makedirs(work, exist_ok=True)
    pin, pout = os.path.join(work, "in.zarr"), os.path.join(work, "out.zarr")
    shape, chunk = (a.nz or a.size, a.size, a.size), (a.chunk,) * 3
    if a.t:
        shape, chunk = (a.t,) + shape, (a.t_chunk,) + chunk
    comp = None if a.codec == "bytes" else a.codec
    codecs = S.codecs_json(comp, a.level, (a.shard_inner,) * len(shape) if a.shard_inner else None)
    try:
        t0 = time.perf_counter()
        S.create_array(pin, "float32", shape, chunk, codecs)
        S.write_synth(pin, S.SYNTH_STEP_NOISE_F32, nthreads=a.threads)
        t_make = time.perf_counter() - t0
        stats = []
        for _ in range(a.repeat):
            if a.procs > 1:
                from zarrs_tools_amd.zarrs_filter import run_rows_parallel
                st = run_rows_parallel("guided_filter", pin, pout,
                                       {"epsilon": a.eps, "radius": a.radius}, shape, a.procs,
                                       nthreads=a.threads, devices=[0] * a.procs)
                st["threads"] = a.threads
                stats.append(st)
            else:
                stats.append(S.guided_filter(pin, pout, a.eps, a.radius, nthreads=a.threads))
        best = min(stats, key=lambda s: s["wall_s"])
        vox = best["voxels"]
        res = {
            "metric": "GiB/s filtered end-to-end (Zarr V3 store -> store, warm page cache)",
            "value": round(vox * 4 / 2 ** 30 / best["wall_s"], 3),
            "unit": "GiB/s",
            "config": {"shape": shape, "chunk": chunk, "radius": a.radius, "eps": a.eps,
                       "codec": a.codec, "level": a.level, "shard_inner": a.shard_inner,
                       "host_threads": best["threads"], "processes": a.procs},
            "wall_s": round(best["wall_s"], 3),
            "phases": {k: round(best[k], 3) for k in
                       ("decode_s", "encode_s", "h2d_s", "kernel_s", "d2h_s")},
            "bytes_read": best["bytes_read"], "bytes_written": best["bytes_written"],
            "input_store_bytes_per_s": round(best["bytes_read"] / best["wall_s"] / 1e9, 3),
            "walls": [round(s["wall_s"], 3) for s in stats],
            "make_input_s": round(t_make, 2),
        }
        if a.check and a.t:
            # 4-D: a corner sub-box of the first t-chunk row; its block plus the 2r halo makes
            # the same windows as the whole array (chunked == whole with the halo)
            import numpy as np
            from oracle import oracle as O
            h = 2 * a.radius
            sub = (a.t_chunk, 16, 16, 64)
            bshape = tuple(min(s_ + h, n) for s_, n in zip(sub, shape))
            block = S.read_array(pin, (0,) * 4, bshape)
            got = S.read_array(pout, (0,) * 4, sub)
            ref = O.guided_filter_apply_ndarray(block, a.eps, a.radius)[tuple(slice(0, s_) for s_ in sub)]
            err = float(np.max(np.abs(got.astype(np.float64) - ref) /
                               np.maximum(1.0, np.abs(ref))))
            res["check"] = {"sub_box": sub, "max_rel_err": err, "ok": err <= 1e-5}
        elif a.check:
            import numpy as np
            from oracle import oracle as O
            c = a.chunk
            block = S.read_array(pin, (0, 0, 0), (min(c + 2 * a.radius, a.size), a.size, a.size))
            got = S.read_array(pout, (0, 0, 0), (c, a.size, a.size))
            ref = O.guided_filter_apply_ndarray(block, a.eps, a.radius)[:c]
            err = float(np.max(np.abs(got.astype(np.float64) - ref) /
                               np.maximum(1.0, np.abs(ref))))
            res["check"] = {"planes": c, "max_rel_err": err, "ok": err <= 1e-5}
        if a.cpu_chunks:
            res["cpu_baseline"] = cpu_store_baseline(pin, os.path.join(work, "cpu.zarr"), shape,
                                                     chunk, a.eps, a.radius, a.threads,
                                                     a.cpu_chunks)
        print(json.dumps(res), flush=True)
    finally:
        if not a.keep:
            shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
