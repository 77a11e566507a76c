#!/usr/bin/env python3
"""Write pmc_traffic.json (the per-launch HBM traffic bench.py reports as roofline.traffic) from
the FETCH_SIZE / WRITE_SIZE passes of tools/profile_pmc.sh, keyed to the library build (sha256),
the workload and the world size, so bench.py only reports it for the build it was measured on.

Usage: make_traffic_json.py PMC_DIR OUT_JSON [size radius [G/N]]  (merges into OUT_JSON's entries;
G/N keys the entry to a `bench.py --share G/N` proxy run)
       make_traffic_json.py --legs PMC_DIR OUT_JSON [legs...]  (bench.py's extra legs)
Method (MI355X_MICROARCH.md, HBM / rocprofv3): one launch (bench.py --steps 1 --warmup 0), each
counter in its own run; FETCH_SIZE and WRITE_SIZE are KiB; FETCH_SIZE x2 is the gfx950
correction for wide (128 B) reads counted as 64 B.
"""
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def total(d, counter, pat="gf3d"):
    v, n = 0.0, set()
    for f in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"] and r["Counter_Name"] == counter:
                v += float(r["Counter_Value"])
                n.add(r["Dispatch_Id"])
    return v, len(n)


def lib_sha() -> str:
    h = hashlib.sha256()
    with open(os.path.join(ROOT, "zarrs_tools_amd", "libzarrs_tools_amd.so"), "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def merge(out, keep, d):
    entries = []
    if os.path.exists(out):
        try:
            old = json.load(open(out))
            entries = old.get("entries", [old]) if isinstance(old, dict) else list(old)
        except ValueError:
            entries = []
    entries = [e for e in entries if e.get("lib_sha256") == d["lib_sha256"] and keep(e)]
    entries.append(d)
    with open(out, "w") as f:
        json.dump({"entries": entries}, f, indent=1)
    print(json.dumps(d))


def legs_main(pmc, out, legs):
    """Entries for bench.py's extra legs from tools/profile_pmc_legs.sh: every kernel of one
    call (bench.py --only-extra LEG) except the synthetic-input generators."""
    sha = lib_sha()
    for leg in legs:
        rd = wr = 0.0
        names = set()
        for c, dst in (("FETCH_SIZE", "r"), ("WRITE_SIZE", "w")):
            for f in glob.glob(os.path.join(pmc, f"{leg}_{c}", "**", "run_counter_collection.csv"),
                               recursive=True):
                for r in csv.DictReader(open(f)):
                    if r["Counter_Name"] != c or "synth" in r["Kernel_Name"]:
                        continue
                    names.add(r["Kernel_Name"].split("(")[0][:80])
                    if dst == "r":
                        rd += float(r["Counter_Value"]) * 1024 * 2
                    else:
                        wr += float(r["Counter_Value"]) * 1024
        d = {"lib_sha256": sha, "leg": leg, "hbm_bytes_per_call": rd + wr, "read_bytes": rd,
             "write_bytes": wr, "kernels": sorted(names),
             "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of "
                       "bench.py --only-extra LEG (one call); FETCH_SIZE x2 (gfx950 wide-read "
                       "correction), KiB -> bytes; synthetic-input kernels excluded"}
        merge(out, lambda e, leg=leg: e.get("leg") != leg, d)


def main():
    if sys.argv[1] == "--legs":
        return legs_main(sys.argv[2], sys.argv[3], sys.argv[4:] or
                         ["g2", "t_share", "pyramid_octant", "gaussian"])
    pmc, out = sys.argv[1], sys.argv[2]
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
    radius = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    share = [int(v) for v in sys.argv[5].split("/")] if len(sys.argv) > 5 else None
    fetch, nf = total(os.path.join(pmc, "fetch"), "FETCH_SIZE")
    write, nw = total(os.path.join(pmc, "write"), "WRITE_SIZE")
    # one step per pass: one launch, or the interior + edge launches of a share's slab
    if nf != nw or not 1 <= nf <= 2:
        sys.exit(f"expected the launches of one step per pass, got {nf} / {nw}")
    h = hashlib.sha256()
    with open(os.path.join(ROOT, "zarrs_tools_amd", "libzarrs_tools_amd.so"), "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    vox = size ** 3
    if share is not None:  # the voxels of that rank's slab (bench.py's slab_assignment)
        sys.path.insert(0, ROOT)
        from zarrs_tools_amd.shard import slab_assignment
        a = slab_assignment(share[0], share[1], size, 256, 2 * radius)
        vox = a.out_nz * size * size
    rd, wr = fetch * 1024 * 2, write * 1024
    d = {"lib_sha256": h.hexdigest(), "global_shape": [size] * 3, "radius": radius, "world": 1,
         "kernel": "gf3d_fused_kernel (interior + edge launches of one step)", "launches": nf,
         "hbm_bytes_per_launch": rd + wr, "read_bytes_per_voxel": round(rd / vox, 3),
         "write_bytes_per_voxel": round(wr / vox, 3),
         "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of bench.py "
                   "--steps 1 --warmup 0; FETCH_SIZE x2 (gfx950 wide-read correction), KiB -> "
                   "bytes; Infinity-Cache hits are counted by these counters"}
    if share is not None:
        d["share"] = share
    # the SQ instruction counters of the same kernel (tools/profile_pmc.sh passes sq1 / sq2),
    # per output voxel, and the wave-cycle ratios: reported beside the traffic by bench.py
    sq = {}
    for pas in ("sq1", "sq2"):
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            v, n = total(os.path.join(pmc, pas), c)
            if n:
                sq[c] = v / n  # per launch
    if sq:
        d["sq_per_voxel"] = {k[len("SQ_INSTS_"):]: round(sq[k] / vox, 4) for k in sq
                             if k.startswith("SQ_INSTS_")}
        wc = sq.get("SQ_WAVE_CYCLES")
        if wc:
            d["sq_wave_cycle_ratios"] = {k[len("SQ_"):] : round(sq[k] / wc, 4) for k in
                                         ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                                          "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS") if k in sq}
    # merge: one entry per (shape, radius, world); entries of other builds are dropped
    entries = []
    if os.path.exists(out):
        try:
            old = json.load(open(out))
            entries = old.get("entries", [old]) if isinstance(old, dict) else list(old)
        except ValueError:
            entries = []
    entries = [e for e in entries if e.get("lib_sha256") == d["lib_sha256"] and
               (e.get("global_shape"), e.get("radius"), e.get("world", 1), e.get("share")) !=
               (d["global_shape"], d["radius"], d["world"], d.get("share"))]
    entries.append(d)
    with open(out, "w") as f:
        json.dump({"entries": entries}, f, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
