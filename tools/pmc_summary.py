"""Summarise rocprofv3 counter CSVs (tools/profile_pmc.sh output) for the kernels whose name
contains a pattern: the total over the run, the number of launches, the value per call and per
voxel of one call. A call is one launch unless CALLS is given (e.g. 2 when the profiled program
ran the op twice, each op being several launches); VOXELS = the voxels one call processes.

Usage: pmc_summary.py PMC_DIR [PATTERN [VOXELS [CALLS]]]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "gf3d"
vox = float(sys.argv[3]) if len(sys.argv) > 3 else 1024 ** 3
calls = int(sys.argv[4]) if len(sys.argv) > 4 else None
agg = collections.defaultdict(float)
launches = collections.defaultdict(set)
for f in sorted(glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            launches[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
per = {k: v / (calls or max(1, len(launches[k]))) for k, v in agg.items()}
print(f"kernel pattern {pat!r}, voxels per call {vox:.6g}, "
      f"{'calls ' + str(calls) if calls else 'call = one launch'}")
for k, v in sorted(agg.items()):
    print(f"{k:28s} total {v:14.4g}  launches {len(launches[k]):3d}  per call {per[k]:14.4g}"
          f"  per voxel {per[k] / vox:10.4f}")
if "SQ_WAVE_CYCLES" in per:
    wc = per["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
              "SQ_ACTIVE_INST_LDS"):
        if k in per:
            print(f"  {k} / WAVE_CYCLES = {per[k] / wc:.3f}")
if "FETCH_SIZE" in per:
    print(f"  HBM-side read bytes/voxel per call (FETCH_SIZE x2 gfx950 correction): "
          f"{per['FETCH_SIZE'] * 1024 * 2 / vox:.2f}")
if "WRITE_SIZE" in per:
    print(f"  write bytes/voxel per call: {per['WRITE_SIZE'] * 1024 / vox:.2f}")
if "TCC_HIT_sum" in per and "TCC_MISS_sum" in per:
    h, m = per["TCC_HIT_sum"], per["TCC_MISS_sum"]
    print(f"  L2 hit rate {h / max(1.0, h + m):.3f}")
