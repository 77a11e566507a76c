"""Summarise rocprofv3 counter CSVs (tools/profile_pmc.sh output) for one kernel."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "gf3d"
vox = float(sys.argv[3]) if len(sys.argv) > 3 else 1024 ** 3
agg = collections.defaultdict(float)
for f in sorted(glob.glob(f"{d}/*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print(f"{k:28s} {v:16.4g}   per voxel {v / vox:10.4f}")
if "SQ_WAVE_CYCLES" in agg:
    wc = agg["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
              "SQ_ACTIVE_INST_LDS"):
        if k in agg:
            print(f"  {k} / WAVE_CYCLES = {agg[k] / wc:.3f}")
if "FETCH_SIZE" in agg:
    print(f"  HBM-side read bytes/voxel (FETCH_SIZE x2 gfx950 correction): "
          f"{agg['FETCH_SIZE'] * 1024 * 2 / vox:.2f}")
if "WRITE_SIZE" in agg:
    print(f"  write bytes/voxel: {agg['WRITE_SIZE'] * 1024 / vox:.2f}")
