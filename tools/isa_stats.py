"""Per-kernel ISA statistics from a hipcc -S listing: VGPR/SGPR counts, spills, and the
instruction mix of the whole kernel body (used to track VALU/LDS/SALU per step)."""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read().split("\n")
pat = sys.argv[2] if len(sys.argv) > 2 else ""
cur = None
bodies = {}
for line in src:
    m = re.match(r"^(_Z\w+):", line)
    if m:
        cur = m.group(1)
        bodies[cur] = []
        continue
    if cur and line.startswith("\t.size"):
        cur = None
        continue
    if cur:
        bodies[cur].append(line)
meta = {}
for name in bodies:
    m = re.search(rf"\.set {re.escape(name)}\.num_vgpr, (\d+)", "\n".join(src))
    meta[name] = m.group(1) if m else "?"
for name, body in bodies.items():
    if pat not in name:
        continue
    c = Counter()
    for l in body:
        l = l.strip()
        if not l or l.startswith((";", ".")) or l.endswith(":"):
            continue
        op = l.split()[0]
        if op.startswith("v_mov_b32_dpp") or "dpp" in l.split(";")[0] and op.startswith("v_"):
            c["dpp"] += 1
        if op.startswith("v_pk_"): c["valu_pk"] += 1
        if op.startswith(("v_add_f64", "v_fma_f64", "v_mul_f64", "v_cvt_f64", "v_cvt_f32_f64")): c["valu_f64"] += 1
        if op.startswith("v_"): c["valu"] += 1
        elif op.startswith("s_waitcnt"): c["waitcnt"] += 1
        elif op.startswith("s_barrier"): c["barrier"] += 1
        elif op.startswith("s_"): c["salu"] += 1
        elif op.startswith("ds_"): c["lds"] += 1
        elif op.startswith(("buffer_", "global_")): c["vmem"] += 1
        elif op.startswith("scratch_"): c["scratch"] += 1
    print(f"{name[:90]}\n   vgpr={meta[name]} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
