"""Generate the committed golden fixtures (tests/golden/*.npy + cases.json).

Inputs are the seeded synthetic volumes of SURVEY.md §8(d) (or the reference's own KAT input);
expected outputs come from the C oracle (oracle/zt_oracle.c), which is itself pinned bit-exactly
by the reference's known-answer tests (guided_filter.rs:364-369, summed_area_table.rs:306-313;
see tests/test_oracle.py). Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402

GUIDED = [
    # name, shape, chunk, eps, radius, dtype_in, dtype_out
    ("kat_4x4_r2", None, (2, 2), 1.0, 2, "float32", "float32"),
    ("g3_f32_r1", (20, 21, 22), (8, 8, 8), 2500.0, 1, "float32", "float32"),
    ("g3_f32_r2", (24, 24, 24), (10, 10, 10), 2500.0, 2, "float32", "float32"),
    ("g3_f32_r4", (40, 36, 34), (16, 16, 16), 2500.0, 4, "float32", "float32"),
    ("g3_u16_f32_r2", (18, 19, 33), (8, 8, 16), 40000.0, 2, "uint16", "float32"),
    ("g3_f32_u8_r3", (16, 17, 18), (8, 8, 8), 100.0, 3, "float32", "uint8"),
    ("g2_f32_r3", (37, 41), (16, 16), 2500.0, 3, "float32", "float32"),
    ("g1_f32_r2", (50,), (16,), 2500.0, 2, "float32", "float32"),
    ("g4_f32_r1", (6, 10, 11, 12), (2, 4, 4, 4), 2500.0, 1, "float32", "float32"),
]

DOWNSAMPLE = [
    # name, shape, stride, dtype_in, dtype_out, discrete
    ("ds_u16_odd", (17, 18, 19), (2, 2, 2), "uint16", "uint16", False),
    ("ds_f32_mixed", (9, 10, 11), (2, 3, 2), "float32", "float32", False),
    ("ds_u8_f32", (8, 6, 5), (2, 2, 2), "uint8", "float32", False),
    ("ds_u8_mode", (8, 9, 10), (2, 2, 2), "uint8", "uint8", True),
    ("ds_i16_short_axis", (3, 8, 8), (4, 2, 2), "int16", "int16", False),
]


def synth_input(shape, dtype):
    if dtype == "uint16":
        return O.synth_u16(shape)
    v = O.synth_step_noise_f32(shape)
    if dtype == "float32":
        return v
    return O.cast_from_f32(v, dtype)


def main():
    cases = {"guided_filter": [], "downsample": []}
    for name, shape, chunk, eps, r, din, dout in GUIDED:
        if shape is None:  # the reference's own test input: value = row + col (4x4 f32)
            v = np.array([[i + j for j in range(4)] for i in range(4)], dtype=np.float32)
        else:
            v = synth_input(shape, din)
        vin_f32 = O.cast_to_f32(v, din) if din != "float32" else v
        out_f32 = O.guided_filter_apply(vin_f32, chunk, eps, r, nthreads=8)
        out = O.cast_from_f32(out_f32, dout) if dout != "float32" else out_f32
        np.save(os.path.join(HERE, f"{name}_in.npy"), v, allow_pickle=False)
        np.save(os.path.join(HERE, f"{name}_out.npy"), out, allow_pickle=False)
        np.save(os.path.join(HERE, f"{name}_out_f32.npy"), out_f32, allow_pickle=False)
        cases["guided_filter"].append(dict(name=name, shape=list(v.shape), chunk_shape=list(chunk),
                                           epsilon=eps, radius=r, dtype_in=din, dtype_out=dout))
    for name, shape, stride, din, dout, discrete in DOWNSAMPLE:
        v = synth_input(shape, din)
        if din == "int16":
            v = (v.astype(np.int32) - 300).astype(np.int16)
        if discrete:  # few distinct labels so the mode is meaningful
            v = (v % 4).astype(np.uint8)
        out = O.downsample(v, din, stride, dout, discrete=discrete)
        np.save(os.path.join(HERE, f"{name}_in.npy"), v, allow_pickle=False)
        np.save(os.path.join(HERE, f"{name}_out.npy"), out, allow_pickle=False)
        cases["downsample"].append(dict(name=name, shape=list(shape), stride=list(stride),
                                        dtype_in=din, dtype_out=dout, discrete=discrete))
    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump(cases, f, indent=1)
    print("wrote", sum(len(v) for v in cases.values()), "cases")


if __name__ == "__main__":
    main()
