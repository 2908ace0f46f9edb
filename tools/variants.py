#!/usr/bin/env python3
"""Variant builds of libomg.so for A/B timing: copies octree-mg_amd/csrc to
/tmp, applies text patches, builds octree-mg_amd/_variants/libomg_<name>.so
(load with OMG_LIB=...; tools/ab_bench.sh times them interleaved with the
default library).  Delete the _variants afterwards: they travel to the GPU
box with every gpurun call.   usage: tools/variants.py name [name ...]"""
import os
import shutil
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# name -> [(file, old, new), ...]
VARIANTS = {
    # the periodic rhs pass (k_box_sums3<SUB>): 16 leaves per wave (2048
    # waves, two per SIMD on C3's level 1) / chunks of 8 rows / both
    "sumslpw16": [("omg_tiles.hip", "constexpr int kSumsLPW = 32, kSumsR = 4;", "constexpr int kSumsLPW = 16, kSumsR = 4;")],
    "sumsr8": [("omg_tiles.hip", "constexpr int kSumsLPW = 32, kSumsR = 4;", "constexpr int kSumsLPW = 32, kSumsR = 8;")],
    "sumsr2": [("omg_tiles.hip", "constexpr int kSumsLPW = 32, kSumsR = 4;", "constexpr int kSumsLPW = 32, kSumsR = 2;")],
}


def build(name):
    d = f"/tmp/omgv/{name}/csrc"
    shutil.rmtree(os.path.dirname(d), ignore_errors=True)
    os.makedirs(os.path.join(os.path.dirname(os.path.dirname(d)), "include"), exist_ok=True)
    shutil.copy(os.path.join(R, "include", "omg.h"), os.path.join(os.path.dirname(os.path.dirname(d)), "include"))
    shutil.copytree(os.path.join(R, "octree-mg_amd", "csrc"), d)
    for f, a, b in VARIANTS[name]:
        p = os.path.join(d, f)
        s = open(p).read()
        assert a in s, (name, a)
        open(p, "w").write(s.replace(a, b))
    out = os.path.join(R, "octree-mg_amd", "_variants", f"libomg_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    for o in os.listdir(d):
        if o.endswith(".o"):
            os.remove(os.path.join(d, o))
    subprocess.run(["make", "-j8", "-C", d, f"OUT={out}"], check=True, stdout=subprocess.DEVNULL)
    print("built", out)


if __name__ == "__main__":
    for n in sys.argv[1:]:
        build(n)
