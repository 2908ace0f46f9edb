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
    # plain k_gsrb4 with a tenth, idle wave (as the correction form's loader)
    "b4w10": [("omg_block.hip", "constexpr int b4_threads(int pro) { return pro ? B4BS + 64 : B4BS; }",
               "constexpr int b4_threads(int pro) { return B4BS + 64; }"),
              ("omg_block.hip", "  if (PRO && tid >= B4BS) {",
               "  if (!PRO && tid >= B4BS) {\n    for (int t = -4 - AH; t <= zend + 4; t += AH)\n      for (int u = 0; u < AH; u++) __syncthreads();\n    return;\n  }\n  if (PRO && tid >= B4BS) {"),
              ("omg_block.hip", "else k_gsrb4<OP_HELM, 0><<<n_cols, B4BS, 0, st>>>", "else k_gsrb4<OP_HELM, 0><<<n_cols, B4BS + 64, 0, st>>>"),
              ("omg_block.hip", "else k_gsrb4<OP_LPL, 0><<<n_cols, B4BS, 0, st>>>", "else k_gsrb4<OP_LPL, 0><<<n_cols, B4BS + 64, 0, st>>>")],
    # k_gsrb4's plain form (the down-smoothing) with 2 planes of loads in
    # flight, as its correction form (r06)
    "b4ah2": [("omg_block.hip", "constexpr int AH = PRO ? 2 : kB3Ahead;", "constexpr int AH = 2;")],
    # k_gsrb3 (every form) with 2 planes ahead
    "b3ah2": [("omg_block.hip", "constexpr int kB3Ahead = 4;", "constexpr int kB3Ahead = 2;"),
              ("omg_block.hip", "constexpr int AH = PRO ? 2 : kB3Ahead;", "constexpr int AH = PRO ? 2 : 4;")],
    # the periodic rhs pass (k_box_sums3<SUB>): 16 leaves per wave (2048
    # waves, two per SIMD on C3's level 1) / chunks of 8 rows / both
    "sumslpw16": [("omg_tiles.hip", "constexpr int kSumsLPW = 32, kSumsR = 4;", "constexpr int kSumsLPW = 16, kSumsR = 4;")],
    "sumsr8": [("omg_tiles.hip", "constexpr int kSumsLPW = 32, kSumsR = 4;", "constexpr int kSumsLPW = 32, kSumsR = 8;")],
    "sumsr2": [("omg_tiles.hip", "constexpr int kSumsLPW = 32, kSumsR = 4;", "constexpr int kSumsLPW = 32, kSumsR = 2;")],
    # physical faces in the block passes (r06; timing only, not parity-correct):
    # no ghost formed in substeps 2-4 / no physical work in the store wave /
    # the plain load
    # paired 16-B loads in k_gsrb4's plain form, at 5 waves per SIMD (spills)
    "pairw5": [("omg_block.hip", "__global__ void __launch_bounds__(b4_threads(PRO)) k_gsrb4",
                "__global__ void __launch_bounds__(b4_threads(PRO)) __attribute__((amdgpu_waves_per_eu(5))) k_gsrb4")],
    "phnofix": [("omg_block.hip", "if (PHYS) b3_fix(", "if (false) b3_fix(")] * 5,
    "phnostore": [("omg_block.hip", "if (PHYS && ((zlo && k == 2) || (zhi && k == B3NC))) {", "if (false) {"),
                  ("omg_block.hip", "if (PHYS && ((w == 0 && (fl & 1)) || (w == 3 && (fl & 2)))) {", "if (false) {"),
                  ("omg_block.hip", "if (PHYS && ((jr == 0 && (fl & 4)) || (jr == B3NC - 1 && (fl & 8)))) {", "if (false) {")] * 2,
    "phnoload": [("omg_block.hip", "    if (!PHYS) q = b3_ld(src, bo[kB3S * zs + slot] + xyb + po);", "    if (true) q = b3_ld(src, bo[kB3S * zs + slot] + xyb + po);")] * 2,
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
        open(p, "w").write(s.replace(a, b, 1))
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
