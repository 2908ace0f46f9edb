"""Timing-only builds (not parity-correct unless noted): copies
octree-mg_amd/csrc to /tmp, patches omg_block.hip (or FILES[name]), builds
octree-mg_amd/_variants/libomg_b3p_<name>.so (load with OMG_LIB=...)."""
import os, shutil, subprocess, sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = {"subnt": "omg_tiles.hip", "subntld": "omg_tiles.hip", "z8": "omg_api.cpp", "z2": "omg_api.cpp"}
# (default: omg_block.hip)
VARIANTS = {
    # the plain pass at 6 waves per SIMD (3 workgroups per CU; 79 VGPRs, 20 B
    # of scratch), the other forms unchanged
    "occ6": [("__global__ void __launch_bounds__(B3BS) k_gsrb3", "__global__ void __launch_bounds__(B3BS, (PRO == 0 && !RES) ? 6 : 1) k_gsrb3")],
    # the coarse tile with a 3-cell rim (22 x 14), as before r05/s47
    "ct22": [("constexpr int B3CO = 2; ", "constexpr int B3CO = 3; ")],
    # every thread loads its own cells' rhs, as before r05/s46
    "rhsall": [("constexpr bool kB3HaloRhs = false;", "constexpr bool kB3HaloRhs = true;")],
    # the periodic rhs pass writes back only the pairs whose bits change
    # (parity-correct: the values are the same either way)
    "subchg": [("omg_tiles.hip", """        v[r].x = v[r].x - m;
        v[r].y = v[r].y - m;
        if (own[r]) sums_st<kSubNTSt>(src[r] + rc, v[r]);""", """        const double2 o = v[r];
        v[r].x = o.x - m;
        v[r].y = o.y - m;
        const bool chg = __double_as_longlong(v[r].x) != __double_as_longlong(o.x) ||
                         __double_as_longlong(v[r].y) != __double_as_longlong(o.y);
        if (own[r] && chg) sums_st<kSubNTSt>(src[r] + rc, v[r]);""")],
    # 2 / 6 planes of loads in flight instead of 4 (parity-correct)
    "a2": [("constexpr int kB3Ahead = 4;", "constexpr int kB3Ahead = 2;")],
    "a6": [("constexpr int kB3Ahead = 4;", "constexpr int kB3Ahead = 6;")],
    # (column lengths: r05/s38 measured 8 and 2 against 4, s40 16 against 8;
    # the product now takes 16 on levels of >= 32768 boxes; OMG_BLOCK3_COLUMN
    # sets any even length up to kB3MaxZ at run time)
    # the store wave idle (no flush at all) / interior stores only (no ghost pushes)
    "nostw": [("        flush(t + u);\n", "")],
    "nopush": [("        if (k == 1 || k == B3NC) {\n          const bool lf = leftv(jr);", "        if (false) {\n          const bool lf = leftv(jr);"),
               ("      // x faces: per row the cells x = 0, 15, 16, 31 (lane: row l/4, which l%4)\n      {", "      if (false) {"),
               ("      // y faces: the cells of rows j = 1 (lanes 0..31) and j = 16 (32..63)\n      {", "      if (false) {")],
    # subtract_rhs pass (k_box_sums3<SUB>) with non-temporal stores / loads too
    "subnt": [("kSubNTLd = false, kSubNTSt = false", "kSubNTLd = false, kSubNTSt = true")],
    "subntld": [("kSubNTLd = false, kSubNTSt = false", "kSubNTLd = true, kSubNTSt = true")],
    # coarse planes not loaded (the ring gets a register value)
    "noload": [("a = b3_ld(C.phi, o);\n    b = b3_ld(cold, o);", "a = (double)o;\n    b = 0.0;")],
    # no coarse res stores in the store wave
    "nost": [("if (PRO) cflush(t + u);", "")],
    # no coarse loads before the loop (planes -2, -1 stay zero)
    "noprol": [("      cload(-2, a0, b0);\n      cload(-1, a1, b1);", "      a0 = b0 = a1 = b1 = 0.0;")],
    # one coarse load per cell and no res stores (a precomputed res)
    "half_nost": [("a = b3_ld(C.phi, o);\n    b = b3_ld(cold, o);", "a = b3_ld(C.phi, o);\n    b = 0.0;"),
                  ("if (PRO) cflush(t + u);", "")],
    # every store of the pass non-temporal
    # (measured r05/s31: nt 2.4 % faster, now the product's; sc0 sc1 0.8 %)
    # the stores without nt (as before s31)
    "tst": [('"global_store_dwordx2 %0, %1, %2 nt\\n\\ts_nop 1"', '"global_store_dwordx2 %0, %1, %2\\n\\ts_nop 1"')],
    # the phi / rhs loads non-temporal too
    "ntld": [("return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + off);",
              "return __builtin_nontemporal_load(reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + off));")],
    # no correction added (its LDS reads die with it)
    "nocorr": [("ot = ot + (f0 + fx + fy + fz);", "")],
}
names = sys.argv[1:] or list(VARIANTS)
for name in names:
    d = f"/tmp/b3pv/{name}"   # (omg_internal.h includes ../../include/omg.h: /tmp/include)
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs("/tmp/include", exist_ok=True)
    shutil.copy(os.path.join(R, "include", "omg.h"), "/tmp/include/omg.h")
    shutil.copytree(os.path.join(R, "octree-mg_amd", "csrc"), d)
    for rep in VARIANTS[name]:
        f, a, b = rep if len(rep) == 3 else (FILES.get(name, "omg_block.hip"),) + tuple(rep)
        p = os.path.join(d, f)
        s = open(p).read()
        assert a in s, (name, a)
        s = s.replace(a, b)
        open(p, "w").write(s)
    out = os.path.join(R, "octree-mg_amd", "_variants", f"libomg_b3p_{name}.so")
    subprocess.run(["make", "-j8", "-C", d, f"OUT={out}"], check=True, stdout=subprocess.DEVNULL)
    # the include path of omg_api.cpp (../../include/omg.h) resolves from the copy's parent
    print("built", out)
