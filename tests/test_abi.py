"""The C-ABI library builds for gfx950, loads, and exports every symbol that
include/omg.h declares (no compute calls: this runs without a GPU)."""
import ctypes
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "omg.h")
LIB = os.path.join(ROOT, "octree-mg_amd", "libomg.so")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(omg_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared()
    for must in ("omg_ctx_create", "omg_tree_setup", "omg_fas_vcycle", "omg_fas_fmg",
                 "omg_smooth_boxes", "omg_fill_ghost_cells_lvl", "omg_restrict_lvl",
                 "omg_prolong", "omg_update_coarse", "omg_correct_children"):
        assert must in names


def test_library_exports_all_declared_symbols():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "octree-mg_amd", "csrc")], check=True)
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    from tests.mgdriver import omg
    assert set(declared()) == set(omg.device.SIGNATURES)


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", LIB],
                         capture_output=True, text=True)
    # the embedded offload bundle names the target
    data = open(LIB, "rb").read()
    assert b"gfx950" in data


def test_last_error_without_gpu_is_clean():
    from tests.mgdriver import omg
    L = omg.device.lib()
    assert isinstance(L.omg_last_error(), bytes)
