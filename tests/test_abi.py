"""The drop-in boundary: libimpc_qp.so loads on a GPU-less host and exports every function that
include/*.h declares; the Python mirror binds exactly those; the product refuses to run without
a device instead of falling back to any CPU path."""
import ctypes as C
import glob
import os
import re

import pytest

import impc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(impc_\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return names


def test_headers_declare_the_boundary():
    names = declared()
    for must in ("impc_batch_create", "impc_batch_set_values", "impc_batch_warm_start", "impc_batch_solve",
                 "impc_batch_get", "impc_batch_destroy", "impc_mpc_build_values"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(impc.LIB_PATH)
    missing = [n for n in sorted(declared()) if not hasattr(lib, n)]
    assert not missing, missing


def test_python_mirror_binds_every_declared_symbol():
    assert set(impc.EXPORTED) == declared()


def test_struct_layouts_match_headers():
    # impc_settings: 22 8-byte fields (OSQPSettings mirror); impc_info: 8 fields
    assert C.sizeof(impc.Settings) == 22 * 8
    assert C.sizeof(impc.Info) == 8 * 8 and impc.INFO_DTYPE.itemsize == 64
    assert C.sizeof(impc.Stats) == 16 * 8  # 13 facts + the structured team shape (lanes, var / row slots)


def test_default_settings_are_osqp_defaults():
    s = impc.default_settings()
    assert (s.rho, s.sigma, s.scaling, s.max_iter, s.eps_abs, s.eps_rel, s.alpha) == \
        (0.1, 1e-6, 10, 4000, 1e-3, 1e-3, 1.6)
    assert (s.check_termination, s.warm_start, s.polish, s.adaptive_rho_interval) == (25, 1, 0, 0)


def test_version_string():
    assert impc.lib.impc_version().decode().startswith("impc")
    bid = impc.lib.impc_build_id().decode()
    assert bid.startswith("src-") and len(bid) >= 20 and bid != "src-unknown", bid


def test_no_device_fails_loudly():
    """Without a GPU the context cannot be created and the error says why (no CPU fallback)."""
    import torch
    if torch.cuda.device_count() > 0:  # counts without starting torch's own HIP runtime
        pytest.skip("a GPU is present")
    with pytest.raises(impc.ImpcError) as e:
        impc.Context(0)
    assert "impc_ctx_create" in str(e.value)


def test_replan_struct_layouts_match_the_header(tmp_path):
    """impc_replan_config / _inputs / _view: the ctypes mirror's size and field offsets equal the
    C compiler's for include/impc_replan.h (gcc on the header itself)."""
    import shutil
    import subprocess
    from impc.replan import ReplanConfig, ReplanInputs, ReplanView
    if not shutil.which("gcc"):
        pytest.skip("no C compiler")
    structs = (("impc_replan_config", ReplanConfig), ("impc_replan_inputs", ReplanInputs),
               ("impc_replan_view", ReplanView))
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "impc_replan.h"', "int main(void) {"]
    for cname, py in structs:
        lines.append(f'printf("%zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("%zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src, exe = tmp_path / "layout.c", tmp_path / "layout"
    src.write_text("\n".join(lines))
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = []
    for _, py in structs:
        want.append(C.sizeof(py))
        want += [getattr(py, f).offset for f, _ in py._fields_]
    assert got == want
